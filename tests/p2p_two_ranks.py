"""One rank of the direct-peer-exchange tests (tests/test_gpu_dist.py::
test_dist_spmv_p2p_*): WORLD_SIZE ranks share cuda:0, blobs exchanged over
gloo, a local (RCCL-free) communicator each, lhpc_dist_spmv with registered y
windows.  Prints one JSON line.  Test infrastructure.

Cases (argv[1]):
  barrier   three calls per matrix, host barrier + synchronize around each
            call (fp32 XTILE row-range plan, fp64 per-block plans)
  loop      the iterative loop with NO host ordering between calls: x ← y
            copied on the call's stream after every call, so the READY /
            DONE flags are the only ordering between the ranks; four calls
  pingpong  two windows (ya, yb): y of call n is x of call n+1, four calls,
            no host ordering
  tiny      1–3-row blocks (small n, many chunks) in fp32 and fp64, and a
            window whose 16-B phase differs between the ranks (word stores)
  rollback  rank 1's import fails (injected) after both exported: both ranks
            raise and undo the window, an AUTO-exchange call then fails the
            same way on both (no window: RCCL, which a local comm lacks — no
            rank takes the P2P path alone), and a second setup lines the
            windows up again: its P2P calls are bit-exact
  reset     P2P calls, a collective lhpc_dist_p2p_reset (new flag arrays),
            re-export / import (peers' flags remapped by generation), calls
  cg        lhpc_dist_cg_solve over WORLD_SIZE ranks (K = 2, p_work a window,
            dots through the P2P scalar all-gather) equals the world-1 solve
            with K = 2·WORLD_SIZE (the same blocks) bit for bit; P2P all-reduce
            of [r+1, 2r]
  chain     cross-step overlap: five chained lhpc_dist_spmv_begin calls over
            two windows (y of call n is x of call n+1), no end in between —
            each stage's column part waits for the previous call's DONE(j)
  stencil   the 7-point stencil over z-slabs of uneven depth (37 planes over
            WORLD_SIZE ranks, ragged 19 × 23 planes), both ping-pong buffers
            registered windows of different size per rank: six steps of
            lhpc_dist_stencil7_f32_x with the P2P halo (boundary planes stored
            into the neighbours' ghost planes, READY/DONE with the neighbours
            only), no host ordering between steps; each slab equals the
            single-domain lhpc_stencil7_f32 result bit for bit
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import libhpc_amd as L  # noqa: E402
from tests import _support as S  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "barrier"
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
out = {"rank": rank, "case": case, "ok": [], "status": []}


def problem(n, per_row, K, dt, seed):
    rp, col, val = L.gen_uniform_csr(n, n, per_row, dtype=dt, dist=1, seed=seed)
    x = L.gen_values(dt, 1, n, seed + 1)
    cuts = L.interleaved_cuts(rp, world, K)
    return rp, col, val, x, cuts, L.interleaved_local_csr(rp, col, val, cuts, world, K, rank)


def iterate_oracle(rp, col, val, x, steps):
    ys, cur = [], x
    for _ in range(steps):
        _, cur, _ = S.spmv_oracle(rp, col, val, cur)
        ys.append(cur)
    return ys


if case == "barrier":
    for n, per_row, K, dt in ((3_000_000, 6, 2, L.F32), (20_000, 7, 3, L.F64)):
        rp, col, val, x, cuts, local = problem(n, per_row, K, dt, 0xE100 + K)
        _, want, _ = S.spmv_oracle(rp, col, val, x)
        comm = L.DistComm.local(world, rank, 0)
        xd = torch.from_numpy(x).to(dev)
        y = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
        comm.p2p_setup_torch(y)
        with L.DistSpMVPlan(comm, n, n, K, cuts, *local) as d:
            for it in range(3):
                y.fill_(float("nan"))
                torch.cuda.synchronize()
                dist.barrier()  # every rank's y reset before anyone's next pushes (READY covers the stream, not this fill)
                d(xd, y)
                torch.cuda.synchronize()
                out["ok"].append(bool(np.array_equal(y.cpu().numpy(), want)))
                dist.barrier()
        out["status"].append(comm.p2p_status())
        comm.close()
elif case in ("loop", "pingpong"):
    steps = 4
    for n, per_row, K, dt in ((2_000_000, 3, 2, L.F32), (30_000, 3, 3, L.F64)):
        rp, col, val, x, cuts, local = problem(n, per_row, K, dt, 0xE200 + K)
        want = iterate_oracle(rp, col, val, x, steps)
        comm = L.DistComm.local(world, rank, 0)
        s = torch.cuda.current_stream(dev)
        xd = torch.from_numpy(x).to(dev)
        if case == "loop":
            y = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
            comm.p2p_setup_torch(y)
        else:
            ya = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
            yb = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
            comm.p2p_setup_torch(ya)  # two windows, same order on every rank
            comm.p2p_setup_torch(yb)
        torch.cuda.synchronize()
        dist.barrier()  # windows mapped everywhere; from here on no host ordering
        snaps = []
        with L.DistSpMVPlan(comm, n, n, K, cuts, *local, options={"dist_exchange": L.DIST_EXCHANGE_P2P}) as d:
            cur = xd
            for it in range(steps):
                if case == "loop":
                    d(cur, y, stream=s)
                    snaps.append(y.clone())  # on the stream, after the call's DONE wait
                    xd.copy_(y)  # x ← y on the call's stream (reads y before the next READY)
                    cur = xd
                else:
                    dst = ya if it % 2 == 0 else yb
                    d(cur, dst, stream=s)
                    snaps.append(dst.clone())
                    cur = dst
            torch.cuda.synchronize()
        for it in range(steps):
            out["ok"].append(bool(np.array_equal(snaps[it].cpu().numpy(), want[it])))
        dist.barrier()
        out["status"].append(comm.p2p_status())
        comm.close()
elif case == "tiny":
    for n, K, dt, shift in ((41, 16, L.F64, 0), (43, 16, L.F32, 0), (41, 9, L.F32, 1), (37, 5, L.F64, 0)):
        rp, col, val, x, cuts, local = problem(n, 3, K, dt, 0xE300 + n + K)
        _, want, _ = S.spmv_oracle(rp, col, val, x)
        comm = L.DistComm.local(world, rank, 0)
        xd = torch.from_numpy(x).to(dev)
        # shift: rank 1's window starts one element into its buffer, so the
        # two windows differ in 16-B phase and the pushes use word stores
        base = torch.full((n + 4,), float("nan"), dtype=xd.dtype, device=dev)
        off = shift if rank == 1 else 0
        y = base[off:off + n]
        comm.p2p_setup_torch(y)
        torch.cuda.synchronize()
        dist.barrier()
        with L.DistSpMVPlan(comm, n, n, K, cuts, *local, options={"dist_exchange": L.DIST_EXCHANGE_P2P}) as d:
            for it in range(2):
                d(xd, y)
                torch.cuda.synchronize()
                out["ok"].append(bool(np.array_equal(y.cpu().numpy(), want)))
                dist.barrier()
                y.fill_(float("nan"))
                torch.cuda.synchronize()
                dist.barrier()
        out["status"].append(comm.p2p_status())
        comm.close()
elif case == "rollback":
    n, K = 50_000, 2
    rp, col, val, x, cuts, local = problem(n, 5, K, L.F32, 0xE400)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    comm = L.DistComm.local(world, rank, 0)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
    try:
        comm.p2p_setup_torch(y, _fail_import=(rank == 1))
        out["ok"].append(False)  # must raise on every rank
    except L.LhpcError:
        out["ok"].append(True)
    with L.DistSpMVPlan(comm, n, n, K, cuts, *local) as d:  # AUTO exchange
        try:
            d(xd, y)
            torch.cuda.synchronize()
            out["ok"].append(False)  # no window and no RCCL: every rank must refuse
        except L.LhpcError as e:
            out["ok"].append(e.status == -1)
    dist.barrier()
    comm.p2p_setup_torch(y)  # window 0 again, on both ranks
    torch.cuda.synchronize()
    dist.barrier()
    with L.DistSpMVPlan(comm, n, n, K, cuts, *local) as d:
        for it in range(2):
            d(xd, y)
            torch.cuda.synchronize()
            out["ok"].append(bool(np.array_equal(y.cpu().numpy(), want)))
            dist.barrier()
    out["status"].append(comm.p2p_status())
    comm.close()
elif case == "reset":
    n, K = 60_000, 3
    rp, col, val, x, cuts, local = problem(n, 4, K, L.F64, 0xE500)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    comm = L.DistComm.local(world, rank, 0)
    xd = torch.from_numpy(x).to(dev)
    for rnd in range(3):
        y = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
        comm.p2p_setup_torch(y)
        torch.cuda.synchronize()
        dist.barrier()
        with L.DistSpMVPlan(comm, n, n, K, cuts, *local, options={"dist_exchange": L.DIST_EXCHANGE_P2P}) as d:
            for it in range(2):
                d(xd, y)
                torch.cuda.synchronize()
                out["ok"].append(bool(np.array_equal(y.cpu().numpy(), want)))
                dist.barrier()
        out["status"].append(comm.p2p_status())
        comm.p2p_reset()  # collective: every rank, then a barrier before re-export
        dist.barrier()
    comm.close()
elif case == "chain":
    steps = 5
    for n, per_row, K, dt in ((3_000_000, 4, 2, L.F32), (40_000, 3, 3, L.F64)):
        rp, col, val, x, cuts, local = problem(n, per_row, K, dt, 0xE600 + K)
        want = iterate_oracle(rp, col, val, x, steps)
        comm = L.DistComm.local(world, rank, 0)
        s = torch.cuda.current_stream(dev)
        xd = torch.from_numpy(x).to(dev)
        ya = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
        yb = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
        comm.p2p_setup_torch(ya)
        comm.p2p_setup_torch(yb)
        torch.cuda.synchronize()
        dist.barrier()
        snaps = []
        with L.DistSpMVPlan(comm, n, n, K, cuts, *local, options={"dist_exchange": L.DIST_EXCHANGE_P2P}) as d:
            cur = xd
            for it in range(steps):
                dst = ya if it % 2 == 0 else yb
                d.begin(cur, dst, stream=s)
                if it > 0:
                    snaps.append(cur.clone())  # complete once this call's chained stage waited for it
                cur = dst
            d.end(stream=s)
            snaps.append(cur.clone())
            torch.cuda.synchronize()
        for it in range(steps):
            out["ok"].append(bool(np.array_equal(snaps[it].cpu().numpy(), want[it])))
        dist.barrier()
        out["status"].append(comm.p2p_status())
        comm.close()
elif case == "cg":
    ny, nx = 90, 77
    rp, col, val = S.laplacian_2d(ny, nx)
    n = rp.size - 1
    b = torch.from_numpy(np.random.default_rng(0xE700).uniform(-1, 1, n)).to(dev)
    # the one-rank solve of the same four blocks (world-1 local communicator)
    c1 = L.DistComm.local(1, 0, 0)
    K1 = 2 * world  # the same blocks on one rank
    cuts1 = L.interleaved_cuts(rp, 1, K1)
    with L.DistSpMVPlan(c1, n, n, K1, cuts1, *L.interleaved_local_csr(rp, col, val, cuts1, 1, K1, 0)) as d1:
        x1, it1, _ = d1.cg(b, torch.zeros(n, dtype=torch.float64, device=dev), torch.empty(n, dtype=torch.float64,
                                                                                          device=dev), tol=1e-10,
                           max_iter=5000)
        x1 = x1.cpu().numpy()
    c1.close()
    comm = L.DistComm.local(world, rank, 0)
    pw = torch.full((n,), float("nan"), dtype=torch.float64, device=dev)
    comm.p2p_setup_torch(pw)
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([rank + 1.0, 2.0 * rank], dtype=torch.float64, device=dev)
    comm.allreduce_sum_f64(t, stream=torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    out["ok"].append(t.cpu().tolist() == [world * (world + 1) / 2.0, world * (world - 1) * 1.0])
    cuts = L.interleaved_cuts(rp, world, 2)
    assert np.array_equal(cuts, cuts1)
    with L.DistSpMVPlan(comm, n, n, 2, cuts, *L.interleaved_local_csr(rp, col, val, cuts, world, 2, rank)) as d:
        x2, it2, _ = d.cg(b, torch.zeros(n, dtype=torch.float64, device=dev), pw, tol=1e-10, max_iter=5000)
        x2 = x2.cpu().numpy()
    out["ok"].append(it1 == it2)
    out["ok"].append(bool(np.array_equal(x1, x2)))
    dist.barrier()
    out["status"].append(comm.p2p_status())
    comm.close()
elif case == "stencil":
    from libhpc_amd.dist import slab_bounds
    nz, ny, nx, steps = 37, 19, 23, 6
    P = (ny + 2) * (nx + 2)
    rng = np.random.default_rng(0xE800)
    full = np.zeros((nz + 2, ny + 2, nx + 2), dtype=np.float32)
    full[1:-1, 1:-1, 1:-1] = rng.uniform(-1, 1, (nz, ny, nx)).astype(np.float32)
    # the single-domain reference: the same kernel family on the whole grid
    ga, gb = torch.from_numpy(full.ravel().copy()).to(dev), torch.zeros(full.size, dtype=torch.float32, device=dev)
    for _ in range(steps):
        L.stencil7(ga, gb, nz, ny, nx, 1, -6.0, 1.0)
        ga, gb = gb, ga
    torch.cuda.synchronize()
    want = ga.cpu().numpy().reshape(nz + 2, ny + 2, nx + 2)
    z0, z1 = slab_bounds(nz, rank, world)
    nzl = z1 - z0
    comm = L.DistComm.local(world, rank, 0)
    ua = torch.from_numpy(full[z0:z1 + 2].ravel().copy()).to(dev)  # slab + both z ghost planes
    ub = torch.zeros((nzl + 2) * P, dtype=torch.float32, device=dev)
    if rank > 0:
        ua[:P] = float("nan")  # inner ghosts: only the neighbour's stores may fill them
    if rank < world - 1:
        ua[(nzl + 1) * P:] = float("nan")
    comm.p2p_setup_torch(ua)
    comm.p2p_setup_torch(ub)
    torch.cuda.synchronize()
    dist.barrier()
    s = torch.cuda.Stream(dev)
    with torch.cuda.stream(s):
        a, b = ua, ub
        for _ in range(steps):
            comm.stencil7(a, b, nzl, ny, nx, 1, -6.0, 1.0, stream=s, exchange=L.DIST_EXCHANGE_P2P)
            a, b = b, a
    s.synchronize()
    got = a.cpu().numpy().reshape(nzl + 2, ny + 2, nx + 2)[1:-1]
    out["ok"].append(bool(np.array_equal(got, want[z0 + 1:z1 + 1])))
    out["ok"].append(nzl >= 1)
    dist.barrier()
    out["status"].append(comm.p2p_status())
    comm.close()
else:
    raise SystemExit(f"unknown case {case}")
print(json.dumps(out), flush=True)
dist.destroy_process_group()
