"""The native multi-GPU layer behind the C ABI (include/lhpc.h lhpc_dist_*:
one RCCL communicator and comm stream per process) on the GPU box's single
GPU, world 1: the communicator, the fp64 all-reduce, the distributed SpMV
(stage, per-chunk reduce into y, broadcast schedule, event ordering) through
both of its local-plan forms, and the halo stencil.  RCCL cannot put two
ranks on one GPU; the multi-rank data layout and broadcast schedule are
checked on the CPU (tests/test_dist.py::test_native_dist_partition_identity)."""
import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(lhpc, gpu):
    c = lhpc.DistComm(lhpc.dist_unique_id(), 1, 0, 0)
    yield c
    c.close()


def test_comm_world1_allreduce(lhpc, gpu, comm):
    import torch
    assert comm.nranks == 1 and comm.rank == 0
    t = torch.arange(1000, dtype=torch.float64, device=gpu)
    comm.allreduce_sum_f64(t, stream=torch.cuda.current_stream(gpu))
    torch.cuda.synchronize()
    assert torch.equal(t.cpu(), torch.arange(1000, dtype=torch.float64))


def test_unique_ids_differ(lhpc, gpu):
    assert lhpc.dist_unique_id() != lhpc.dist_unique_id()


@pytest.mark.parametrize("n,per_row,K", [(3_000_000, 6, 1), (3_000_000, 6, 2), (3_000_000, 6, 3),
                                         (20_000, 7, 2), (20_000, 7, 4)])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("range_gather", [False, True])
def test_dist_spmv_world1_matches_single_plan(lhpc, gpu, comm, n, per_row, K, dtype, range_gather):
    """lhpc_dist_spmv at world 1 with K chunks equals the single-plan SpMV bit
    for bit on dyadic values (XTILE row-range plan for the 3M-column matrix,
    one plan per block for the small one), twice in a row, y != x.
    range_gather: the row-range plan gets per-range gather pieces (as a plan
    whose xg exceeds the Infinity Cache does) and each chunk's range is
    gathered right before its reduce instead of one stage — into one
    range-sized xg ring (the local plans' default, options.xtile_ring = 2),
    or with one slot per entry (xtile_ring = 1): same y, less device memory."""
    import torch
    dt = lhpc.F32 if dtype == "f32" else lhpc.F64
    rp, col, val = lhpc.gen_uniform_csr(n, n, per_row, dtype=dt, dist=1, seed=0xD200 + K)
    x = lhpc.gen_values(dt, 1, n, 0xD201)
    xd = torch.from_numpy(x).to(gpu)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    cuts = lhpc.interleaved_cuts(rp, 1, K)
    lrp, lc, lv = lhpc.interleaved_local_csr(rp, col, val, cuts, 1, K, 0)
    infos = []
    for ring in ((0, 1) if range_gather else (0,)):
        opts = {"xtile_ranges": 2, "xtile_ring": ring} if range_gather else None
        with lhpc.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv, options=opts) as d:
            infos.append(d.local_info())
            for _ in range(2):
                y = torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu)
                d(xd, y)
                torch.cuda.synchronize()
                assert np.array_equal(y.cpu().numpy(), want), ring
    if range_gather and K > 1 and infos[0]["kernel"] == lhpc.KERNEL_XTILE:
        # the ring holds the largest range's xg instead of every entry's
        nnz = int(lc.size)
        assert infos[0]["device_bytes"] < infos[1]["device_bytes"] - 0.3 * nnz * val.itemsize, infos


@pytest.mark.parametrize("mode", ["allgather", "broadcast"])
@pytest.mark.parametrize("uniform", [True, False])
def test_dist_spmv_world1_rccl_exchange(lhpc, gpu, comm, mode, uniform):
    """The RCCL y exchange driven at world 1 (options.dist_world1: the
    in-place collective is a no-op there, so y must come out unchanged):
    equal-size blocks go through one in-place ncclAllGather per chunk,
    unequal ones (power-law rows) or options.dist_broadcast through the
    broadcast group; three calls, K = 3; then the exchange alone
    (lhpc_dist_exchange) leaves y as it is."""
    import torch
    opts = {"dist_world1": 1, "dist_broadcast": 1 if mode == "broadcast" else 0}
    n, K = 600_000, 3
    if uniform:
        rp, col, val = lhpc.gen_uniform_csr(n, n, 6, dtype=lhpc.F32, dist=1, seed=0xD300)
    else:
        rp, col, val = lhpc.gen_powerlaw_csr(n, n, dtype=lhpc.F32, dist=1, seed=0xD301)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0xD302)
    xd = torch.from_numpy(x).to(gpu)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    cuts = lhpc.interleaved_cuts(rp, 1, K)
    with lhpc.DistSpMVPlan(comm, n, n, K, cuts, *lhpc.interleaved_local_csr(rp, col, val, cuts, 1, K, 0),
                           options=opts) as d:
        for _ in range(3):
            y = torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu)
            d(xd, y)
            torch.cuda.synchronize()
            assert np.array_equal(y.cpu().numpy(), want)
        d.exchange(y)
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), want)


@pytest.mark.parametrize("K", [1, 2, 3, 4])
@pytest.mark.parametrize("case", [(3_000_000, 6, "f32"), (2_500_000, 5, "f64"), (20_000, 7, "f64")],
                         ids=["xtile-f32", "xtile-f64", "blocks-f64"])
@pytest.mark.parametrize("streams", [1, 2])
def test_dist_spmv_chained_world1(lhpc, gpu, comm, K, case, streams):
    """Cross-step overlap (lhpc_dist_spmv_begin / _end) at world 1 with the
    RCCL exchange issued (options.dist_world1): five chained calls, y of call
    n is x of call n+1 (ping-pong), no end between them — each chained stage
    gathers x by column parts, part j waiting only for exchange j of the call
    before (XTILE row-range plans; the per-block plans of the small matrix
    wait for the whole exchange instead).  Every iterate equals the oracle's
    bit for bit (dyadic values; snapshots of y(n) taken on the stream after
    the chained stage of call n+1 has waited for it).  streams: the chunk
    reduces on the caller's stream only, or alternating with a second one
    (options.dist_reduce_streams, default 2)."""
    import torch
    n, per_row, dts = case
    dt = lhpc.F32 if dts == "f32" else lhpc.F64
    rp, col, val = lhpc.gen_uniform_csr(n, n, per_row, dtype=dt, dist=1, seed=0xD400 + K)
    x = lhpc.gen_values(dt, 1, n, 0xD401)
    steps = 5
    want, cur = [], x
    for _ in range(steps):
        _, cur, _ = S.spmv_oracle(rp, col, val, cur)
        want.append(cur)
    cuts = lhpc.interleaved_cuts(rp, 1, K)
    s = torch.cuda.current_stream(gpu)
    with lhpc.DistSpMVPlan(comm, n, n, K, cuts, *lhpc.interleaved_local_csr(rp, col, val, cuts, 1, K, 0),
                           options={"dist_world1": 1, "dist_reduce_streams": streams}) as d:
        bufs = [torch.from_numpy(x).to(gpu), torch.full((n,), float("nan"), dtype=torch.float32 if dts == "f32"
                                                        else torch.float64, device=gpu)]
        bufs.append(torch.full_like(bufs[1], float("nan")))
        snaps = []
        cur_x = bufs[0]
        for it in range(steps):
            y = bufs[1 + it % 2]
            d.begin(cur_x, y, stream=s)
            if it > 0:
                snaps.append(cur_x.clone())  # y of call it-1: complete once call it's stage waited for it
            cur_x = y
        d.end(stream=s)
        snaps.append(cur_x.clone())
        torch.cuda.synchronize()
    for it in range(steps):
        assert np.array_equal(snaps[it].cpu().numpy(), want[it]), it


@pytest.mark.parametrize("K", [1, 2, 4])
@pytest.mark.parametrize("dtype", ["f64", "f32"])
def test_dist_cg_world1(lhpc, gpu, comm, K, dtype):
    """lhpc_dist_cg_solve at world 1 (RCCL communicator, K blocks of rows,
    block-order dots, chained stages) on the 2-D Laplacian: fp64 — the fp64
    CG restatement's iteration count ±1 and x within 1e-8·‖x‖; fp32 —
    converged and within 1e-4·‖x‖ of the fp64 solution."""
    import torch
    ny, nx = 80, 70
    dt = np.float64 if dtype == "f64" else np.float32
    rp, col, val = S.laplacian_2d(ny, nx, dtype=dt, shift=0.0 if dtype == "f64" else 0.5)
    n = rp.size - 1
    b = np.random.default_rng(0xD500 + K).uniform(-1, 1, n)
    want, it_o, _ = S.cg_oracle(rp, col, val.astype(np.float64), b, tol=1e-10, max_iter=5000)
    cuts = lhpc.interleaved_cuts(rp, 1, K)
    tol = 1e-10 if dtype == "f64" else 1e-5
    with lhpc.DistSpMVPlan(comm, n, n, K, cuts, *lhpc.interleaved_local_csr(rp, col, val, cuts, 1, K, 0)) as d:
        bd = torch.from_numpy(b.astype(dt)).to(gpu)
        x = torch.zeros(n, dtype=bd.dtype, device=gpu)
        p = torch.empty_like(x)
        x, it, res = d.cg(bd, x, p, tol=tol, max_iter=5000, check_every=2)
        x = x.cpu().numpy().astype(np.float64)
    assert res <= tol
    if dtype == "f64":
        assert abs(it - it_o) <= 2  # checked every 2nd iteration
        assert np.linalg.norm(x - want) <= 1e-8 * np.linalg.norm(want)
    else:
        assert np.linalg.norm(x - want) <= 1e-4 * np.linalg.norm(want)


def test_dist_spmv_rejects_aliased_xy(lhpc, gpu, comm):
    import torch
    n = 1000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 5, dtype=lhpc.F32, dist=1)
    cuts = lhpc.interleaved_cuts(rp, 1, 2)
    with lhpc.DistSpMVPlan(comm, n, n, 2, cuts, *lhpc.interleaved_local_csr(rp, col, val, cuts, 1, 2, 0)) as d:
        xd = torch.ones(n, device=gpu)
        with pytest.raises(lhpc.LhpcError):
            d(xd, xd)


@pytest.mark.parametrize("nz,ny,nx", [(37, 45, 1100), (9, 19, 512), (1, 5, 7), (2, 3, 1024)])
def test_dist_stencil7_world1_matches_single_domain(lhpc, gpu, comm, nz, ny, nx):
    """lhpc_dist_stencil7_f32 at world 1 (no neighbours: outer ghost planes
    kept) is bit-identical to lhpc_stencil7_f32 on the same slab."""
    import torch
    shape = (nz + 2, ny + 2, nx + 2)
    u = S.random_padded(shape, seed=nz * 13 + nx, zero_ghost=False).reshape(-1)
    out0 = S.random_padded(shape, seed=77).reshape(-1)
    want = S.stencil7_oracle(u, nz, ny, nx, 1, -6.0, 1.0, out=out0.copy())
    ud = torch.from_numpy(u).to(gpu)
    od = torch.from_numpy(out0.copy()).to(gpu)
    comm.stencil7(ud, od, nz, ny, nx, 1, -6.0, 1.0)
    assert np.array_equal(od.cpu().numpy(), want)


P2P_CASES = {"barrier": 6, "loop": 8, "pingpong": 8, "tiny": 8, "rollback": 4, "reset": 6, "chain": 10, "cg": 3,
             "stencil": 2, "stencil/3": 2, "pingpong/3": 8, "chain/3": 10, "cg/3": 3}


@pytest.mark.parametrize("case", list(P2P_CASES))
def test_dist_spmv_p2p_two_ranks_one_gpu(lhpc, gpu, case):
    """The direct peer exchange (lhpc_dist_p2p_export/_import, READY/DONE
    flags, push kernel) with two processes on the box's one GPU: IPC-mapped
    windows, RCCL-free local communicators, blobs over gloo; every rank's
    assembled y equals the oracle bit for bit (dyadic).  Cases
    (tests/p2p_two_ranks.py): host-barriered calls (fp32 XTILE row-range and
    fp64 per-block plans); the iterative loop x ← y with no host ordering
    between calls (the flags are the only ordering); two windows ping-ponged
    (y of call n is x of call n+1); 1–3-row blocks and windows of different
    16-B phase; a setup whose import fails on one rank rolled back on both
    (then an AUTO call refused on both, and a fresh setup bit-exact); three
    rounds of setup / calls / collective reset (flag arrays re-allocated and
    remapped by generation); chained calls (lhpc_dist_spmv_begin: the
    stage's column part j waits for the previous call's per-chunk DONE(j)
    flags, ping-pong windows, five calls, one end); the distributed CG
    (lhpc_dist_cg_solve, p_work a window, dots all-gathered through the P2P
    scalar slots) at world 2 × K 2 bit-identical to a world-1 × K 4 solve of
    the same block split, and the P2P all-reduce; ping-pong, chained calls
    and the CG again with three ranks (two peers per rank); the stencil's
    P2P halo over two and three ranks (slabs of different depth, so the middle rank
    has both neighbours), six ping-pong steps bit-identical to the single
    domain.  (On one GPU the pushes are device-local; over xGMI they are the
    same stores.)"""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    port = str(29631 + list(P2P_CASES).index(case))
    name, _, w = case.partition("/")
    world = int(w or 2)
    env = dict(os.environ, WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
    procs = [subprocess.Popen([sys.executable, os.path.join(root, "tests", "p2p_two_ranks.py"), name],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0"), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=240)
            assert p.returncode == 0, e[-3000:]
            outs.append(json.loads(o.strip().splitlines()[-1]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for o in outs:
        assert all(o["ok"]) and len(o["ok"]) == P2P_CASES[case], o
        assert all(s == 0 for s in o["status"]), o
