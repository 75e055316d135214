"""Distributed CG (libhpc_amd.dist.DistCG) on CPU with gloo, world 2 and 3:
the same control flow bench/GPU runs use (RCCL all-reduce of the dots, all-gather
of p), with the oracle SpMV as the local product and torch CPU vector ops.
Pinned to the fp64 CG restatement (oracle.c): iterations ±1, solution within
1e-8 relative."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from libhpc_amd.dist import DistCG, InterleavedBlocks, TorchCPUOps
        from tests import _support as S
        rp, col, val = S.laplacian_2d(41, 29)
        n = rp.size - 1
        b = np.random.default_rng(5).uniform(-1, 1, n)
        ib = InterleavedBlocks(n, world, 1)
        lrp, lc, lv = ib.local_csr(rp, col, val, rank, 0)
        r0, r1 = ib.rows(rank, 0)

        def local(p_full, q_blk):  # oracle as the local product (CPU test only)
            _, y, _ = S.spmv_oracle(lrp, lc, lv, p_full.numpy())
            q_blk.copy_(torch.from_numpy(y))

        bl = torch.zeros(ib.B, dtype=torch.float64)
        bl[:r1 - r0] = torch.from_numpy(b[r0:r1])
        x = torch.zeros(ib.B, dtype=torch.float64)
        solver = DistCG(ib, rank, local, TorchCPUOps(), like=bl)
        x, it, res = solver.solve(bl, x, tol=1e-10, max_iter=2000)
        want, it_o, _ = S.cg_oracle(rp, col, val, b, tol=1e-10, max_iter=2000)
        err = np.linalg.norm(x[:r1 - r0].numpy() - want[r0:r1])
        dist.destroy_process_group()
        q.put((rank, it, it_o, res, err, float(np.linalg.norm(want))))
    except Exception as e:  # report, never hang the parent
        q.put((rank, repr(e), 0, 0, 0, 0))


@pytest.mark.parametrize("world", [2, 3])
def test_dist_cg_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for rank, it, it_o, r, err, norm in res:
        assert isinstance(it, int), f"rank {rank}: {it}"
        assert abs(it - it_o) <= 1 and r <= 1e-10
    total_err = np.sqrt(sum(e ** 2 for *_, e, _ in res))
    assert total_err <= 1e-8 * res[0][5]


def _native_cg_emulation(rp, col, val, b, world, K, tol=1e-10, max_iter=2000):
    """The schedule of lhpc_dist_cg_solve, rank by rank on the CPU: rank r owns
    blocks k·world + r of the interleaved nnz-balanced cuts, keeps full-length
    b / x / p, computes q on its rows (oracle rows), the dots as one partial per
    block added in GLOBAL block order (what the all-gather + k_sum_blocks do),
    the r and x/p updates on its rows, then p's blocks travel to every rank by
    the native exchange schedule (lhpc_dist_exchange_schedule, P2P pushes)."""
    import libhpc_amd as L
    from tests import _support as S
    n = rp.size - 1
    cuts = L.interleaved_cuts(rp, world, K)
    own = [[(int(cuts[k * world + r]), int(cuts[k * world + r + 1])) for k in range(K)] for r in range(world)]
    blk = [(int(cuts[i]), int(cuts[i + 1])) for i in range(world * K)]
    xs = [np.zeros(n) for _ in range(world)]
    ps = [np.zeros(n) for _ in range(world)]
    rs = [np.zeros(n) for _ in range(world)]

    def dot_blocks(a_of, b_of):  # partial per global block, summed in block order
        parts = []
        for i, (a0, a1) in enumerate(blk):
            r = i % world
            parts.append(float(np.dot(a_of(r)[a0:a1], b_of(r)[a0:a1])))
        acc = 0.0
        for v in parts:
            acc += v
        return acc

    scheds = [L.dist_exchange_schedule(cuts, world, K, r, L.DIST_EXCHANGE_P2P) for r in range(world)]

    def exchange(vs):  # every rank pushes its blocks into every peer's copy
        for r in range(world):
            for e in scheds[r]:
                o0, o1 = e["offset"], e["offset"] + e["count"]
                for q in range(world):
                    if q != r:
                        vs[q][o0:o1] = vs[r][o0:o1]

    bb = dot_blocks(lambda r: b, lambda r: b)
    qs = []
    for r in range(world):
        _, q, _ = S.spmv_oracle(rp, col, val, xs[r])
        for a0, a1 in own[r]:
            rs[r][a0:a1] = b[a0:a1] - q[a0:a1]
            ps[r][a0:a1] = rs[r][a0:a1]
    exchange(ps)
    rr = dot_blocks(lambda r: rs[r], lambda r: rs[r])
    it = 0
    while it < max_iter and rr > tol * tol * bb:
        it += 1
        qs = [S.spmv_oracle(rp, col, val, ps[r])[1] for r in range(world)]
        pq = dot_blocks(lambda r: ps[r], lambda r: qs[r])
        alpha = rr / pq
        for r in range(world):
            for a0, a1 in own[r]:
                rs[r][a0:a1] -= alpha * qs[r][a0:a1]
        rr_new = dot_blocks(lambda r: rs[r], lambda r: rs[r])
        beta = rr_new / rr
        for r in range(world):
            for a0, a1 in own[r]:
                xs[r][a0:a1] += alpha * ps[r][a0:a1]
                ps[r][a0:a1] = rs[r][a0:a1] + beta * ps[r][a0:a1]
        exchange(ps)
        rr = rr_new
    exchange(xs)
    return xs, it


@pytest.mark.parametrize("world,K", [(2, 2), (4, 1), (3, 2)])
def test_native_dist_cg_schedule(world, K):
    """The native distributed CG's schedule on the CPU (see
    _native_cg_emulation): every rank ends with the same whole x, within 1e-8
    of the fp64 CG restatement with the iteration count ±1, and — because the
    dots add block partials in global block order — bit-identical to the
    one-rank run over the same world·K blocks (the property the GPU test
    tests/p2p_two_ranks.py `cg` checks on the device)."""
    from tests import _support as S
    rp, col, val = S.laplacian_2d(37, 23)
    b = np.random.default_rng(11).uniform(-1, 1, rp.size - 1)
    xs, it = _native_cg_emulation(rp, col, val, b, world, K)
    x1, it1 = _native_cg_emulation(rp, col, val, b, 1, world * K)
    want, it_o, _ = S.cg_oracle(rp, col, val, b, tol=1e-10, max_iter=2000)
    for x in xs:
        assert np.array_equal(x, xs[0]) and np.array_equal(x, x1[0])
    assert it == it1 and abs(it - it_o) <= 1
    assert np.linalg.norm(xs[0] - want) <= 1e-8 * np.linalg.norm(want)
