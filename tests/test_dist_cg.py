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
