"""C5 multi-rank stencil on CPU (gloo): z-slab split + halo exchange must give
exactly the single-domain oracle result (z-slab decomposition with
1-plane halos)."""
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


def _worker(rank, world, port, nz, ny, nx, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from libhpc_amd.dist import DistStencil7, slab_bounds
        from tests import _support as S
        full = S.random_padded((nz + 2, ny + 2, nx + 2), seed=0xC5, zero_ghost=True, ghost=1)
        want = S.stencil7_oracle(full.reshape(-1), nz, ny, nx, 1, -6.0, 1.0).reshape(full.shape)
        z0, z1 = slab_bounds(nz, rank, world)
        nzl = z1 - z0
        # local slab with its own ghost planes; interior halos start as garbage
        loc = np.full((nzl + 2, ny + 2, nx + 2), np.nan, dtype=np.float32)
        loc[1:-1] = full[z0 + 1:z1 + 1]
        if rank == 0:
            loc[0] = full[0]
        if rank == world - 1:
            loc[-1] = full[-1]
        u = torch.from_numpy(loc.reshape(-1).copy())
        out = torch.zeros_like(u)

        def compute(ut, ot, zb, ze):  # oracle on planes [zb, ze) of the slab (CPU test only)
            if ze <= zb:
                return
            a = ut.numpy().reshape(nzl + 2, ny + 2, nx + 2)
            sub = np.ascontiguousarray(a[zb:ze + 2])
            res = S.stencil7_oracle(sub.reshape(-1), ze - zb, ny, nx, 1, -6.0, 1.0).reshape(sub.shape)
            ot.numpy().reshape(nzl + 2, ny + 2, nx + 2)[zb + 1:ze + 1] = res[1:-1]

        DistStencil7(nzl, ny, nx, rank, world, compute).step(u, out)
        got = out.numpy().reshape(nzl + 2, ny + 2, nx + 2)[1:-1, 1:-1, 1:-1]
        ok = np.array_equal(got, want[z0 + 1:z1 + 1, 1:-1, 1:-1])
        dist.destroy_process_group()
        q.put((rank, ok))
    except Exception as e:
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world,nz", [(2, 16), (3, 17), (4, 9)])
def test_halo_exchange_matches_single_domain(world, nz):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, nz, 12, 20, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for rank, ok in res:
        assert ok is True, f"rank {rank}: {ok}"


def test_slab_bounds_cover():
    from libhpc_amd.dist import slab_bounds
    for nz in (1, 7, 512):
        for w in (1, 2, 3, 8):
            spans = [slab_bounds(nz, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == nz
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
