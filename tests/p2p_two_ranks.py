"""One rank of the direct-peer-exchange test (tests/test_gpu_dist.py::
test_dist_spmv_p2p_two_ranks_one_gpu): WORLD_SIZE ranks share cuda:0, blobs
exchanged over gloo, a local (RCCL-free) communicator each, lhpc_dist_spmv
with the registered y window.  Prints one JSON line.  Test infrastructure."""
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

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
out = {"rank": rank, "ok": []}
for n, per_row, K, dt in ((3_000_000, 6, 2, L.F32), (20_000, 7, 3, L.F64)):
    rp, col, val = L.gen_uniform_csr(n, n, per_row, dtype=dt, dist=1, seed=0xE100 + K)
    x = L.gen_values(dt, 1, n, 0xE101)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    cuts = L.interleaved_cuts(rp, world, K)
    lrp, lc, lv = L.interleaved_local_csr(rp, col, val, cuts, world, K, rank)
    comm = L.DistComm.local(world, rank, 0)
    xd = torch.from_numpy(x).to(dev)
    y = torch.full((n,), float("nan"), dtype=xd.dtype, device=dev)
    comm.p2p_setup_torch(y)
    with L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv) as d:
        for it in range(3):
            y.fill_(float("nan"))
            torch.cuda.synchronize()
            dist.barrier()  # every rank's y reset before anyone's next pushes (READY covers the stream, not this fill)
            d(xd, y)
            torch.cuda.synchronize()
            good = bool(np.array_equal(y.cpu().numpy(), want))
            out["ok"].append(good)
            dist.barrier()
    out.setdefault("status", []).append(comm.p2p_status())
    comm.close()
print(json.dumps(out), flush=True)
dist.destroy_process_group()
