"""Host issue cost of one lhpc_dist_spmv step (RCCL exchange issued at world
1, K chunks per rank): with a tiny matrix the GPU work is a few µs, so the
host time per call of a long unsynchronised run of chained begins is what
the API calls and launches cost the CPU.  At W = 8 a C2 step is ≈ 100 µs on
the model; if the host needs about as long to issue it, the step is
host-bound.  One JSON line per (n, K): host µs per call (issue only, no
sync), wall µs per call including the final synchronise, and the GPU
timeline per call from events on the stream."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
comm = L.DistComm(L.dist_unique_id(), 1, 0, 0)
stream = torch.cuda.current_stream()
for n in (200_000, 2_000_000):
    rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=L.F32)
    x = torch.from_numpy(L.gen_values(L.F32, 0, n, L.SEED_X)).to(dev)
    for K in (1, 2, 4):
        cuts = L.interleaved_cuts(rp, 1, K)
        lrp, lc, lv = L.interleaved_local_csr(rp, col, val, cuts, 1, K, 0)
        for mode in ("rccl", "none"):
            opts = {"dist_exchange": L.DIST_EXCHANGE_RCCL if mode == "rccl" else L.DIST_EXCHANGE_NONE,
                    "dist_world1": 1}
            with L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv, options=opts) as d:
                ya, yb = torch.empty_like(x), torch.empty_like(x)
                ya.copy_(x)
                bufs = [ya, yb]
                for i in range(20):
                    d.begin(bufs[i & 1], bufs[(i & 1) ^ 1], stream=stream)
                d.end(stream=stream)
                torch.cuda.synchronize()
                reps = 400
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                t0 = time.perf_counter()
                for i in range(reps):
                    d.begin(bufs[i & 1], bufs[(i & 1) ^ 1], stream=stream)
                t1 = time.perf_counter()
                d.end(stream=stream)
                e1.record()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                print(json.dumps({"n": n, "K": K, "exchange": mode, "host_issue_us": (t1 - t0) / reps * 1e6,
                                  "wall_us": (t2 - t0) / reps * 1e6,
                                  "gpu_us": e0.elapsed_time(e1) / reps * 1e3}), flush=True)
comm.close()
