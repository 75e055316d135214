"""XTILE call time vs the number of x tiles: n = 10M rows, 15 uniform columns
per row, n_cols from one tile (contiguous xg segments) to C2's 245 tiles.
Run under rocprofv3 --kernel-trace --stats for the gather/reduce split."""
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L

dev = torch.device("cuda:0")
n = 10_000_000
for n_cols in [int(a) for a in (sys.argv[1:] or ["40960", "409600", "2457600", "10000000"])]:
    rp, col, val = L.gen_uniform_csr(n, n_cols, 15, dtype=L.F32)
    x = torch.from_numpy(L.gen_values(L.F32, 0, n_cols, L.SEED_X)).to(dev)
    y = torch.empty(n, device=dev)
    with L.SpMVPlan(rp, col, val, n_cols, flags=L.PLAN_FORCE_XTILE) as p:
        for _ in range(3):
            p(x, y)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            p(x, y)
        e1.record(); torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 10
        print(json.dumps(dict(n_cols=n_cols, tiles=p.info()["slices"], ms=t, gflops=2 * col.shape[0] / t / 1e6)), flush=True)
