"""Per-rank local SpMV time of bench.py's N>1 decomposition, simulated on one
GPU: rank 0's K interleaved-chunk plans for world W (no collective)."""
import json
import os
import sys
import time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L
from libhpc_amd.dist import InterleavedBlocks

dev = torch.device("cuda:0")
n = 10_000_000
rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=L.F32)
x = torch.from_numpy(L.gen_values(L.F32, 0, n, L.SEED_X)).to(dev)
t1 = None  # W = 1 time: the ideal at W is t1 / W
for W, K in ((1, 1), (2, 1), (2, 2), (2, 4), (4, 1), (4, 2), (4, 4), (8, 1), (8, 2), (8, 4)):
    ib = InterleavedBlocks(n, W, K)
    plans = [L.SpMVPlan(*ib.local_csr(rp, col, val, 0, k), n) for k in range(K)]
    ys = [torch.empty(ib.B, device=dev) for _ in range(K)]
    for _ in range(3):
        for p, y in zip(plans, ys):
            p(x, y)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        for p, y in zip(plans, ys):
            p(x, y)
    e1.record(); torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20
    t1 = t if t1 is None else t1
    print(json.dumps(dict(W=W, K=K, ms=t, ideal_ms=t1 / W, eff=t1 / W / t, kernel=plans[0].info()["kernel"],
                          slices=plans[0].info()["slices"])), flush=True)
    for p in plans:
        p.close()
