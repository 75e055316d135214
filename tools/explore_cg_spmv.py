"""SpMV kernel choice for the CG Laplacian (fp64, 5 nnz/row): ROWGROUP L,R variants vs ADAPTIVE."""
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L

dev = torch.device("cuda:0")
rp, col, val = L.gen_laplacian_2d(4096, 4096, L.F64)
n = rp.size - 1
x = torch.rand(n, dtype=torch.float64, device=dev)
y = torch.empty_like(x)
ref = None
for name, flags, env in (("auto", 0, None), ("rg1,1", 1 << 4, "1,1"), ("rg2,1", 1 << 4, "2,1"), ("rg2,2", 1 << 4, "2,2"),
                         ("rg4,1", 1 << 4, "4,1"), ("rg4,2", 1 << 4, "4,2"), ("rg4,4", 1 << 4, "4,4"),
                         ("rg8,2", 1 << 4, "8,2"), ("rg8,4", 1 << 4, "8,4"), ("adaptive", 1 << 5, None)):
    if env:
        os.environ["LHPC_SPMV_ROWGROUP"] = env
    else:
        os.environ.pop("LHPC_SPMV_ROWGROUP", None)
    with L.SpMVPlan(rp, col, val, n, flags=flags) as pl:
        for _ in range(3):
            pl(x, y)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            pl(x, y)
        e1.record(); torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 20 * 1e-3
        if ref is None:
            ref = y.clone()
        alg = col.size * 12 + (n + 1) * 4 + 2 * n * 8
        print(json.dumps(dict(k=name, us=t * 1e6, TBps=alg / t / 1e12, info=pl.info()["kernel"],
                              maxdiff=float((y - ref).abs().max()))), flush=True)
