"""ROWGROUP (default L,R) vs ADAPTIVE across short-row shapes that stay off XSLICE."""
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L

dev = torch.device("cuda:0")


def bench(rp, col, val, n_cols, flags):
    x = torch.rand(n_cols, dtype=torch.float64 if val.dtype.itemsize == 8 else torch.float32, device=dev)
    with L.SpMVPlan(rp, col, val, n_cols, flags=flags) as pl:
        y = pl(x)
        for _ in range(3):
            pl(x, y)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            pl(x, y)
        e1.record(); torch.cuda.synchronize()
        return e0.elapsed_time(e1) / 20 * 1e3, pl.info()


cases = []
for per in (3, 5, 8, 10, 15, 24, 40):
    cases.append((f"uniform n=1M per={per} f32", L.gen_uniform_csr(1_000_000, 1_000_000, per, dtype=L.F32), 1_000_000))
cases.append(("uniform n=100k per=10 f64 (C1)", L.gen_uniform_csr(100_000, 100_000, 10, dtype=L.F64), 100_000))
cases.append(("powerlaw n=1M f32", L.gen_powerlaw_csr(1_000_000, 1_000_000, lmax=2000, dtype=L.F32), 1_000_000))
rp, col, val = L.gen_laplacian_2d(2048, 2048, L.F32)
cases.append(("laplacian 2048^2 f32", (rp, col, val), 2048 * 2048))
rp, col, val = L.gen_laplacian_2d(4096, 4096, L.F64)
cases.append(("laplacian 4096^2 f64", (rp, col, val), 4096 * 4096))
for name, (rp, col, val), nc in cases:
    ta, ia = bench(rp, col, val, nc, 0)
    tr, ir = bench(rp, col, val, nc, 1 << 4)
    td, idd = bench(rp, col, val, nc, 1 << 5)
    print(json.dumps(dict(case=name, auto_us=ta, auto_kernel=ia["kernel"], auto_L=ia["lanes_per_row"],
                          rowgroup_us=tr, adaptive_us=td)), flush=True)
