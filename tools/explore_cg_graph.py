"""Same-box A/B of the CG iteration issue paths on the bench's 4096² fp64
Laplacian (bench.py --workload cg): lhpc_cg_solve as a plain loop (null
stream), lhpc_cg_solve replaying 10-iteration HIP graph blocks (non-null
stream), and the Python building-block solver (libhpc_amd.dist.DistCG with
HipOps, the round-3 bench path).  50 iterations per solve, tol 0; µs per
iteration, best of 5, and whether the two native paths agree bit for bit."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402
from libhpc_amd.dist import DistCG, HipOps, InterleavedBlocks  # noqa: E402

dev = torch.device("cuda:0")
nx = int(os.environ.get("NX", "4096"))
rp, col, val = L.gen_laplacian_2d(nx, nx, L.F64)
n = nx * nx
b = torch.from_numpy(L.gen_values(L.F64, 0, n, L.SEED_X)).to(dev)
ITERS, REPS = 50, 5
plan = L.SpMVPlan(rp, col, val, n)
s = torch.cuda.Stream(dev)


def native(stream):
    x = torch.zeros(n, dtype=torch.float64, device=dev)
    with torch.cuda.stream(stream):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        L.cg(plan, b, x, tol=0.0, max_iter=ITERS, check_every=10, stream=stream)
        stream.synchronize()
        return (time.perf_counter() - t0) / ITERS, x


ib = InterleavedBlocks(n, 1, 1)
solver = DistCG(ib, 0, lambda pf, qb: plan(pf, qb), HipOps(None), like=b,
                local_spmv_dot=lambda pf, qb, wb, out: L.spmv_dot(plan, pf, qb, wb, out))


def blocks():
    x = torch.zeros_like(b)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    solver.solve(b, x, tol=0.0, max_iter=ITERS, check_every=ITERS)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / ITERS, x


out = {}
for name, fn in (("loop", lambda: native(torch.cuda.default_stream(dev))), ("graph", lambda: native(s)),
                 ("blocks", blocks)):
    fn()
    ts, xs = [], None
    for _ in range(REPS):
        t, xs = fn()
        ts.append(t)
    out[name] = {"us_per_iter": min(ts) * 1e6, "all_us": [t * 1e6 for t in ts]}
    out[name]["x"] = xs
same = torch.equal(out["loop"].pop("x"), out["graph"].pop("x"))
out["blocks"].pop("x")
print(json.dumps({"n": n, "iters": ITERS, "graph_equals_loop": same, **out}), flush=True)
