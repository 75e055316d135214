"""Per-rank local SpMV time of bench.py's N>1 decomposition, simulated on one
GPU: rank 0's K interleaved chunks for world W (no collective), as K chunk
plans ("plans") and as one row-range plan staged once ("split")."""
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L
from libhpc_amd.dist import InterleavedBlocks

dev = torch.device("cuda:0")
n = 10_000_000
rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=L.F32)
x = torch.from_numpy(L.gen_values(L.F32, 0, n, L.SEED_X)).to(dev)


def timed(step):
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        step()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 20


t1 = None  # W = 1 time: the ideal at W is t1 / W
for W, K in ((1, 1), (2, 1), (2, 2), (2, 4), (4, 1), (4, 2), (4, 4), (8, 1), (8, 2), (8, 4)):
    ib = InterleavedBlocks(n, W, K)
    plans = [L.SpMVPlan(*ib.local_csr(rp, col, val, 0, k), n) for k in range(K)]
    ys = [torch.empty(ib.B, device=dev) for _ in range(K)]

    def step_plans():
        for p, y in zip(plans, ys):
            p(x, y)
    t = timed(step_plans)
    t1 = t if t1 is None else t1
    rec = dict(W=W, K=K, ms=t, ideal_ms=t1 / W, eff=t1 / W / t, kernel=plans[0].info()["kernel"],
               slices=plans[0].info()["slices"])
    for p in plans:
        p.close()
    if K > 1:
        lrp, lc, lv, splits = ib.local_csr_all(rp, col, val, 0)
        sp = L.SpMVPlan(lrp, lc, lv, n, splits=splits)

        def step_split():
            sp.stage(x)
            for k, y in enumerate(ys):
                sp.range(k, y)
        ts = timed(step_split)
        rec.update(split_ms=ts, split_eff=t1 / W / ts)
        if sp.info()["launches"] > 3:  # per-range gather pieces: lhpc_spmv runs gather k / reduce k
            yall = torch.empty(sp.n_rows, device=dev)
            tr = timed(lambda: sp(x, yall))
            rec.update(range_gather_ms=tr, range_gather_eff=t1 / W / tr)
        sp.close()
    print(json.dumps(rec), flush=True)
