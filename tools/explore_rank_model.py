"""Per-rank local work of the N > 1 SpMV (bench.py --gpus N, lhpc_dist_spmv),
simulated on one GPU for the step model (tools/step_model.py): rank 0's K
interleaved nnz-balanced blocks of the C2 (fp32) and C3 (fp64) matrices for
world W, as the row-range XTILE plan lhpc_dist_spmv builds.  Per (dtype, W,
K): the stage (tile gather) alone, the whole local call (stage + K chunk
reduces + fix-ups), the local call through the native plan with exchange
NONE, and the same local call with the stage launched by column part (the
chained form).  One JSON line each.  No collective runs here."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
n = 10_000_000
REPS = 20


def timed(step):
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        step()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / REPS


for dts in (os.environ.get("DTYPES", "f32 f64")).split():
    dt = L.F32 if dts == "f32" else L.F64
    rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=dt)
    x = torch.from_numpy(L.gen_values(dt, 0, n, L.SEED_X)).to(dev)
    t1 = None
    for W in (1, 2, 4, 8):
        for K in (1, 2, 3, 4):
            cuts = L.interleaved_cuts(rp, W, K)
            lrp, lc, lv = L.interleaved_local_csr(rp, col, val, cuts, W, K, 0)
            rec = {"dtype": dts, "W": W, "K": K, "local_rows": int(lrp.shape[0] - 1), "local_nnz": int(lc.shape[0])}
            comm = L.DistComm.local(W, 0, 0)
            y = torch.empty(n, dtype=x.dtype, device=dev)
            with L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv,
                                options={"dist_exchange": L.DIST_EXCHANGE_NONE}) as d:
                rec["local_ms"] = timed(lambda: d(x, y))
            if K > 1:  # the chunk reduces on one stream (round 3's schedule)
                with L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv,
                                    options={"dist_exchange": L.DIST_EXCHANGE_NONE, "dist_reduce_streams": 1}) as d:
                    rec["local_ms_1stream"] = timed(lambda: d(x, y))
            comm.close()
            if K > 1:
                splits = [int(v) for v in (lambda ls: ls[1:-1])(
                    [sum(int(cuts[k * W + 1] - cuts[k * W]) for k in range(j)) for j in range(K + 1)])]
                try:
                    sp = L.SpMVPlan(lrp, lc, lv, n, splits=splits)
                    rec["stage_ms"] = timed(lambda: sp.stage(x))
                    rec["launches"] = sp.info()["launches"]
                    sp.close()
                except L.LhpcError as e:
                    rec["stage_ms"] = None
                    rec["note"] = str(e)
            if t1 is None:
                t1 = rec["local_ms"]
            rec["ideal_ms"] = t1 / W
            rec["eff"] = t1 / W / rec["local_ms"]
            print(json.dumps(rec), flush=True)
    del rp, col, val, x
