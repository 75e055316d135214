"""Per-rank local work (W = 4 / 8, K = 1 / 2, C2 fp32 and C3 fp64) with the XTILE
reduce index stream chosen automatically, forced perm, or forced iperm
(lhpc_options.xtile_reduce): which suits the small per-rank plans."""
import json, os, sys
import torch
sys.path.insert(0, os.getcwd())
import libhpc_amd as L
dev = torch.device("cuda:0")
n = 10_000_000
def timed(step, reps=30):
    for _ in range(3): step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): step()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps
for dts in ("f32", "f64"):
    dt = L.F32 if dts == "f32" else L.F64
    rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=dt)
    x = torch.from_numpy(L.gen_values(dt, 0, n, L.SEED_X)).to(dev)
    for W in (4, 8):
        for K in (1, 2):
            cuts = L.interleaved_cuts(rp, W, K)
            lrp, lc, lv = L.interleaved_local_csr(rp, col, val, cuts, W, K, 0)
            comm = L.DistComm.local(W, 0, 0)
            y = torch.empty(n, dtype=x.dtype, device=dev)
            rec = {"dtype": dts, "W": W, "K": K}
            for name, red in (("auto", 0), ("perm", 1), ("iperm", 2)):
                with L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv,
                                    options={"dist_exchange": L.DIST_EXCHANGE_NONE, "xtile_reduce": red}) as d:
                    rec[name] = timed(lambda: d(x, y))
            comm.close()
            print(json.dumps(rec), flush=True)
