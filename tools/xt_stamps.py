"""Phase timing of the XTILE reduce from in-kernel stamps (diagnostic build:
make -C libhpc_amd/csrc BUILD=../_build_stamps OUT=../_lib_stamps
EXTRA_HIPFLAGS=-DLHPC_XT_STAMPS ../_lib_stamps/liblhpc.so — not under _ab/,
which gpurun does not send — loaded with LHPC_LIB_PATH).  One SpMV after warm-up; per block: s_memtime deltas between
the phase boundaries of k_xtile_reduce (thread 0 of each block), and the
realtime span.  Prints JSON: median / mean / p90 per phase in cycles."""
import ctypes as C
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import libhpc_amd as L  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
dt = L.F64 if wl == "c3" else L.F32
n = 10_000_000
if wl == "c4":
    rp, col, val = L.gen_powerlaw_csr(n, n, dtype=dt)
else:
    rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=dt)
x = torch.from_numpy(L.gen_values(dt, 0, n, L.SEED_X)).cuda()
plan = L.SpMVPlan(rp, col, val, n)
y = torch.empty(n, dtype=x.dtype, device=x.device)
for _ in range(5):
    plan(x, y)
torch.cuda.synchronize()
L.lib.lhpc_probe_xtile_stamps_clear()
plan(x, y)
torch.cuda.synchronize()
nb = plan.info()["n_blocks"]
nblk = 8 * ((nb + 7) // 8)
buf = np.zeros(nblk * 10, dtype=np.uint64)
assert L.lib.lhpc_probe_xtile_stamps(C.c_void_p(buf.ctypes.data), C.c_int64(buf.size)) == 0
st = buf.reshape(nblk, 10).astype(np.int64)
st = st[st[:, 1] != 0]
names = ["rt1+scan1", "scan2", "phaseA_issue", "rowptr+waitxg", "phaseB+segscan", "combine", "ystore"]
cols = [1, 2, 3, 4, 5, 6, 7, 8]
out = {"workload": wl, "blocks": int(st.shape[0])}
for i, nm in enumerate(names):
    d = st[:, cols[i + 1]] - st[:, cols[i]]
    out[nm] = {"median": float(np.median(d)), "mean": float(d.mean()), "p90": float(np.percentile(d, 90))}
tot = st[:, 8] - st[:, 1]
out["total_cycles"] = {"median": float(np.median(tot)), "mean": float(tot.mean())}
rt = st[:, 9] - st[:, 0]
out["block_realtime_us"] = {"median": float(np.median(rt)) / 100.0, "mean": float(rt.mean()) / 100.0}
t0, t1 = st[:, 0].min(), st[:, 9].max()
out["kernel_span_us"] = float(t1 - t0) / 100.0
# average concurrent blocks = sum of block times / span
out["avg_concurrent_blocks"] = float(rt.sum()) / float(t1 - t0)
out["clock_mhz_est"] = float(np.median(tot / np.maximum(rt, 1))) * 100.0
print(json.dumps(out, indent=1))
