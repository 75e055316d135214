"""Run by tests/test_debug_build.py in a child process with LHPC_LIB_PATH
pointing at the debug build (libhpc_amd/_lib_debug/liblhpc.so: device bounds
traps LHPC_DEVICE_CHECK + a synchronous check after every launch).  Valid
plans must run trap-free and bit-exact through every XTILE index stream
(perm / iperm), long rows across chunks, split ranges and fp32/fp64.
Test infrastructure only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import libhpc_amd as L  # noqa: E402
from tests import _support as S  # noqa: E402
from tests.test_gpu_spmv import FAMILIES, _csr_from_lengths  # noqa: E402

assert os.path.realpath(L.LIB_PATH) == os.path.realpath(os.environ["LHPC_LIB_PATH"]), L.LIB_PATH
dev = torch.device("cuda:0")
lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 3000 + [0, 0] + [30000]
n = len(lengths)
for ip in (0, 1):
    opts = {"xtile_reduce": L.XTILE_REDUCE_IPERM if ip else L.XTILE_REDUCE_PERM}
    for dt in (np.float32, np.float64):
        rp, col, val = _csr_from_lengths(lengths, 200_000, 0xD0 + ip, dyadic=True)
        val = val.astype(dt)
        x = (np.random.default_rng(7).integers(-8, 9, size=200_000) / 8.0).astype(dt)
        _, yr, _ = S.spmv_oracle(rp, col, val, x)
        splits = [1, 57, 2000, n - 1]
        with L.SpMVPlan(rp, col, val, 200_000, flags=FAMILIES["xtile"], splits=splits, options=opts) as plan:
            xd = torch.from_numpy(x).to(dev)
            y = plan(xd).cpu().numpy()
            assert np.array_equal(y, yr), ("xtile", ip, dt)
            bounds = [0] + splits + [n]
            ys = [torch.empty(bounds[k + 1] - bounds[k], dtype=xd.dtype, device=dev) for k in range(len(bounds) - 1)]
            plan.stage(xd)
            for k, yk in enumerate(ys):
                plan.range(k, yk)
            assert np.array_equal(torch.cat(ys).cpu().numpy(), yr), ("ranges", ip, dt)
for name in ("adaptive", "rowgroup", "xslice"):
    g = S.load_golden("spmv_powerlaw_dyadic_f32_n2000.npz")
    with L.SpMVPlan(g["row_ptr"], g["col_idx"], g["val"], int(g["n_cols"]), flags=FAMILIES[name]) as plan:
        y = plan(torch.from_numpy(g["x"]).to(dev)).cpu().numpy()
    assert np.array_equal(y, g["y_exact"].astype(np.float32)), name
# CG error path: a solve whose 4th iteration body fails after
# enqueueing its work returns LHPC_ERR_INTERNAL and frees the plan only once
# its stream has drained; a second solve on another stream then equals a
# clean solve bit for bit (SELL: fused loop; spmv_no_sell: ADAPTIVE loop)
rp, col, val = S.laplacian_2d(150, 130, dtype=np.float64)
n = rp.size - 1
b = torch.from_numpy(np.random.default_rng(21).uniform(-1, 1, n)).to(dev)
for opts in (None, {"spmv_no_sell": 1}):
    with L.SpMVPlan(rp, col, val, n, options=opts) as plan:
        s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
        x_ref, it_ref, r_ref = L.cg(plan, b, tol=1e-10, max_iter=200, check_every=8, stream=s1)
        s1.synchronize()
        L.lib.lhpc_debug_cg_fail_at(3)
        try:
            L.cg(plan, b, tol=1e-10, max_iter=200, check_every=8, stream=s1)
            raise AssertionError("the injected CG fault did not surface")
        except L.LhpcError as e:
            assert e.status == -6, e.status
        x2, it2, r2 = L.cg(plan, b, tol=1e-10, max_iter=200, check_every=8, stream=s2)
        s2.synchronize()
        assert torch.equal(x2, x_ref) and (it2, r2) == (it_ref, r_ref), (opts, it2, it_ref)
torch.cuda.synchronize()
print("DEBUG BUILD OK")
