"""Pin the oracle (oracle/oracle.c) before trusting it.

* blur: bit-exact against the golden fixtures produced by the reference's own
  container + BM_x_blur/BM_y_blur loop semantics (oracle/_ref/ref_probe);
  the SSE CPU baselines (restating test_hpc_benchmark.cpp:425-441, :575-601)
  are bit-exact too.
* SpMV (absent from the reference — parity unpinned by it): pinned to exact
  arithmetic — Fractions-exact fixtures — and cross-checked with
  scipy.sparse; the AVX2 CPU baseline stays within the 1e-6 bound.
* generators: deterministic, thread-count independent, checksums frozen.
"""
import glob
import hashlib
import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from tests import _support as S


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(S.GOLDEN, "spmv_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_spmv_oracle_vs_exact_fixtures(path):
    g = S.load_golden(os.path.basename(path))
    y64, yr, asum = S.spmv_oracle(g["row_ptr"], g["col_idx"], g["val"], g["x"])
    if "dyadic" in path:
        assert np.array_equal(y64, g["y_exact"])
        assert np.array_equal(yr, g["y_exact"].astype(g["val"].dtype))
    else:
        # sequential fp64: |err| <= (k-1) * 2^-53 * sum|p| for a k-term row
        lens = np.diff(g["row_ptr"].astype(np.int64))
        bound = np.maximum(lens, 1) * 2.0 ** -53 * asum
        assert np.all(np.abs(y64 - g["y_exact"]) <= bound + 1e-300)


def test_spmv_oracle_vs_fsum_and_scipy(lhpc):
    import scipy.sparse as sp
    n = 3000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=lhpc.F32, seed=77)
    x = lhpc.gen_values(lhpc.F32, 0, n, 78)
    y64, _, asum = S.spmv_oracle(rp, col, val, x)
    fs = np.array([math.fsum(float(val[k]) * float(x[col[k]]) for k in range(rp[i], rp[i + 1]))
                   for i in range(n)])
    assert np.all(np.abs(y64 - fs) <= 15 * 2.0 ** -53 * asum + 1e-300)
    A = sp.csr_matrix((val.astype(np.float64), col, rp), shape=(n, n))
    assert np.allclose(A @ x.astype(np.float64), y64, rtol=0, atol=1e-12)


@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_cpu_simd_baseline_within_bound(lhpc, dtype):
    dt = lhpc.F32 if dtype == "f32" else lhpc.F64
    n = 20_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=dt, seed=5)
    x = lhpc.gen_values(dt, 0, n, 6)
    y, used = S.spmv_cpu_simd(rp, col, val, x, threads=2)
    assert used == 2
    y64, _, asum = S.spmv_oracle(rp, col, val, x)
    S.assert_spmv_close(y, y64, asum)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(S.GOLDEN, "blur_*.npz"))),
                         ids=lambda p: os.path.basename(p)[:-4])
def test_blur_oracle_vs_reference_fixtures(path):
    g = S.load_golden(os.path.basename(path))
    ny, nx, ghost, nb = (int(g[k]) for k in ("ny", "nx", "ghost", "nblur"))
    ydir = os.path.basename(path).startswith("blur_y")
    assert np.array_equal(S.blur_oracle(g["a"], ny, nx, ghost, nb, ydir), g["b"])


@pytest.mark.parametrize("ydir", [False, True])
def test_sse_blur_baseline_bit_exact(ydir):
    ny, nx, g = 96, 256, 8
    a = S.random_padded(((ny + 2 * g) * (nx + 2 * g),), seed=3)
    want = S.blur_oracle(a, ny, nx, g, 8, ydir)
    lib = S.load_oracle()
    b = np.empty(ny * nx, dtype=np.float32)
    (lib.cpu_blur_y_sse if ydir else lib.cpu_blur_x_sse)(a.ctypes.data, b.ctypes.data, ny, nx, g, 2)
    assert np.array_equal(b, want)


def test_ref_probe_reproduces_fixture():
    """When the reference-header probe is built, re-running it reproduces the
    committed bytes (guards the fixture provenance)."""
    if not os.path.exists(S.REF_PROBE):
        pytest.skip("oracle/_ref/ref_probe not built (needs /root/reference at build time)")
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        pre = os.path.join(td, "t")
        subprocess.run([S.REF_PROBE, "blur", "y", "131", "257", "0x5EED0010", "0", pre], check=True)
        g = S.load_golden("blur_y_131x257_randghost.npz")
        assert np.array_equal(np.fromfile(pre + "_a.f32", np.float32), g["a"])
        assert np.array_equal(np.fromfile(pre + "_b.f32", np.float32), g["b"])


def test_stencil7_oracle_matches_numpy():
    nz, ny, nx = 5, 6, 7
    u = S.random_padded((nz + 2, ny + 2, nx + 2), seed=11)
    out = S.stencil7_oracle(u.reshape(-1), nz, ny, nx, 1, -6.0, 1.0).reshape(u.shape)
    c = u[1:-1, 1:-1, 1:-1]
    s = (((((u[:-2, 1:-1, 1:-1] + u[2:, 1:-1, 1:-1]) + u[1:-1, :-2, 1:-1]) + u[1:-1, 2:, 1:-1])
          + u[1:-1, 1:-1, :-2]) + u[1:-1, 1:-1, 2:])
    assert np.array_equal(out[1:-1, 1:-1, 1:-1], np.float32(-6.0) * c + np.float32(1.0) * s)
    assert np.all(out[0] == 0) and np.all(out[:, :, -1] == 0)  # ghosts untouched


def test_generator_checksums_frozen(lhpc):
    want = json.load(open(os.path.join(S.GOLDEN, "gen_checksums.json")))
    rp, col, val = lhpc.gen_uniform_csr(100_000, 100_000, 10, dtype=lhpc.F64)
    h = hashlib.sha256()
    for a in (rp, col, val, lhpc.gen_values(lhpc.F64, 0, 100_000, lhpc.SEED_X)):
        h.update(np.ascontiguousarray(a).tobytes())
    assert h.hexdigest() == want["C1_uniform_n1e5_10_f64"]


def test_generator_thread_count_independent():
    code = ("import sys, hashlib, numpy as np; sys.path.insert(0, %r); import libhpc_amd as L; "
            "rp,col,val=L.gen_powerlaw_csr(50000,50000,lmax=3000); "
            "print(hashlib.sha256(rp.tobytes()+col.tobytes()+val.tobytes()).hexdigest())" % S.ROOT)
    outs = set()
    for t in ("1", "3", "8"):
        env = dict(os.environ, OMP_NUM_THREADS=t)
        outs.add(subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                                check=True).stdout.strip())
    assert len(outs) == 1


def test_generator_shapes(lhpc):
    rp, col, val = lhpc.gen_uniform_csr(5000, 700, 15, dtype=lhpc.F32)
    assert rp.dtype == np.int32 and rp[-1] == 75_000
    for i in range(0, 5000, 97):
        seg = col[rp[i]:rp[i + 1]]
        assert np.all(np.diff(seg) > 0) and seg.min() >= 0 and seg.max() < 700
    rp, col, _ = lhpc.gen_powerlaw_csr(100_000, 100_000, lmax=10_000)
    lens = np.diff(rp.astype(np.int64))
    assert lens.max() == 10_000 and lens.min() >= 1
    assert 10 < lens.mean() < 20  # mean ≈ 15 for alpha = 1.792
    assert np.sum(lens == 10_000) >= 3  # rows 0, n/2, n-1 forced (then shuffled)
    d = lhpc.gen_values(lhpc.F32, 1, 10_000, 1)
    assert set(np.unique(d * 8).astype(int)) <= set(range(-8, 9))


def test_partition_rows(lhpc):
    rp = np.array([0, 5, 5, 6, 20, 21, 30], dtype=np.int64)
    cuts = lhpc.csr_partition_rows(rp, 3)
    assert cuts[0] == 0 and cuts[-1] == 6 and np.all(np.diff(cuts) >= 0)
    for p in range(1, 3):
        target = -(-p * 30 // 3)
        assert rp[cuts[p]] >= target and (cuts[p] == 0 or rp[cuts[p] - 1] < target)
    rp32 = rp.astype(np.int32)
    assert np.array_equal(lhpc.csr_partition_rows(rp32, 3), cuts)
