"""Test helpers: the oracle (CPU restatement, oracle/oracle.c) via ctypes and
numpy-facing wrappers.  Test infrastructure only."""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
REF_PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")
REF_SORT_SO = os.path.join(ROOT, "oracle", "_ref", "libref_sort.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

_p, _i, _i64, _f = C.c_void_p, C.c_int, C.c_int64, C.c_float
_lib = None


def load_oracle():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "_build/liboracle.so"],
                           check=True, capture_output=True)
        lib = C.CDLL(ORACLE_SO)
        lib.oracle_spmv_f32.argtypes = [_i64, _p, _i, _p, _p, _p, _p, _p, _p]
        lib.oracle_spmv_f64.argtypes = [_i64, _p, _i, _p, _p, _p, _p, _p]
        lib.cpu_spmv_simd.argtypes = [_i, _i64, _p, _i, _p, _p, _p, _p, _i]
        lib.cpu_spmv_simd.restype = _i
        lib.oracle_blur_x.argtypes = [_p, _p, _i64, _i64, _i64, _i]
        lib.oracle_blur_y.argtypes = [_p, _p, _i64, _i64, _i64, _i]
        lib.cpu_blur_x_sse.argtypes = [_p, _p, _i64, _i64, _i64, _i]
        lib.cpu_blur_y_sse.argtypes = [_p, _p, _i64, _i64, _i64, _i]
        lib.cpu_blur_x_sse.restype = _i
        lib.cpu_blur_y_sse.restype = _i
        lib.oracle_stencil7.argtypes = [_p, _p, _i64, _i64, _i64, _i64, _f, _f, _i]
        lib.oracle_cg_f64.argtypes = [_i64, _p, _i, _p, _p, _p, _p, C.c_double, _i, _p]
        lib.oracle_cg_f64.restype = _i
        lib.oracle_radix_sort_u32.argtypes = [_p, _p, _i64, _i, _i]
        lib.oracle_radix_sort_u64.argtypes = [_p, _p, _i64, _i, _i]
        for f in (lib.oracle_coo_to_csr_f32, lib.oracle_coo_to_csr_f64):
            f.argtypes = [_i64, _i64, _i64, _p, _p, _p, _p, _p, _p]
            f.restype = _i64
        _lib = lib
    return _lib


def _ptr(a):
    return a.ctypes.data if a is not None else None


def _bits(rp):
    return 64 if rp.dtype == np.int64 else 32


def spmv_oracle(rp, col, val, x):
    """(y64, y_rounded, abs_sum): fp64 sequential ascending-k sums."""
    lib = load_oracle()
    n = rp.shape[0] - 1
    y64 = np.empty(n, dtype=np.float64)
    asum = np.empty(n, dtype=np.float64)
    if val.dtype == np.float32:
        y32 = np.empty(n, dtype=np.float32)
        lib.oracle_spmv_f32(n, _ptr(rp), _bits(rp), _ptr(col), _ptr(val), _ptr(x), _ptr(y64),
                            _ptr(y32), _ptr(asum))
        return y64, y32, asum
    lib.oracle_spmv_f64(n, _ptr(rp), _bits(rp), _ptr(col), _ptr(val), _ptr(x), _ptr(y64), _ptr(asum))
    return y64, y64.copy(), asum


def spmv_cpu_simd(rp, col, val, x, threads=0):
    lib = load_oracle()
    n = rp.shape[0] - 1
    y = np.empty(n, dtype=val.dtype)
    used = lib.cpu_spmv_simd(0 if val.dtype == np.float32 else 1, n, _ptr(rp), _bits(rp), _ptr(col),
                             _ptr(val), _ptr(x), _ptr(y), threads)
    return y, used


# Parity bound for fp SpMV (north_star: "fp within 1e-6 relative"): per row
# |y - y_exact| <= 1e-6 * sum_k |a_k x_k| (+ a denormal floor), and norm-wise
# ||dy||_inf <= 1e-6 * ||y||_inf when y is not all-cancellation.
SPMV_RTOL = 1e-6


def assert_spmv_close(y, y64, asum, rtol=SPMV_RTOL):
    y = np.asarray(y, dtype=np.float64)
    err = np.abs(y - y64)
    bound = rtol * asum + 1e-30
    bad = np.nonzero(err > bound)[0]
    assert bad.size == 0, (
        f"{bad.size} rows exceed |dy| <= {rtol}*sum|a*x|; first row {bad[0]}: "
        f"got {y[bad[0]]!r} want {y64[bad[0]]!r} bound {bound[bad[0]]!r}")
    ninf = np.max(np.abs(y64)) if y64.size else 0.0
    if ninf > 0:
        assert np.max(err) <= rtol * max(ninf, np.max(asum) * 1e-3), "norm-wise error above 1e-6"


def blur_oracle(a, ny, nx, ghost, nblur, ydir):
    lib = load_oracle()
    b = np.empty(ny * nx, dtype=np.float32)
    (lib.oracle_blur_y if ydir else lib.oracle_blur_x)(_ptr(a), _ptr(b), ny, nx, ghost, nblur)
    return b


def stencil7_oracle(u, nz, ny, nx, g, c0, c1, out=None):
    lib = load_oracle()
    if out is None:
        out = np.zeros_like(u)
    lib.oracle_stencil7(_ptr(u), _ptr(out), nz, ny, nx, g, c0, c1, 0)
    return out


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def random_padded(shape, seed, zero_ghost=False, ghost=0):
    rng = np.random.default_rng(seed)
    a = rng.uniform(-1, 1, size=shape).astype(np.float32)
    if zero_ghost and ghost:
        m = np.zeros(shape, dtype=bool)
        sl = tuple(slice(ghost, s - ghost) for s in shape)
        m[sl] = True
        a[~m] = 0
    return a


# ------------------------------------------------------------ sort / COO→CSR
def sort_oracle(keys, vals=None, begin=0, end=None):
    """Stable LSD restatement (oracle.c); returns sorted copies."""
    lib = load_oracle()
    k = np.ascontiguousarray(keys).copy()
    v = None if vals is None else np.ascontiguousarray(vals, dtype=np.uint32).copy()
    end = k.dtype.itemsize * 8 if end is None else end
    fn = lib.oracle_radix_sort_u64 if k.dtype == np.uint64 else lib.oracle_radix_sort_u32
    fn(_ptr(k), _ptr(v), k.size, begin, end)
    return k if v is None else (k, v)


def coo_oracle(n_rows, n_cols, rows, cols, vals):
    """(row_ptr int64, col int32, val) or None for out-of-range input."""
    lib = load_oracle()
    nnz = rows.size
    rp = np.zeros(n_rows + 1, dtype=np.int64)
    col = np.empty(max(nnz, 1), dtype=np.int32)
    val = np.empty(max(nnz, 1), dtype=vals.dtype)
    fn = lib.oracle_coo_to_csr_f32 if vals.dtype == np.float32 else lib.oracle_coo_to_csr_f64
    u = fn(n_rows, n_cols, nnz, _ptr(rows), _ptr(cols), _ptr(vals), _ptr(rp), _ptr(col), _ptr(val))
    if u < 0:
        return None
    return rp, col[:u].copy(), val[:u].copy()


_ref_sort = None


def load_ref_sort():
    """The reference's own CPU radix sort (oracle/_ref/libref_sort.so), or None
    when it was not built (reference absent and no prebuilt copy)."""
    global _ref_sort
    if _ref_sort is None and os.path.exists(REF_SORT_SO):
        lib = C.CDLL(REF_SORT_SO)
        for f in ("ref_radix_sort_u32", "ref_radix_sort_v4_u32", "ref_generate_random", "ref_gpu_test_keys"):
            getattr(lib, f).argtypes = [_p, C.c_size_t]
        _ref_sort = lib
    return _ref_sort


def ref_gpu_test_keys(n):
    """The reference GPU test's keys (mt19937 default seed, U[100, 2^32-101]),
    from oracle/_ref, or None."""
    lib = load_ref_sort()
    if lib is None:
        return None
    a = np.empty(n, dtype=np.uint32)
    lib.ref_gpu_test_keys(_ptr(a), n)
    return a


# ------------------------------------------------------------ CG
def cg_oracle(rp, col, val, b, x0=None, tol=1e-8, max_iter=1000):
    """fp64 CG restatement (oracle.c): (x, iterations, ‖r‖/‖b‖)."""
    lib = load_oracle()
    n = rp.size - 1
    v = np.ascontiguousarray(val, dtype=np.float64)
    bb = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros(n) if x0 is None else np.array(x0, dtype=np.float64)
    res = C.c_double(0.0)
    it = lib.oracle_cg_f64(n, _ptr(rp), _bits(rp), _ptr(col), _ptr(v), _ptr(bb), _ptr(x), tol, max_iter,
                           C.byref(res))
    return x, it, res.value


def laplacian_2d(nx, ny, dtype=np.float64, shift=0.0):
    """5-point Dirichlet Laplacian CSR (libhpc_amd.gen_laplacian_2d; int32 row_ptr)."""
    import libhpc_amd as L
    rp, col, val = L.gen_laplacian_2d(nx, ny, L.F32 if dtype == np.float32 else L.F64, shift)
    return rp.astype(np.int32), col, val


def sampled_rows_fp64(rp, col, val, x, m, seed=0x5EED00C1):
    """(rows, y64, Σ|a·x|) on m seeded rows, fp64 numpy (no oracle/ code):
    the full-size checks where the oracle's whole-matrix pass is too slow."""
    n = rp.shape[0] - 1
    rows = np.sort(np.random.default_rng(seed).choice(n, size=min(m, n), replace=False))
    lo, hi = rp[rows].astype(np.int64), rp[rows + 1].astype(np.int64)
    lens = hi - lo
    idx = np.repeat(lo - np.concatenate(([0], np.cumsum(lens)[:-1])), lens) + np.arange(lens.sum())
    prod = val[idx].astype(np.float64) * x[col[idx]].astype(np.float64)
    seg = np.repeat(np.arange(rows.size), lens)
    return rows, np.bincount(seg, weights=prod, minlength=rows.size), \
        np.bincount(seg, weights=np.abs(prod), minlength=rows.size)
