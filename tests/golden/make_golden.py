"""Regenerate the golden fixtures in tests/golden/ (committed; run here, where
/root/reference and oracle/_ref/ref_probe exist).

Provenance of every fixture:
  blur_*.npz     produced by oracle/_ref/ref_probe, a driver compiled against
                 the REFERENCE's own lib/hpc/include/HPCHighDimensionFlatArray.hpp:
                 input a.data() and output b.data() bytes of the reference
                 container, b computed with the BM_x_blur / BM_y_blur loop
                 (test_hpc_benchmark.cpp:354-368, :444-457) through the
                 reference operator().
  layout.json    flat offsets reported by the reference container's at().
  spmv_*.npz     SpMV has no reference implementation.  Inputs
                 come from the deterministic generators (or are hand-built
                 edge shapes); y_exact is the EXACT row sum computed with
                 Python Fractions and rounded once to float64 — independent
                 of both the oracle and the GPU kernels.
  sort_ref_*.npz keys from the reference's own input generators and their
                 order as produced by the REFERENCE's CPU radix sort
                 (oracle/_ref/libref_sort.so, compiled from
                 lib/sort/radix_cpu/include/radix_sort_cpu.hpp + src/helper.cpp):
                 sort::radix::radix_sort (radix_sort_cache_thread_v2<256>).
  gen_checksums.json  sha256 of generator outputs for the BASELINE configs,
                 so a generator change cannot silently change the workload.

Usage:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
import libhpc_amd as L  # noqa: E402  (host-side generators only; no GPU used)

PROBE = os.path.join(ROOT, "oracle", "_ref", "ref_probe")


def exact_spmv(rp, col, val, x):
    y = np.empty(rp.shape[0] - 1, dtype=np.float64)
    for i in range(rp.shape[0] - 1):
        s = Fraction(0)
        for k in range(int(rp[i]), int(rp[i + 1])):
            s += Fraction(float(val[k])) * Fraction(float(x[col[k]]))
        y[i] = float(s)  # correctly rounded
    return y


def save_spmv(name, rp, col, val, x, n_cols, note):
    y = exact_spmv(rp, col, val, x)
    np.savez_compressed(os.path.join(HERE, name), row_ptr=rp, col_idx=col, val=val, x=x,
                        n_cols=np.int64(n_cols), y_exact=y, note=np.str_(note))
    print("wrote", name, "rows", rp.shape[0] - 1, "nnz", col.shape[0])


def spmv_fixtures():
    # uniform, dyadic-exact values: every summation order gives identical y
    for n, per, dt, dist, tag in ((1000, 15, L.F32, 1, "dyadic_f32_n1000"),
                                  (65, 15, L.F32, 0, "rand_f32_n65"),
                                  (63, 15, L.F64, 0, "rand_f64_n63"),
                                  (1, 1, L.F32, 0, "rand_f32_n1"),
                                  (64, 64, L.F64, 1, "dyadic_f64_n64_full")):
        rp, col, val = L.gen_uniform_csr(n, n, per, dtype=dt, dist=dist, seed=0xF1 + n)
        x = L.gen_values(dt, dist, n, 0xF2 + n)
        save_spmv(f"spmv_{tag}.npz", rp, col, val, x, n, f"uniform {per}/row")
    # rectangular: n_cols != n_rows, int64 row_ptr
    rp, col, val = L.gen_uniform_csr(4099, 3001, 7, dtype=L.F64, dist=1, seed=0xF3, narrow=False)
    x = L.gen_values(L.F64, 1, 3001, 0xF4)
    save_spmv("spmv_dyadic_f64_4099x3001_rp64.npz", rp, col, val, x, 3001, "rectangular, int64 row_ptr")
    # empty rows interleaved, including leading/trailing empties
    lens = np.array([0, 3, 0, 0, 17, 1, 0, 64, 65, 0, 2, 0], dtype=np.int64)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.empty(int(rp[-1]), dtype=np.int32)
    L._check(L.lib.lhpc_gen_fill_cols(lens.size, 200, rp.astype(np.int64).ctypes.data, 0xF5,
                                      col.ctypes.data), "fill")
    val = L.gen_values(L.F32, 0, col.size, 0xF6)
    x = L.gen_values(L.F32, 0, 200, 0xF7)
    save_spmv("spmv_empty_rows_f32.npz", rp, col, val, x, 200, "empty rows incl. first/last")
    # one dense row of 10^4 entries between short rows
    lens = np.array([2, 10_000, 5], dtype=np.int64)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    col = np.empty(int(rp[-1]), dtype=np.int32)
    L._check(L.lib.lhpc_gen_fill_cols(3, 20_000, rp.astype(np.int64).ctypes.data, 0xF8,
                                      col.ctypes.data), "fill")
    val = L.gen_values(L.F32, 0, col.size, 0xF9)
    x = L.gen_values(L.F32, 0, 20_000, 0xFA)
    save_spmv("spmv_dense_row_f32.npz", rp, col, val, x, 20_000, "single 10^4-nnz row")
    # power-law rows (skew), dyadic
    rp, col, val = L.gen_powerlaw_csr(2000, 2000, lmax=1500, dtype=L.F32, dist=1, seed=0xFB)
    x = L.gen_values(L.F32, 1, 2000, 0xFC)
    save_spmv("spmv_powerlaw_dyadic_f32_n2000.npz", rp, col, val, x, 2000, "power law lmax 1500")


def blur_fixtures():
    if not os.path.exists(PROBE):
        print("oracle/_ref/ref_probe missing: run `make -C oracle` where /root/reference exists")
        return
    with tempfile.TemporaryDirectory() as td:
        for ny, nx in ((64, 64), (131, 257)):
            for zero in (0, 1):
                for d in ("x", "y"):
                    pre = os.path.join(td, f"b{d}{ny}_{nx}_{zero}")
                    subprocess.run([PROBE, "blur", d, str(ny), str(nx), "0x5EED0010", str(zero), pre],
                                   check=True)
                    a = np.fromfile(pre + "_a.f32", dtype=np.float32)
                    b = np.fromfile(pre + "_b.f32", dtype=np.float32)
                    name = f"blur_{d}_{ny}x{nx}_{'zeroghost' if zero else 'randghost'}.npz"
                    np.savez_compressed(os.path.join(HERE, name), a=a, b=b, ny=np.int64(ny),
                                        nx=np.int64(nx), ghost=np.int64(8), nblur=np.int64(8))
                    print("wrote", name)


def layout_fixture():
    if not os.path.exists(PROBE):
        return
    out = []
    for args in (["layout2", "5", "7", "8"], ["layout2", "3", "4", "0"], ["layout2", "9", "2", "1"],
                 ["layout3", "4", "5", "6"], ["layout3", "1", "1", "1"]):
        r = subprocess.run([PROBE] + args, check=True, capture_output=True, text=True)
        out.append(json.loads(r.stdout))
    with open(os.path.join(HERE, "layout.json"), "w") as f:
        json.dump({"source": "oracle/_ref/ref_probe (reference HPCHighDimensionFlatArray.hpp)",
                   "cases": out}, f, indent=1)
    print("wrote layout.json")


def gen_checksums():
    def h(*arrs):
        m = hashlib.sha256()
        for a in arrs:
            m.update(np.ascontiguousarray(a).tobytes())
        return m.hexdigest()
    sums = {}
    rp, col, val = L.gen_uniform_csr(100_000, 100_000, 10, dtype=L.F64)
    sums["C1_uniform_n1e5_10_f64"] = h(rp, col, val, L.gen_values(L.F64, 0, 100_000, L.SEED_X))
    rp, col, val = L.gen_uniform_csr(1_000_000, 1_000_000, 15, dtype=L.F32)
    sums["uniform_n1e6_15_f32"] = h(rp, col, val, L.gen_values(L.F32, 0, 1_000_000, L.SEED_X))
    rp, col, val = L.gen_powerlaw_csr(1_000_000, 1_000_000, dtype=L.F32)
    sums["powerlaw_n1e6_f32"] = h(rp, col, val)
    with open(os.path.join(HERE, "gen_checksums.json"), "w") as f:
        json.dump(sums, f, indent=1)
    print("wrote gen_checksums.json")


def sort_fixtures():
    import ctypes as C
    so = os.path.join(ROOT, "oracle", "_ref", "libref_sort.so")
    if not os.path.exists(so):
        print("oracle/_ref/libref_sort.so missing: run `make -C oracle` where /root/reference exists")
        return
    lib = C.CDLL(so)
    for f in ("ref_radix_sort_u32", "ref_generate_random", "ref_gpu_test_keys"):
        getattr(lib, f).argtypes = [C.c_void_p, C.c_size_t]
    for name, gen, n in (("sort_ref_gpu_keys_5000.npz", lib.ref_gpu_test_keys, 5000),
                         ("sort_ref_cpu_keys_4097.npz", lib.ref_generate_random, 4097)):
        keys = np.empty(n, dtype=np.uint32)
        gen(keys.ctypes.data, n)
        out = keys.copy()
        lib.ref_radix_sort_u32(out.ctypes.data, n)
        np.savez_compressed(os.path.join(HERE, name), keys=keys, sorted=out)
        print("wrote", name)


if __name__ == "__main__":
    sort_fixtures()
    spmv_fixtures()
    blur_fixtures()
    layout_fixture()
    gen_checksums()
