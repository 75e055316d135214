"""CPU checks of the sort / COO→CSR oracle (oracle/oracle.c), pinned to the
reference's own CPU radix sort (compiled from its sources into oracle/_ref,
and the golden order it produced in tests/golden/sort_ref_*.npz) and to
numpy's stable sort.  No GPU."""
import numpy as np
import pytest

from tests import _support as S


@pytest.mark.parametrize("name", ["sort_ref_gpu_keys_5000.npz", "sort_ref_cpu_keys_4097.npz"])
def test_oracle_sort_matches_reference_golden(name):
    g = S.load_golden(name)
    assert np.array_equal(S.sort_oracle(g["keys"]), g["sorted"])
    assert np.all(np.diff(g["sorted"].astype(np.int64)) >= 0)  # the reference test's own property


def test_oracle_sort_matches_reference_library():
    ref = S.load_ref_sort()
    if ref is None:
        pytest.skip("oracle/_ref/libref_sort.so not built (reference absent)")
    for gen in (ref.ref_gpu_test_keys, ref.ref_generate_random):
        keys = np.empty(1_000_003, dtype=np.uint32)
        gen(keys.ctypes.data, keys.size)
        want = keys.copy()
        ref.ref_radix_sort_u32(want.ctypes.data, want.size)
        want4 = keys.copy()
        ref.ref_radix_sort_v4_u32(want4.ctypes.data, want4.size)
        got = S.sort_oracle(keys)
        assert np.array_equal(got, want) and np.array_equal(got, want4)


@pytest.mark.parametrize("kt", [np.uint32, np.uint64])
@pytest.mark.parametrize("begin,end", [(0, None), (0, 12), (4, 28), (3, 3), (7, 9)])
def test_oracle_sort_pairs_is_stable_on_bit_range(kt, begin, end):
    rng = np.random.default_rng(7 + begin)
    n = 20_011
    hi = np.iinfo(kt).max
    keys = rng.integers(0, hi, size=n, dtype=kt, endpoint=True)
    keys[::5] = keys[0]  # heavy duplicates
    vals = np.arange(n, dtype=np.uint32)
    e = keys.dtype.itemsize * 8 if end is None else end
    k, v = S.sort_oracle(keys, vals, begin, e)
    field = (keys >> kt(begin)) & kt((1 << (e - begin)) - 1) if e > begin else np.zeros(n, kt)
    order = np.argsort(field, kind="stable")
    assert np.array_equal(v, vals[order])
    assert np.array_equal(k, keys[order])  # bits outside the range ride along unchanged


def _coo_python(n_rows, n_cols, rows, cols, vals):
    """Independent restatement: dict of lists in input order, summed left to right."""
    acc = {}
    for r, c, v in zip(rows.tolist(), cols.tolist(), vals.tolist()):
        acc.setdefault((r, c), []).append(v)
    keys = sorted(acc)
    rp = np.zeros(n_rows + 1, dtype=np.int64)
    col = np.array([c for _, c in keys], dtype=np.int32)
    val = np.empty(len(keys), dtype=vals.dtype)
    for i, k in enumerate(keys):
        s = vals.dtype.type(acc[k][0])
        for x in acc[k][1:]:
            s = vals.dtype.type(s + vals.dtype.type(x))
        val[i] = s
        rp[k[0] + 1] += 1
    return np.cumsum(rp), col, val


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_oracle_coo_to_csr(dt):
    rng = np.random.default_rng(11)
    n_rows, n_cols, nnz = 300, 97, 5000
    rows = rng.integers(0, n_rows, nnz).astype(np.int32)
    cols = rng.integers(0, n_cols, nnz).astype(np.int32)
    rows[100:140] = 7  # a dense row with duplicates
    cols[100:140] = rng.integers(0, 5, 40)
    rows[rows == 13] = 14  # an empty row
    vals = rng.uniform(-1, 1, nnz).astype(dt)
    got = S.coo_oracle(n_rows, n_cols, rows, cols, vals)
    want = _coo_python(n_rows, n_cols, rows, cols, vals)
    for a, b in zip(got, want):
        assert np.array_equal(a, b)
    assert S.coo_oracle(4, 4, np.array([0, 4], np.int32), np.array([0, 0], np.int32),
                        np.ones(2, dt)) is None
    rp, col, val = S.coo_oracle(5, 5, np.zeros(0, np.int32), np.zeros(0, np.int32), np.zeros(0, dt))
    assert np.array_equal(rp, np.zeros(6, np.int64)) and col.size == 0 and val.size == 0
