""".lcsr container and Matrix Market reader.

The reference has no file formats, so the Matrix Market reader is pinned to an
independent implementation, scipy.io.mmread / mmwrite: the parsed triples
(host, no GPU) and the assembled CSR (GPU, lhpc_coo_to_csr) must equal
scipy's exactly."""
import os

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp


def _rand_csr(n_rows, n_cols, density, dt, seed):
    A = sp.random(n_rows, n_cols, density=density, format="csr", dtype=np.float64,
                  random_state=np.random.default_rng(seed))
    A.sort_indices()
    return A.indptr, A.indices.astype(np.int32), A.data.astype(dt)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("rp_t", [np.int32, np.int64])
@pytest.mark.parametrize("shape", [(200, 300, 0.05), (1, 1, 1.0), (0, 5, 0.0), (50, 0, 0.0), (1000, 17, 0.0)])
def test_lcsr_roundtrip(lhpc, tmp_path, dt, rp_t, shape):
    n_rows, n_cols, d = shape
    if n_rows * n_cols == 0 or d == 0:
        rp = np.zeros(n_rows + 1, rp_t)
        col = np.zeros(0, np.int32)
        val = np.zeros(0, dt)
    else:
        rp, col, val = _rand_csr(n_rows, n_cols, d, dt, n_rows)
        rp = rp.astype(rp_t)
    f = str(tmp_path / "m.lcsr")
    lhpc.save_csr(f, rp, col, val, n_cols)
    rp2, col2, val2, nc2 = lhpc.load_csr(f)
    assert nc2 == n_cols and rp2.dtype == rp_t and val2.dtype == dt
    assert np.array_equal(rp2, rp) and np.array_equal(col2, col) and np.array_equal(val2, val)
    with open(f, "rb") as fh:
        hdr = fh.read(64)
    assert hdr[:8] == b"LHPCCSR1" and os.path.getsize(f) % 1 == 0


def test_lcsr_rejects_corrupt(lhpc, tmp_path):
    rp, col, val = _rand_csr(100, 100, 0.1, np.float32, 3)
    f = str(tmp_path / "m.lcsr")
    lhpc.save_csr(f, rp.astype(np.int64), col, val, 100)
    raw = open(f, "rb").read()
    open(f, "wb").write(raw[:-10])  # truncated
    with pytest.raises(lhpc.LhpcError):
        lhpc.load_csr(f)
    open(f, "wb").write(b"NOTACSR!" + raw[8:])  # bad magic
    with pytest.raises(lhpc.LhpcError):
        lhpc.load_csr(f)


def _mm_cases(tmp_path):
    rng = np.random.default_rng(5)
    cases = {}
    A = sp.random(300, 200, density=0.03, format="coo", random_state=rng)
    cases["general_real"] = (A, {})
    S = sp.random(150, 150, density=0.05, format="coo", random_state=rng)
    S = sp.coo_matrix(S + S.T + sp.eye(150))
    cases["symmetric_real"] = (S, {"symmetry": "symmetric"})
    K = sp.random(90, 90, density=0.08, format="coo", random_state=rng)
    K = sp.coo_matrix(sp.triu(K, 1) - sp.triu(K, 1).T)
    cases["skew"] = (K, {"symmetry": "skew-symmetric"})
    I = sp.coo_matrix((rng.integers(-50, 50, 400).astype(np.int64),
                       (rng.integers(0, 120, 400), rng.integers(0, 130, 400))), shape=(120, 130))
    I.sum_duplicates()
    cases["integer"] = (I, {"field": "integer"})
    P = sp.random(64, 80, density=0.1, format="coo", random_state=rng)
    cases["pattern"] = (P, {"field": "pattern"})
    out = {}
    for name, (M, kw) in cases.items():
        path = str(tmp_path / f"{name}.mtx")
        scipy.io.mmwrite(path, M, **kw)
        out[name] = path
    return out


def _sorted_triples(r, c, v):
    o = np.lexsort((c, r))
    return r[o], c[o], v[o]


def test_matrix_market_triples_match_scipy(lhpc, tmp_path):
    for name, path in _mm_cases(tmp_path).items():
        rows, cols, vals, n_rows, n_cols = lhpc.read_matrix_market_coo(path)
        ref = scipy.io.mmread(path).tocoo()
        assert (n_rows, n_cols) == ref.shape, name
        got = _sorted_triples(rows.astype(np.int64), cols.astype(np.int64), vals)
        want = _sorted_triples(ref.row.astype(np.int64), ref.col.astype(np.int64), ref.data.astype(np.float64))
        for a, b in zip(got, want):
            assert np.array_equal(a, b), name


def test_matrix_market_rejects_unsupported(lhpc, tmp_path):
    p = str(tmp_path / "dense.mtx")
    scipy.io.mmwrite(p, np.arange(6.0).reshape(2, 3))  # "array" format
    with pytest.raises(lhpc.LhpcError):
        lhpc.read_matrix_market_coo(p)
    q = str(tmp_path / "bad.mtx")
    open(q, "w").write("%%MatrixMarket matrix coordinate real general\n3 3 1\n4 1 1.0\n")  # row out of range
    with pytest.raises(lhpc.LhpcError):
        lhpc.read_matrix_market_coo(q)


@pytest.mark.gpu
def test_matrix_market_to_csr_on_gpu(lhpc, gpu, tmp_path):
    for name, path in _mm_cases(tmp_path).items():
        ref = scipy.io.mmread(path).tocsr()
        ref.sum_duplicates()
        ref.sort_indices()
        for dt, ldt in ((np.float64, lhpc.F64), (np.float32, lhpc.F32)):
            rp, col, val, n_cols = lhpc.read_matrix_market(path, dtype=ldt)
            assert n_cols == ref.shape[1]
            assert np.array_equal(rp, ref.indptr.astype(np.int64)), name
            assert np.array_equal(col, ref.indices.astype(np.int32)), name
            want = ref.data.astype(np.float64)
            if dt == np.float32:  # values rounded to f32 before assembly; no duplicates in these files
                want = want.astype(np.float32)
            assert np.array_equal(val, want), name
        # the .lcsr round trip of the assembled matrix feeds an SpMV plan
        f = str(tmp_path / f"{name}.lcsr")
        rp, col, val, n_cols = lhpc.read_matrix_market(path)
        lhpc.save_csr(f, rp, col, val, n_cols)
        rp2, col2, val2, nc2 = lhpc.load_csr(f)
        x = np.linspace(-1, 1, nc2)
        with lhpc.SpMVPlan(rp2, col2, val2, nc2) as plan:
            y = plan(x)
        assert np.allclose(y, ref @ x, rtol=1e-12, atol=1e-12)
