"""The fp64 CG restatement (oracle.c:oracle_cg_f64) against a dense solve
(no reference counterpart, so the solution of A·x = b is
the pin).  No GPU."""
import numpy as np
import scipy.sparse as sp

from tests import _support as S


def test_oracle_cg_solves_laplacian():
    rp, col, val = S.laplacian_2d(30, 20)
    n = rp.size - 1
    b = np.random.default_rng(1).uniform(-1, 1, n)
    x, it, res = S.cg_oracle(rp, col, val, b, tol=1e-12, max_iter=2000)
    A = sp.csr_matrix((val, col, rp), shape=(n, n)).toarray()
    want = np.linalg.solve(A, b)
    assert res <= 1e-12 and it < 2000
    assert np.linalg.norm(x - want) <= 1e-9 * np.linalg.norm(want)


def test_oracle_cg_zero_rhs_and_warm_start():
    rp, col, val = S.laplacian_2d(8, 8)
    x, it, res = S.cg_oracle(rp, col, val, np.zeros(64))
    assert it == 0 and np.all(x == 0)
    b = np.linspace(-1, 1, 64)
    x1, it1, _ = S.cg_oracle(rp, col, val, b, tol=1e-13)
    x2, it2, _ = S.cg_oracle(rp, col, val, b, x0=x1, tol=1e-10)
    assert it2 <= 1 and np.allclose(x2, x1, rtol=0, atol=1e-12)
