"""GPU conjugate gradient (lhpc_cg_solve and its building blocks; SURVEY §8f
rank 3) against the fp64 CG restatement in oracle/oracle.c.

Tolerances (floating point: the GPU sums dots in a different fixed order):
fp64 — same iteration count ±1 and ‖x_gpu − x_oracle‖ ≤ 1e-8·‖x_oracle‖ at
tol 1e-10; fp32 vectors — converged to tol 1e-5 and within 1e-4 of the fp64
solution.  Building blocks: fp64 dots within 1e-12 relative of numpy."""
import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu


def _dev(gpu, a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


@pytest.mark.parametrize("shape", [(64, 48), (200, 150), (7, 1)])
@pytest.mark.parametrize("flags", [0, 1 << 4, 1 << 6])
def test_cg_fp64_matches_oracle(lhpc, gpu, shape, flags):
    rp, col, val = S.laplacian_2d(*shape)
    n = rp.size - 1
    b = np.random.default_rng(n).uniform(-1, 1, n)
    want, it_o, res_o = S.cg_oracle(rp, col, val, b, tol=1e-10, max_iter=5000)
    with lhpc.SpMVPlan(rp, col, val, n, flags=flags) as plan:
        x, it, res = lhpc.cg(plan, _dev(gpu, b), tol=1e-10, max_iter=5000)
    x = x.cpu().numpy()
    assert abs(it - it_o) <= 1 and res <= 1e-10
    assert np.linalg.norm(x - want) <= 1e-8 * np.linalg.norm(want)


def test_cg_fp32(lhpc, gpu):
    rp, col, val = S.laplacian_2d(128, 128, dtype=np.float32, shift=0.5)
    n = rp.size - 1
    b = np.random.default_rng(3).uniform(-1, 1, n).astype(np.float32)
    want, _, _ = S.cg_oracle(rp, col, val, b.astype(np.float64), tol=1e-12, max_iter=5000)
    with lhpc.SpMVPlan(rp, col, val, n) as plan:
        x, it, res = lhpc.cg(plan, _dev(gpu, b), tol=1e-5, max_iter=5000, check_every=5)
    assert res <= 1e-5 and it % 5 == 0
    x = x.cpu().numpy().astype(np.float64)
    assert np.linalg.norm(x - want) <= 1e-4 * np.linalg.norm(want)


@pytest.mark.parametrize("check_every,max_iter", [(4, 5000), (7, 5000), (6, 20), (5, 3)])
def test_cg_graph_blocks_match_loop(lhpc, gpu, check_every, max_iter):
    """On a non-null stream lhpc_cg_solve replays the check_every iterations
    between two convergence checks as a captured HIP graph (ADAPTIVE / SELL plans);
    on the null stream it runs the plain loop.  Both issue the same kernels in
    the same order: x bit-identical, same iteration count and residual — for
    even and odd check_every (both graph parities), a max_iter that ends in
    the middle of a block (the tail runs the loop), and one too short for
    any block; then the fp64 oracle's tolerance."""
    import torch
    rp, col, val = S.laplacian_2d(96, 80)
    n = rp.size - 1
    b = _dev(gpu, np.random.default_rng(17).uniform(-1, 1, n))
    with lhpc.SpMVPlan(rp, col, val, n) as plan:
        assert plan.info()["kernel"] == lhpc.KERNEL_SELL  # ≤ 5 nonzeros per row (test_gpu_sell.py)
        x0, it0, r0 = lhpc.cg(plan, b, tol=1e-10, max_iter=max_iter, check_every=check_every,
                              stream=torch.cuda.default_stream(gpu))
        s = torch.cuda.Stream(gpu)
        with torch.cuda.stream(s):
            x1, it1, r1 = lhpc.cg(plan, b, tol=1e-10, max_iter=max_iter, check_every=check_every, stream=s)
            x2, it2, r2 = lhpc.cg(plan, b, tol=1e-10, max_iter=max_iter, check_every=check_every, stream=s)
        s.synchronize()
    assert (it0, r0) == (it1, r1) == (it2, r2)
    assert torch.equal(x0, x1) and torch.equal(x1, x2)
    if max_iter == 5000:
        want, it_o, _ = S.cg_oracle(rp, col, val, b.cpu().numpy(), tol=1e-10, max_iter=5000)
        assert it0 - check_every <= it_o <= it0 and it0 % check_every == 0
        assert np.linalg.norm(x0.cpu().numpy() - want) <= 1e-8 * np.linalg.norm(want)


def test_cg_warm_start_and_zero_rhs(lhpc, gpu):
    import torch
    rp, col, val = S.laplacian_2d(32, 32)
    n = rp.size - 1
    with lhpc.SpMVPlan(rp, col, val, n) as plan:
        x, it, res = lhpc.cg(plan, torch.zeros(n, dtype=torch.float64, device=gpu))
        assert it == 0 and res == 0.0 and torch.count_nonzero(x) == 0
        b = _dev(gpu, np.linspace(-1, 1, n))
        x1, it1, _ = lhpc.cg(plan, b, tol=1e-12)
        x2, it2, _ = lhpc.cg(plan, b, x=x1.clone(), tol=1e-10)
        assert it2 <= 1 and torch.allclose(x2, x1, rtol=0, atol=1e-11)


def test_cg_breakdown_reported(lhpc, gpu):
    """[[0,1],[1,0]] with b = e0: p·Ap = 0 on the first step → non-finite → error."""
    rp = np.array([0, 1, 2], np.int32)
    col = np.array([1, 0], np.int32)
    val = np.array([1.0, 1.0])
    with lhpc.SpMVPlan(rp, col, val, 2) as plan:
        with pytest.raises(lhpc.LhpcError):
            lhpc.cg(plan, _dev(gpu, np.array([1.0, 0.0])))


def test_cg_building_blocks(lhpc, gpu):
    import torch
    rng = np.random.default_rng(7)
    n = 1_000_003
    for dt in (np.float64, np.float32):
        a, b, x, p, r, q = (rng.uniform(-1, 1, n).astype(dt) for _ in range(6))
        out = torch.zeros(1, dtype=torch.float64, device=gpu)
        lhpc.vec_dot(_dev(gpu, a), _dev(gpu, b), out)
        want = float(np.dot(a.astype(np.float64), b.astype(np.float64)))
        assert abs(out.item() - want) <= 1e-12 * np.abs(a.astype(np.float64) * b).sum()
        num = torch.tensor([0.75], dtype=torch.float64, device=gpu)
        den = torch.tensor([1.5], dtype=torch.float64, device=gpu)
        xd, pd, rd, qd = (_dev(gpu, v) for v in (x, p, r, q))
        rr = torch.zeros(1, dtype=torch.float64, device=gpu)
        lhpc.cg_step_xr(num, den, xd, pd, rd, qd, rr)
        al = dt(0.5)
        xw = (x + al * p).astype(dt)
        rw = (r - al * q).astype(dt)
        assert np.array_equal(xd.cpu().numpy(), xw) and np.array_equal(rd.cpu().numpy(), rw)
        assert abs(rr.item() - float(np.dot(rw.astype(np.float64), rw))) <= 1e-12 * n
        lhpc.cg_step_p(num, den, rd, pd)
        assert np.array_equal(pd.cpu().numpy(), (rw + al * p).astype(dt))


def test_cg_fused_steps_match_separate(lhpc, gpu):
    """lhpc_cg_step_r + lhpc_cg_step_xp (the solver's fused pair) leave x, r,
    p and r·r bit-identical to lhpc_cg_step_xr + lhpc_cg_step_p; β = NULL
    updates x only."""
    import torch
    rng = np.random.default_rng(8)
    n = 777_777
    for dt in (np.float64, np.float32):
        x, p, r, q = (rng.uniform(-1, 1, n).astype(dt) for _ in range(4))
        an = torch.tensor([0.3], dtype=torch.float64, device=gpu)
        ad = torch.tensor([1.7], dtype=torch.float64, device=gpu)
        bd_ = torch.tensor([2.9], dtype=torch.float64, device=gpu)
        x1, p1, r1, q1 = (_dev(gpu, v) for v in (x, p, r, q))
        x2, p2, r2, q2 = (_dev(gpu, v) for v in (x, p, r, q))
        rr1 = torch.zeros(1, dtype=torch.float64, device=gpu)
        rr2 = torch.zeros(1, dtype=torch.float64, device=gpu)
        lhpc.cg_step_xr(an, ad, x1, p1, r1, q1, rr1)
        lhpc.cg_step_p(rr1, bd_, r1, p1)
        lhpc.cg_step_r(an, ad, r2, q2, rr2)
        lhpc.cg_step_xp(an, ad, rr2, bd_, x2, p2, r2)
        for u, v in ((x1, x2), (p1, p2), (r1, r2), (rr1, rr2)):
            assert torch.equal(u, v)
        x3, p3 = _dev(gpu, x), _dev(gpu, p)
        lhpc.cg_step_xp(an, ad, None, None, x3, p3, None)
        al = dt(0.3 / 1.7)
        assert np.array_equal(x3.cpu().numpy(), (x + al * p).astype(dt)) and np.array_equal(p3.cpu().numpy(), p)


def test_dist_cg_hip_ops_world1(lhpc, gpu):
    """The multi-GPU solver's data path at world 1 (HipOps, padded block plan)
    converges to the same solution as lhpc_cg_solve."""
    import torch
    from libhpc_amd.dist import DistCG, HipOps, InterleavedBlocks
    rp, col, val = S.laplacian_2d(100, 70)
    n = rp.size - 1
    b = np.random.default_rng(11).uniform(-1, 1, n)
    ib = InterleavedBlocks(n, 1, 1)
    lrp, lc, lv = ib.local_csr(rp, col, val, 0, 0)
    with lhpc.SpMVPlan(lrp, lc, lv, n) as plan, lhpc.SpMVPlan(rp, col, val, n) as full:
        bd = torch.zeros(ib.B, dtype=torch.float64, device=gpu)
        bd[:n] = _dev(gpu, b)
        x = torch.zeros_like(bd)
        solver = DistCG(ib, 0, lambda pf, qb: plan(pf, qb), HipOps(), like=bd,
                        local_spmv_dot=lambda pf, qb, wb, out: lhpc.spmv_dot(plan, pf, qb, wb, out))
        x, it, res = solver.solve(bd, x, tol=1e-10, max_iter=3000)
        x1, it1, res1 = lhpc.cg(full, _dev(gpu, b), tol=1e-10, max_iter=3000)
    assert abs(it - it1) <= 1 and res <= 1e-10
    assert torch.linalg.norm(x[:n] - x1) <= 1e-8 * torch.linalg.norm(x1)


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("maxlen", [0, 1, 5, 9])
def test_adaptive_short_rows(lhpc, gpu, dt, maxlen):
    """ADAPTIVE blocks of short rows (≤ 256 rows of ≤ 2048 nonzeros per
    block, lhpc_spmv_csr.hip csr_build_blocks; 512-row blocks measured slower,
    DESIGN.md §4): rows of 0..maxlen nonzeros (maxlen 0: an all-empty
    matrix), dyadic values, y bit-exact against the oracle through lhpc_spmv
    and lhpc_spmv_dot, and the fused dot within 1e-12·Σ|w·y| of numpy on the
    stored y."""
    import torch
    n = 300_001
    rng = np.random.default_rng(0xAD + maxlen)
    lens = rng.integers(0, maxlen + 1, size=n)
    rp = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(lens, out=rp[1:])
    nnz = int(rp[-1])
    col = rng.integers(0, n, size=nnz).astype(np.int32)
    val = (rng.integers(-8, 9, size=nnz) / 8.0).astype(dt)
    xh = (rng.integers(-8, 9, size=n) / 8.0).astype(dt)
    wh = (rng.integers(-8, 9, size=n) / 4.0).astype(dt)
    want = S.spmv_oracle(rp, col, val, xh)[1]
    x, w = _dev(gpu, xh), _dev(gpu, wh)
    with lhpc.SpMVPlan(rp, col, val, n, flags=lhpc.PLAN_FORCE_ADAPTIVE) as plan:
        info = plan.info()
        assert info["kernel"] == lhpc.KERNEL_ADAPTIVE
        if maxlen and maxlen <= 5:  # ≤ 2048 / 256 nonzeros per row on average: 256-row blocks
            assert info["n_blocks"] == -(-n // 256)
        y0 = plan(x)
        y = torch.full_like(y0, float("nan"))
        out = torch.zeros(1, dtype=torch.float64, device=gpu)
        lhpc.spmv_dot(plan, x, y, w, out)
        torch.cuda.synchronize()
        assert torch.equal(y, y0)
        yh = y.cpu().numpy()
        assert np.array_equal(yh, want)
        yw = yh.astype(np.float64) * wh.astype(np.float64)
        assert abs(out.item() - yw.sum()) <= 1e-12 * max(np.abs(yw).sum(), 1e-300)


@pytest.mark.parametrize("flags", [0, 1 << 4, 1 << 6])
@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_spmv_dot(lhpc, gpu, flags, dt):
    """lhpc_spmv_dot: y bit-identical to lhpc_spmv (same kernel), w·y within
    1e-12·Σ|w·y| of numpy (fused ADAPTIVE epilogue, or SpMV + dot for the
    other families); long rows (> 2048 nnz) take the one-row block path."""
    import torch
    rp, col, val = lhpc.gen_powerlaw_csr(60_000, 60_000, lmax=5000, dtype=lhpc.F64 if dt == np.float64 else lhpc.F32,
                                         seed=0x5D07)
    n = rp.size - 1
    x = _dev(gpu, np.random.default_rng(1).uniform(-1, 1, n).astype(dt))
    w = _dev(gpu, np.random.default_rng(2).uniform(-1, 1, n).astype(dt))
    with lhpc.SpMVPlan(rp, col, val, n, flags=flags) as plan:
        y0 = plan(x)
        y = torch.empty_like(y0)
        out = torch.zeros(1, dtype=torch.float64, device=gpu)
        lhpc.spmv_dot(plan, x, y, w, out)
        assert torch.equal(y, y0)
        yw = y.cpu().numpy().astype(np.float64) * w.cpu().numpy().astype(np.float64)
        assert abs(out.item() - yw.sum()) <= 1e-12 * np.abs(yw).sum()


def test_cg_concurrent_solve_on_one_plan_is_refused(lhpc, gpu):
    """the solve's work (vectors, scalars, captured graphs)
    belongs to the plan, so a second solve on the same plan while one runs
    returns LHPC_ERR_BUSY (-7) instead of racing on it; a solve after the
    first one ended runs normally, and the first solve's x is unaffected."""
    import threading
    import time
    import torch
    ny = nx = 1024  # ≈ 0.2 ms per iteration: 3000 iterations keep the first solve busy for ≫ 0.1 s
    rp, col, val = S.laplacian_2d(ny, nx)
    b = np.random.default_rng(0xC6).uniform(-1, 1, ny * nx)
    with lhpc.SpMVPlan(rp, col, val, ny * nx) as plan:
        bd = _dev(gpu, b)
        ref, it_ref, _ = lhpc.cg(plan, bd, tol=0.0, max_iter=300, check_every=10)
        ref = ref.cpu().numpy()
        out, started = {}, threading.Event()

        def long_solve():
            started.set()
            out["long"] = lhpc.cg(plan, bd, tol=0.0, max_iter=3000, check_every=10)
        t = threading.Thread(target=long_solve)
        t.start()
        started.wait()
        time.sleep(0.1)
        busy = None
        try:
            lhpc.cg(plan, bd, tol=0.0, max_iter=10, check_every=10)
        except lhpc.LhpcError as e:
            busy = e.status
        t.join()
        assert "long" in out and busy == -7, (busy, "long" in out)
        x2, it2, _ = lhpc.cg(plan, bd, tol=0.0, max_iter=300, check_every=10)  # the plan is free again
        assert it2 == it_ref and np.array_equal(x2.cpu().numpy(), ref)
