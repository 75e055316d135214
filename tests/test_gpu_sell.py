"""SELL (lane per row over 64-row slices; lhpc_spmv_csr.hip k_spmv_sell):
the short-row kernel the 5-point CG Laplacian selects.  It must be
bit-identical to ADAPTIVE on the same matrix — y through lhpc_spmv and
lhpc_spmv_dot, and the fused dot — since with ≤ 8 nonzeros per row ADAPTIVE
adds the same products in the same order; with dyadic values both equal the
oracle exactly.  Selection: automatic for short rows whose padded slices
stream no more bytes than CSR + row_ptr, off with options.spmv_no_sell,
refused (LHPC_ERR_UNSUPPORTED) when forced onto a row of 9 nonzeros."""
import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu
FORCE_SELL, FORCE_ADAPTIVE = 1 << 10, 1 << 5


def _dev(gpu, a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _random_short(n, maxlen, seed, dt, dyadic, minlen=0):
    rng = np.random.default_rng(seed)
    lens = rng.integers(minlen, maxlen + 1, size=n)
    rp = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(lens, out=rp[1:])
    nnz = int(rp[-1])
    col = rng.integers(0, max(n, 1), size=nnz).astype(np.int32)
    if dyadic:
        val = (rng.integers(-8, 9, size=nnz) / 8.0).astype(dt)
    else:
        val = rng.uniform(-1, 1, nnz).astype(dt)
    return rp, col, val


def _run(lhpc, gpu, rp, col, val, n_cols, x, w, flags=0, options=None):
    import torch
    with lhpc.SpMVPlan(rp, col, val, n_cols, flags=flags, options=options) as plan:
        info = plan.info()
        y0 = plan(x)
        y = torch.full_like(y0, float("nan"))
        out = torch.zeros(1, dtype=torch.float64, device=gpu)
        lhpc.spmv_dot(plan, x, y, w, out)
        torch.cuda.synchronize()
    return info, y0, y, out.item()


CASES = [  # (name, n, maxlen, minlen)
    ("n1", 1, 3, 1), ("n63", 63, 8, 0), ("n65", 65, 8, 8), ("n257", 257, 5, 0),
    ("n300001_len0to8", 300_001, 8, 0), ("n100000_len8", 100_000, 8, 8), ("empty_rows", 1000, 2, 0),
    # a last block of ≤ 128 rows whose 4th ADAPTIVE wave holds rows (n % 256 in
    # {4, 7-8, 13-16, 25-32, 49-64, 97-128}): the fused dot must still fold the
    # waves as ADAPTIVE does
    ("n8", 8, 8, 0), ("n50", 50, 8, 0), ("n64", 64, 8, 0), ("n100", 100, 8, 0), ("n120", 120, 8, 0),
    ("n2098", 2098, 8, 0),
]


@pytest.mark.parametrize("dt", [np.float32, np.float64], ids=["f32", "f64"])
@pytest.mark.parametrize("dyadic", [True, False], ids=["dyadic", "uniform"])
@pytest.mark.parametrize("name,n,maxlen,minlen", CASES, ids=[c[0] for c in CASES])
def test_sell_bit_identical_to_adaptive(lhpc, gpu, name, n, maxlen, minlen, dyadic, dt):
    rp, col, val = _random_short(n, maxlen, 0x5E11 + n + maxlen, dt, dyadic, minlen)
    rng = np.random.default_rng(n)
    xh = ((rng.integers(-8, 9, size=n) / 8.0) if dyadic else rng.uniform(-1, 1, n)).astype(dt)
    wh = rng.uniform(-1, 1, n).astype(dt)
    x, w = _dev(gpu, xh), _dev(gpu, wh)
    ia, ya0, ya, da = _run(lhpc, gpu, rp, col, val, n, x, w, FORCE_ADAPTIVE)
    isl, ys0, ys, ds = _run(lhpc, gpu, rp, col, val, n, x, w, FORCE_SELL)
    assert ia["kernel"] == lhpc.KERNEL_ADAPTIVE and isl["kernel"] == lhpc.KERNEL_SELL
    assert isl["n_blocks"] == ia["n_blocks"] == -(-n // 256)
    assert isl["slices"] == -(-n // 64) and isl["slice_width"] <= maxlen
    import torch
    assert torch.equal(ys0, ya0) and torch.equal(ys, ys0) and torch.equal(ya, ya0)
    assert ds == da  # the same partials in the same tree
    if dyadic:
        assert np.array_equal(ys0.cpu().numpy(), S.spmv_oracle(rp, col, val, xh)[1])
    else:
        _, y64, asum = S.spmv_oracle(rp, col, val, xh)
        S.assert_spmv_close(ys0.cpu().numpy(), y64, asum)


@pytest.mark.parametrize("dt", [np.float32, np.float64], ids=["f32", "f64"])
@pytest.mark.parametrize("shape", [(96, 80), (1000, 1), (4096, 3)])
def test_sell_auto_on_laplacian(lhpc, gpu, shape, dt):
    """The 5-point Laplacian (≤ 5 nonzeros per row, x local) selects SELL; the
    option spmv_no_sell keeps ADAPTIVE; both give the same y."""
    import torch
    rp, col, val = S.laplacian_2d(*shape, dtype=dt)
    n = rp.size - 1
    x = _dev(gpu, np.random.default_rng(5).uniform(-1, 1, n).astype(dt))
    w = _dev(gpu, np.random.default_rng(6).uniform(-1, 1, n).astype(dt))
    i0, y0, _, d0 = _run(lhpc, gpu, rp, col, val, n, x, w)
    i1, y1, _, d1 = _run(lhpc, gpu, rp, col, val, n, x, w, options={"spmv_no_sell": 1})
    assert i0["kernel"] == lhpc.KERNEL_SELL and i0["slice_width"] == (5 if min(shape) > 2 else 3)
    assert i1["kernel"] == lhpc.KERNEL_ADAPTIVE
    assert torch.equal(y0, y1) and d0 == d1
    assert i0["device_bytes"] < i1["device_bytes"] + 8 * (n // 64 + 1)  # no row_ptr; padding ≤ row_ptr


def test_sell_selection_rules(lhpc, gpu):
    """Auto keeps ADAPTIVE when padding would stream more than CSR + row_ptr
    (row lengths 0..8 at random: slices 8 wide, mean 4); a forced SELL on a
    row of 9 nonzeros is LHPC_ERR_UNSUPPORTED; a matrix with no nonzeros
    forced to SELL stores zeros."""
    import torch
    n = 5000
    rp, col, val = _random_short(n, 8, 1, np.float32, True)
    with lhpc.SpMVPlan(rp, col, val, n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_ADAPTIVE
    rp, col, val = _random_short(n, 4, 2, np.float32, True, minlen=4)
    with lhpc.SpMVPlan(rp, col, val, n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_SELL
    rp9, col9, val9 = _random_short(n, 9, 3, np.float32, True, minlen=9)
    with pytest.raises(lhpc.LhpcError) as e:
        lhpc.SpMVPlan(rp9, col9, val9, n, flags=FORCE_SELL)
    assert e.value.status == -5
    with lhpc.SpMVPlan(rp9, col9, val9, n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_ADAPTIVE
    rp0 = np.zeros(n + 1, dtype=np.int32)
    with lhpc.SpMVPlan(rp0, np.zeros(0, np.int32), np.zeros(0, np.float32), n, flags=FORCE_SELL) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_SELL and p.info()["slice_width"] == 0
        y = p(torch.ones(n, device=gpu))
        torch.cuda.synchronize()
        assert torch.count_nonzero(y).item() == 0


@pytest.mark.parametrize("dt", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("rp64", [False, True], ids=["rp32", "rp64"])
def test_sell_device_build_matches_host_build(lhpc, gpu, dt, rp64):
    """A SELL plan built on the GPU from device-resident CSR
    (LHPC_PLAN_DEVICE_INPUT: slice offsets from the host copy of row_ptr, a
    scatter kernel for col / val) gives the host-built plan's y bit for bit:
    the Laplacian (auto), random 0–8 rows (forced; padded slices), and a
    matrix whose padding makes auto fall back to ADAPTIVE on both paths."""
    import torch
    cases = [(S.laplacian_2d(300, 77, dtype=dt), 0, lhpc.KERNEL_SELL)]
    rpr, colr, valr = _random_short(70_001, 8, 0xD5, dt, False)
    cases.append(((rpr, colr, valr), FORCE_SELL, lhpc.KERNEL_SELL))
    cases.append(((rpr, colr, valr), 0, lhpc.KERNEL_ADAPTIVE))
    for (rp, col, val), flags, kern in cases:
        rp = rp.astype(np.int64 if rp64 else np.int32)
        n = rp.size - 1
        xh = np.random.default_rng(n).uniform(-1, 1, n).astype(dt)
        x = _dev(gpu, xh)
        with lhpc.SpMVPlan(rp, col, val, n, flags=flags) as ph, \
                lhpc.SpMVPlan(_dev(gpu, rp), _dev(gpu, col), _dev(gpu, val), n, flags=flags) as pd:
            assert ph.info()["kernel"] == pd.info()["kernel"] == kern
            assert ph.info()["slice_width"] == pd.info()["slice_width"]
            yh, yd = ph(x), pd(x)
            torch.cuda.synchronize()
            assert torch.equal(yh, yd)
        _, y64, asum = S.spmv_oracle(rp, col, val, xh)
        S.assert_spmv_close(yd.cpu().numpy(), y64, asum)


def test_sell_host_buffers_and_device_input(lhpc, gpu):
    """Host x/y (staged) and device-resident CSR input build the same SELL plan."""
    import torch
    rp, col, val = S.laplacian_2d(300, 200)
    n = rp.size - 1
    xh = np.random.default_rng(9).uniform(-1, 1, n)
    want = S.spmv_oracle(rp, col, val, xh)
    with lhpc.SpMVPlan(rp, col, val, n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_SELL
        yh = p(xh)
    with lhpc.SpMVPlan(_dev(gpu, rp), _dev(gpu, col), _dev(gpu, val), n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_SELL
        yd = p(_dev(gpu, xh)).cpu().numpy()
    assert np.array_equal(yh, yd)
    S.assert_spmv_close(yh, want[1], want[2])


@pytest.mark.parametrize("max_iter,check_every", [(5000, 8), (5000, 1), (13, 4), (7, 1), (1, 1)])
@pytest.mark.parametrize("dt", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("grid", [(150, 130), (72, 271)], ids=["n19500", "n19512"])  # n % 256 = 44 / 56
def test_cg_sell_matches_adaptive(lhpc, gpu, dt, max_iter, check_every, grid):
    """lhpc_cg_solve on a SELL plan — each iteration's x / p update fused
    into the next iteration's SpMV (sell_cg_step), graph blocks on a side
    stream — and on an ADAPTIVE plan of the same Laplacian (the unfused
    k_cg_xp loop): same iterations, residual and x bit for bit, converged or
    stopped at max_iter (the pending x update of the last iteration).  n % 256
    = 56 puts rows in the last block's 4th ADAPTIVE wave."""
    import torch
    rp, col, val = S.laplacian_2d(*grid, dtype=dt, shift=0.0 if dt == np.float64 else 0.5)
    n = rp.size - 1
    b = _dev(gpu, np.random.default_rng(21).uniform(-1, 1, n).astype(dt))
    tol = 1e-10 if dt == np.float64 else 1e-5
    out = []
    for opts in (None, {"spmv_no_sell": 1}):
        with lhpc.SpMVPlan(rp, col, val, n, options=opts) as plan:
            s = torch.cuda.Stream(gpu)
            with torch.cuda.stream(s):
                out.append((plan.info()["kernel"],) + tuple(lhpc.cg(plan, b, tol=tol, max_iter=max_iter,
                                                                     check_every=check_every, stream=s)))
            s.synchronize()
    (k0, x0, it0, r0), (k1, x1, it1, r1) = out
    assert (k0, k1) == (lhpc.KERNEL_SELL, lhpc.KERNEL_ADAPTIVE)
    assert (it0, r0) == (it1, r1) and torch.equal(x0, x1)


@pytest.mark.parametrize("name", ["spmv_dyadic_f64_4099x3001_rp64.npz", "spmv_rand_f32_n1.npz",
                                  "spmv_rand_f32_n65.npz"])
def test_sell_golden(lhpc, gpu, name):
    """The golden vectors through a forced SELL plan: exact on the dyadic
    fixture, within the SpMV tolerance elsewhere; a fixture with a row over 8
    nonzeros (n65: 15 per row) is refused with LHPC_ERR_UNSUPPORTED."""
    g = S.load_golden(name)
    rp, col, val, x = g["row_ptr"], g["col_idx"], g["val"], g["x"]
    n_cols = int(g["n_cols"])
    if np.diff(rp).max() > 8:
        with pytest.raises(lhpc.LhpcError) as e:
            lhpc.SpMVPlan(rp, col, val, n_cols, flags=FORCE_SELL)
        assert e.value.status == -5
        return
    with lhpc.SpMVPlan(rp, col, val, n_cols, flags=FORCE_SELL) as plan:
        assert plan.info()["kernel"] == lhpc.KERNEL_SELL
        y = plan(_dev(gpu, x)).cpu().numpy()
    if "dyadic" in name:
        assert np.array_equal(y, g["y_exact"].astype(val.dtype))
    else:
        S.assert_spmv_close(y, g["y_exact"], S.spmv_oracle(rp, col, val, x)[2])


def test_sell_full_size_cg_config(lhpc, gpu):
    """The bench's CG configuration at full size (4096² 5-point Laplacian,
    fp64, n = 16.8M): the SELL plan's y equals ADAPTIVE's bit for bit and
    10⁵ sampled rows match fp64 numpy; 20 CG iterations (tol 0, graph blocks
    of 10) through the fused SELL loop and the unfused ADAPTIVE loop give the
    same x bit for bit."""
    import torch
    nx = 4096
    rp, col, val = lhpc.gen_laplacian_2d(nx, nx, lhpc.F64)
    n = nx * nx
    xh = np.random.default_rng(0xC6).uniform(-1, 1, n)
    x = _dev(gpu, xh)
    b = _dev(gpu, np.random.default_rng(0xC7).uniform(-1, 1, n))
    out = []
    for opts in (None, {"spmv_no_sell": 1}):
        with lhpc.SpMVPlan(rp, col, val, n, options=opts) as plan:
            y = plan(x)
            s = torch.cuda.Stream(gpu)
            with torch.cuda.stream(s):
                xs, it, res = lhpc.cg(plan, b, tol=0.0, max_iter=20, check_every=10, stream=s)
            s.synchronize()
            out.append((plan.info()["kernel"], y, xs, it, res))
    (k0, y0, x0, it0, r0), (k1, y1, x1, it1, r1) = out
    assert (k0, k1) == (lhpc.KERNEL_SELL, lhpc.KERNEL_ADAPTIVE)
    assert torch.equal(y0, y1)
    rows, y64, asum = S.sampled_rows_fp64(rp, col, val, xh, 100_000)
    yr = y0.cpu().numpy()[rows]
    assert np.all(np.abs(yr - y64) <= 1e-12 * asum + 1e-300)
    assert (it0, r0) == (it1, r1) == (20, r0) and torch.equal(x0, x1)
