"""GPU parity for CSR SpMV through the C ABI (include/lhpc.h) — every kernel
family against the exact-arithmetic golden fixtures and the CPU oracle.

Bars (north_star): index handling bit-exact — dyadic-valued inputs make every
summation order exact, so y must equal the reference bit-for-bit; random
fp inputs within |dy| <= 1e-6 * sum|a*x| per row (tests/_support.py).
SpMV parity is "unpinned by the reference" (the reference has no SpMV, SURVEY
§0): the anchor is exact arithmetic (Fractions) and the fp64 oracle.
"""
import glob
import os

import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu

FAMILIES = {
    "auto": 0,
    "rowgroup": 1 << 4,
    "adaptive": 1 << 5,
    "xslice": 1 << 6,
    "xslice_fast": (1 << 6) | (1 << 7),  # fp32 partials (the fp32 default), separate reduce kernel
    "xslice_exact": (1 << 6) | (1 << 8),  # fp64 partials
    "xtile": 1 << 9,  # x tiles in LDS: tile gather + merge-path chunk reduce
}
GOLDEN_SPMV = sorted(glob.glob(os.path.join(S.GOLDEN, "spmv_*.npz")))


def _run(lhpc, gpu, rp, col, val, x, n_cols, flags, device_buffers=True, options=None):
    import torch
    with lhpc.SpMVPlan(rp, col, val, n_cols, flags=flags, options=options) as plan:
        if device_buffers:
            xd = torch.from_numpy(x).to(gpu)
            y = plan(xd).cpu().numpy()
        else:
            y = plan(x)
        info = plan.info()
    return y, info


@pytest.mark.parametrize("family", list(FAMILIES))
@pytest.mark.parametrize("path", GOLDEN_SPMV, ids=lambda p: os.path.basename(p)[5:-4])
def test_golden(lhpc, gpu, path, family):
    g = S.load_golden(os.path.basename(path))
    rp, col, val, x = g["row_ptr"], g["col_idx"], g["val"], g["x"]
    n_cols = int(g["n_cols"])
    y, info = _run(lhpc, gpu, rp, col, val, x, n_cols, FAMILIES[family])
    if family.startswith("xslice") and rp[-1] > 0:
        assert info["kernel"] == lhpc.KERNEL_XSLICE  # long rows: uint16 lens + wave-reduced rows
    if family == "xtile":
        assert info["kernel"] == lhpc.KERNEL_XTILE
    exact = g["y_exact"]
    if "dyadic" in path:
        assert np.array_equal(y, exact.astype(val.dtype)), "dyadic SpMV must be bit-exact"
    else:
        _, _, asum = S.spmv_oracle(rp, col, val, x)
        S.assert_spmv_close(y, exact, asum)


@pytest.mark.parametrize("family", ["auto", "xslice", "xtile"])
def test_host_buffers_match_device(lhpc, gpu, family):
    g = S.load_golden("spmv_dyadic_f32_n1000.npz")
    args = (g["row_ptr"], g["col_idx"], g["val"], g["x"], int(g["n_cols"]), FAMILIES[family])
    yd, _ = _run(lhpc, gpu, *args, device_buffers=True)
    yh, _ = _run(lhpc, gpu, *args, device_buffers=False)
    assert np.array_equal(yd, yh)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 1000, 4099])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("family", list(FAMILIES))
def test_edge_sizes_vs_oracle(lhpc, gpu, n, dtype, family):
    dt = lhpc.F32 if dtype == "f32" else lhpc.F64
    per = min(n, 15)
    for dist in (0, 1):
        rp, col, val = lhpc.gen_uniform_csr(n, n, per, dtype=dt, dist=dist, seed=0xE000 + n)
        x = lhpc.gen_values(dt, dist, n, 0xE100 + n)
        y, _ = _run(lhpc, gpu, rp, col, val, x, n, FAMILIES[family])
        y64, yr, asum = S.spmv_oracle(rp, col, val, x)
        if dist == 1:
            assert np.array_equal(y, yr)
        else:
            S.assert_spmv_close(y, y64, asum)


def test_empty_matrix_and_zero_rows(lhpc, gpu):
    import torch
    rp = np.zeros(11, dtype=np.int32)
    col = np.zeros(0, dtype=np.int32)
    val = np.zeros(0, dtype=np.float32)
    x = np.ones(7, dtype=np.float32)
    for flags in FAMILIES.values():
        y, _ = _run(lhpc, gpu, rp, col, val, x, 7, flags)
        assert np.array_equal(y, np.zeros(10, dtype=np.float32))
    with lhpc.SpMVPlan(np.zeros(1, dtype=np.int32), col, val, 7) as plan:
        out = plan(torch.ones(7, device=gpu))
        assert out.numel() == 0


@pytest.mark.parametrize("family", list(FAMILIES))
def test_powerlaw_vs_oracle(lhpc, gpu, family):
    n = 200_000
    rp, col, val = lhpc.gen_powerlaw_csr(n, n, lmax=10_000, dtype=lhpc.F32, seed=0xE200)
    x = lhpc.gen_values(lhpc.F32, 0, n, 0xE201)
    y, info = _run(lhpc, gpu, rp, col, val, x, n, FAMILIES[family])
    y64, _, asum = S.spmv_oracle(rp, col, val, x)
    S.assert_spmv_close(y, y64, asum)


def test_c1_config_vs_oracle(lhpc, gpu):
    """BASELINE configs[0] shape (n=1e5, nnz=1e6, fp64) on the GPU."""
    n = 100_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 10, dtype=lhpc.F64)
    x = lhpc.gen_values(lhpc.F64, 0, n, lhpc.SEED_X)
    y, _ = _run(lhpc, gpu, rp, col, val, x, n, 0)
    y64, _, asum = S.spmv_oracle(rp, col, val, x)
    S.assert_spmv_close(y, y64, asum)


@pytest.mark.slow
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_full_size_c2_c3(lhpc, gpu, dtype):
    """BASELINE configs[1]/[2] shape: n=10M, 15/row (nnz=150M) against the
    oracle on every row, plus the dyadic twin bit-exact, plus exact
    linearity A(2x) = 2·A(x) and run-to-run determinism."""
    import torch
    dt = lhpc.F32 if dtype == "f32" else lhpc.F64
    n = 10_000_000
    for dist in (0, 1):
        rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=dt, dist=dist)
        x = lhpc.gen_values(dt, dist, n, lhpc.SEED_X)
        with lhpc.SpMVPlan(rp, col, val, n) as plan:
            assert plan.info()["kernel"] == lhpc.KERNEL_XTILE
            # cache-sized ranges over one xg ring (gather + reduce each):
            # fp32 600 MB of xg → three; fp64 1.2 GB → six (round 6)
            assert plan.info()["launches"] == (6 if dtype == "f32" else 12)
            xd = torch.from_numpy(x).to(gpu)
            y1 = plan(xd).clone()
            y2 = plan(xd).clone()
            y2x = plan(xd * 2)
            torch.cuda.synchronize()
            assert torch.equal(y1, y2), "SpMV must be deterministic run to run"
            assert torch.equal(y2x, y1 * 2), "A(2x) must equal 2·A(x) exactly"
            y = y1.cpu().numpy()
        y64, yr, asum = S.spmv_oracle(rp, col, val, x)
        if dist == 1:
            assert np.array_equal(y, yr)
        else:
            S.assert_spmv_close(y, y64, asum)
        del rp, col, val


@pytest.mark.slow
@pytest.mark.parametrize("blocks", [0, 1])
def test_xtile_large_n_80m(lhpc, gpu, blocks):
    """XTILE beyond C2: n = 80M rows and columns, 15 uniform nonzeros per row
    (nnz = 1.2e9, fp32).  blocks = 1: one plan over 2048 x tiles (146K chunks;
    the dense segment table of starts needed 2.9e8 entries and the plan fell to
    XSLICE until the two-level table, lhpc_plan.hpp xtile_segment_table);
    blocks = 0 (auto): three column blocks of ≈ 683 tiles each, the later ones
    adding into y.  Dyadic values: 10^5 sampled rows bit-exact against fp64 numpy
    (exact here), and run to run determinism on the whole y."""
    import torch
    n = 80_000_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=lhpc.F32, dist=1, seed=0x8000)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0x8001)
    with lhpc.SpMVPlan(rp, col, val, n, options={"xtile_col_blocks": blocks}) as plan:
        info = plan.info()
        # tiles of ≤ 40960 columns (narrowed to a whole multiple of the CUs: 2048 × 39063)
        assert info["kernel"] == lhpc.KERNEL_XTILE and info["slice_width"] <= 40960
        if blocks == 1:
            assert info["slices"] == -(-n // info["slice_width"]) and info["slices"] >= -(-n // 40960)
        else:  # slices: the first block's tiles — B = ⌈2048 / 768⌉ = 3 blocks of ≤ 768
            cols = n // 3 // 64 * 64
            assert info["slices"] == -(-cols // info["slice_width"]) and info["slices"] <= 768
        xd = torch.from_numpy(x).to(gpu)
        y1 = plan(xd).clone()
        y2 = plan(xd)
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)
        y = y1.cpu().numpy()
        del xd, y1, y2
    rows, y64, _ = S.sampled_rows_fp64(rp, col, val, x, 100_000)
    assert np.array_equal(y[rows].astype(np.float64), y64)


@pytest.mark.parametrize("n_cols,dtype,tiles", [(19_040_000, "f32", 465), (20_000_000, "f32", 512),
                                                (30_000_000, "f32", 768), (45_000_000, "f32", 550),
                                                (15_000_000, "f64", 733)])
def test_xtile_reduce_forms_wide_x(lhpc, gpu, n_cols, dtype, tiles, xt_layout):
    """The reduce forms picked by the tile count (lhpc_spmv_xtile.hip
    xtile_g): 200K rows × 15 uniform nonzeros over an x of n_cols columns.
    fp32: 465 tiles (G = 1, row offsets in LDS, 4 blocks per CU; too few to
    be widened to 512), 512 (20M columns widened to a multiple of the CUs;
    G = 1 by count, moved to the G = 2 register form by the LDS budget), 768
    (G = 2), 45M columns as two column blocks of 550 tiles (G = 2, the second
    adding into y); fp64 733 tiles (G = 1, BLK 1024) — each over the three
    reduce layouts (perm, iperm, iperm over aligned segments).  Small nnz, so
    the whole y is checked: dyadic values, bit-exact against the oracle."""
    import torch
    dt = lhpc.F32 if dtype == "f32" else lhpc.F64
    n = 200_000
    rp, col, val = lhpc.gen_uniform_csr(n, n_cols, 15, dtype=dt, dist=1, seed=0x7100 + n_cols % 977)
    x = lhpc.gen_values(dt, 1, n_cols, 0x7101)
    with lhpc.SpMVPlan(rp, col, val, n_cols, options=xt_layout) as plan:
        info = plan.info()
        assert info["kernel"] == lhpc.KERNEL_XTILE and info["slices"] == tiles, info
        y = plan(torch.from_numpy(x).to(gpu)).cpu().numpy()
    assert np.array_equal(y, S.spmv_oracle(rp, col, val, x)[1])


@pytest.mark.slow
@pytest.mark.parametrize("n,tiles", [(20_000_000, (476, 512)), (30_000_000, (513, 1024))])
def test_xtile_register_row_offsets(lhpc, gpu, n, tiles):
    """The fp32 reduce's G = 2 form keeps a chunk's row offsets in registers
    (lhpc_spmv_xtile.hip xt_rreg): n = 30M runs it for its 733 tiles; n = 20M
    (489 tiles, G = 1 by count) is moved onto it because the LDS row-offset
    array would cost a block per CU (xtile_g).  15 uniform nonzeros per row,
    dyadic values: 10^5 sampled rows bit-exact against fp64 numpy, and run to
    run determinism on the whole y."""
    import torch
    rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=lhpc.F32, dist=1, seed=0x7000)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0x7001)
    with lhpc.SpMVPlan(rp, col, val, n) as plan:
        info = plan.info()
        assert info["kernel"] == lhpc.KERNEL_XTILE and tiles[0] <= info["slices"] <= tiles[1]
        xd = torch.from_numpy(x).to(gpu)
        y1 = plan(xd).clone()
        y2 = plan(xd)
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)
        y = y1.cpu().numpy()
        del xd, y1, y2
    rows, y64, _ = S.sampled_rows_fp64(rp, col, val, x, 100_000)
    assert np.array_equal(y[rows].astype(np.float64), y64)


@pytest.mark.slow
@pytest.mark.parametrize("dtype", ["f32", "f64"])
def test_full_size_c4(lhpc, gpu, dtype):
    """BASELINE configs[3] (C4) at full size, as bench.py --workload c4 builds
    it: n = 10M power-law rows (l in [1, 10^4], three rows forced to 10^4
    before the seeded row shuffle), through the default plan (XTILE + chunk fix-ups), against the
    oracle on every row; the dyadic twin bit-exact; fp32 and fp64 (§8d)."""
    import torch
    dt = lhpc.F32 if dtype == "f32" else lhpc.F64
    n = 10_000_000
    for dist in (0, 1):
        rp, col, val = lhpc.gen_powerlaw_csr(n, n, dtype=dt, dist=dist)
        lens = np.diff(rp)
        assert lens.max() == 10_000 and np.count_nonzero(lens == 10_000) >= 3  # forced rows, then shuffled
        x = lhpc.gen_values(dt, dist, n, lhpc.SEED_X)
        with lhpc.SpMVPlan(rp, col, val, n) as plan:
            info = plan.info()
            assert info["kernel"] == lhpc.KERNEL_XTILE and info["n_long_rows"] > 0
            # three (fp32) / six (fp64) cache-sized ranges + the fix-up
            assert info["launches"] == (7 if dtype == "f32" else 13)
            y = plan(torch.from_numpy(x).to(gpu)).cpu().numpy()
        y64, yr, asum = S.spmv_oracle(rp, col, val, x)
        if dist == 1:
            assert np.array_equal(y, yr)
        else:
            S.assert_spmv_close(y, y64, asum)
        del rp, col, val


@pytest.mark.slow
@pytest.mark.parametrize("wl", ["c2", "c3"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_split_plans_at_rank_sizes(lhpc, gpu, wl, world):
    """The N > 1 bench path at full C2 / C3 size: for world N and K = 2
    chunks per rank, the first and the last rank's row-range plan
    (InterleavedBlocks.local_csr_all → stage → range per chunk) reproduce the
    oracle's rows of that rank's blocks — bit-exact on the dyadic twin,
    within the fp bar on random values."""
    import torch
    from libhpc_amd.dist import InterleavedBlocks
    dt = lhpc.F32 if wl == "c2" else lhpc.F64
    n, K = 10_000_000, 2
    for dist in (0, 1):
        rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=dt, dist=dist)
        x = lhpc.gen_values(dt, dist, n, lhpc.SEED_X)
        xd = torch.from_numpy(x).to(gpu)
        y64, yr, asum = S.spmv_oracle(rp, col, val, x)
        ib = InterleavedBlocks(n, world, K)
        for rank in (0, world - 1):
            lrp, lc, lv, splits = ib.local_csr_all(rp, col, val, rank)
            with lhpc.SpMVPlan(lrp, lc, lv, n, splits=splits) as plan:
                assert plan.info()["kernel"] == lhpc.KERNEL_XTILE
                ys = [torch.empty(ib.B, dtype=xd.dtype, device=gpu) for _ in range(K)]
                plan.stage(xd)
                for k in range(K):
                    plan.range(k, ys[k])
                got = [t.cpu().numpy() for t in ys]
            for k in range(K):
                r0, r1 = ib.rows(rank, k)
                g = got[k][:r1 - r0]
                assert np.all(got[k][r1 - r0:] == 0)  # padded empty rows
                if dist == 1:
                    assert np.array_equal(g, yr[r0:r1]), (wl, world, rank, k)
                else:
                    S.assert_spmv_close(g, y64[r0:r1], asum[r0:r1])
        del rp, col, val


def test_partitioned_blocks_concatenate_bit_exact(lhpc, gpu):
    """Row-block split used by multi-GPU runs: per-block plans (rebased row_ptr,
    global columns) concatenate to exactly the unpartitioned y."""
    import torch
    n = 300_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 15, dtype=lhpc.F32)
    x = lhpc.gen_values(lhpc.F32, 0, n, lhpc.SEED_X)
    xd = torch.from_numpy(x).to(gpu)
    with lhpc.SpMVPlan(rp, col, val, n, flags=FAMILIES["rowgroup"]) as plan:
        y_full = plan(xd).cpu().numpy()
    cuts = lhpc.csr_partition_rows(rp, 4)
    parts = []
    for p in range(4):
        r0, r1 = int(cuts[p]), int(cuts[p + 1])
        lrp = (rp[r0:r1 + 1] - rp[r0]).astype(np.int32)
        with lhpc.SpMVPlan(lrp, col[rp[r0]:rp[r1]], val[rp[r0]:rp[r1]], n,
                           flags=FAMILIES["rowgroup"]) as plan:
            parts.append(plan(xd).cpu().numpy())
    assert np.array_equal(np.concatenate(parts), y_full)


def test_interleaved_chunk_plans_on_gpu(lhpc, gpu):
    """The multi-GPU data path at world=1: K interleaved chunk plans (padded
    local CSR blocks, as bench.py --gpus N builds them) assemble to exactly
    the single-plan y."""
    import torch
    from libhpc_amd.dist import DistSpMVOverlap, InterleavedBlocks
    n = 250_003
    rp, col, val = lhpc.gen_powerlaw_csr(n, n, lmax=3000, dtype=lhpc.F32, seed=0xE300)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0xE301)
    xd = torch.from_numpy(x).to(gpu)
    with lhpc.SpMVPlan(rp, col, val, n) as plan:
        y_ref = plan(xd).cpu().numpy()
    ib = InterleavedBlocks(n, 1, 3)
    plans = [lhpc.SpMVPlan(*ib.local_csr(rp, col, val, 0, k), n) for k in range(3)]
    d = DistSpMVOverlap(ib, [lambda xv, yv, p=p: p(xv, yv) for p in plans], like=xd)
    y = d.step(xd).cpu().numpy()
    for p in plans:
        p.close()
    assert np.array_equal(y, y_ref)


# ------------------------------------------------------------------ XTILE
def test_wave_scan_dpp(lhpc, gpu):
    """lhpc::wave_incl_scan (DPP row shifts + row_bcast, used by the XTILE
    reduce) equals a shuffle scan in every wave."""
    import ctypes as C
    import torch
    P = C.CDLL(os.path.join(os.path.dirname(lhpc.LIB_PATH), "liblhpc_probe.so"))
    rng = np.random.default_rng(0xA0)
    n = 256 * 37 + 5
    a = torch.from_numpy(rng.integers(-1000, 1000, size=n).astype(np.int32)).to(gpu)
    d = torch.empty_like(a)
    r = torch.empty_like(a)
    st = P.lhpc_probe_wave_scan(C.c_void_p(a.data_ptr()), C.c_void_p(d.data_ptr()),
                                C.c_void_p(r.data_ptr()), C.c_int64(n),
                                C.c_void_p(torch.cuda.current_stream(gpu).cuda_stream))
    assert st == 0
    torch.cuda.synchronize()
    host = a.cpu().numpy().astype(np.int64)
    exp = np.concatenate([np.cumsum(host[i:i + 64]) for i in range(0, n, 64)])
    assert np.array_equal(r.cpu().numpy(), exp)
    assert np.array_equal(d.cpu().numpy(), exp)


def _csr_from_lengths(lengths, n_cols, seed, dyadic):
    """CSR with the given row lengths, distinct sorted uniform columns per row."""
    rng = np.random.default_rng(seed)
    lengths = np.asarray(lengths, dtype=np.int64)
    rp = np.zeros(len(lengths) + 1, dtype=np.int32)
    np.cumsum(lengths, out=rp[1:])
    cols = []
    for ln in lengths:
        if ln:
            cols.append(np.sort(rng.choice(n_cols, size=int(ln), replace=False)).astype(np.int32))
    col = np.concatenate(cols) if cols else np.zeros(0, dtype=np.int32)
    if dyadic:
        val = (rng.integers(-8, 9, size=col.size) / 8.0)
    else:
        val = rng.uniform(-1.0, 1.0, size=col.size)
    return rp, col, val


@pytest.fixture(params=["perm", "iperm", "iperm_aligned"])
def xt_layout(request):
    """The XTILE reduce index streams: perm (xg scattered into CSR slots) and
    iperm (xg kept in flat order in LDS, each CSR position's x gathered
    through a CSR-order index), pinned through lhpc_options.xtile_reduce;
    iperm_aligned: iperm over aligned segments (every (tile, chunk) segment
    padded to 16 B, loaded in 16-B units; lhpc_options.xtile_align).
    Returns the options dict the test extends."""
    if request.param == "iperm_aligned":
        return {"xtile_reduce": 2, "xtile_align": 2}
    return {"xtile_reduce": 2 if request.param == "iperm" else 1, "xtile_align": 1}


def _check_xtile(lhpc, gpu, lengths, n_cols, dtype, seed, dyadic=True, expect_cont=None, opts=None):
    rp, col, val = _csr_from_lengths(lengths, n_cols, seed, dyadic)
    val = val.astype(dtype)
    rng = np.random.default_rng(seed + 1)
    if dyadic:
        x = (rng.integers(-8, 9, size=n_cols) / 8.0).astype(dtype)
    else:
        x = rng.uniform(-1.0, 1.0, size=n_cols).astype(dtype)
    y, info = _run(lhpc, gpu, rp, col, val, x, n_cols, FAMILIES["xtile"], options=opts)
    assert info["kernel"] == lhpc.KERNEL_XTILE
    if expect_cont is not None:
        assert (info["n_long_rows"] > 0) == expect_cont
    y64, yr, asum = S.spmv_oracle(rp, col, val, x)
    if dyadic:
        assert np.array_equal(y, yr), "dyadic XTILE SpMV must be bit-exact"
    else:
        S.assert_spmv_close(y, y64, asum)
    return info


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_long_rows_across_chunks(lhpc, gpu, dtype, xt_layout):
    """Rows longer than a chunk (4096 nonzeros) are cut by chunk ends and
    finished by the fix-up: a 30k-row, rows of 5000/4096/4095/9000 between
    short rows, a long first and a long last row."""
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 3000 + [0, 0] + [30000]
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA100, expect_cont=True, opts=xt_layout)
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA101, dyadic=False, opts=xt_layout)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_empty_row_runs(lhpc, gpu, dtype, xt_layout):
    """More than Rmax (1024) consecutive empty rows, leading and trailing
    empty rows, and an all-empty tail after the last nonzero."""
    lengths = [0] * 3000 + [7] * 10 + [0] * 2500 + [1] + [0] * 1500 + [4096] + [0] * 2049
    _check_xtile(lhpc, gpu, lengths, 150_000, dtype, 0xA200, opts=xt_layout)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_wide_many_tiles(lhpc, gpu, dtype, xt_layout):
    """n_cols ≫ n_rows: hundreds of tiles, a ragged last tile, 1-nonzero rows."""
    rng = np.random.default_rng(0xA300)
    lengths = rng.integers(0, 40, size=5000)
    _check_xtile(lhpc, gpu, lengths, 9_000_001, dtype, 0xA301, opts=xt_layout)
    _check_xtile(lhpc, gpu, np.ones(70_000, dtype=np.int64), 3_000_017, dtype, 0xA302, opts=xt_layout)


def test_xtile_small_gather_pieces(lhpc, gpu, xt_layout):
    """Several gather workgroups per tile (piece bounds inside a tile) give the same bits."""
    opts = dict(xt_layout, xtile_piece=1000)
    rng = np.random.default_rng(0xA400)
    lengths = rng.integers(0, 60, size=20_000)
    _check_xtile(lhpc, gpu, lengths, 100_000, np.float32, 0xA401, opts=opts)
    for u in (2, 4, 16):  # gather steps in flight (default 8)
        opts["xtile_steps"] = u
        _check_xtile(lhpc, gpu, lengths, 100_000, np.float64, 0xA402, opts=opts)
        _check_xtile(lhpc, gpu, lengths, 100_000, np.float32, 0xA403, opts=opts)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_nt_gather_stores(lhpc, gpu, dtype, xt_layout):
    """Non-temporal xg stores in the gather (options.xtile_store = STORE_NT)
    give the same bits, with full and partial 64-group store blocks and cut rows."""
    opts = dict(xt_layout, xtile_store=lhpc.STORE_NT)
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 3000 + [0, 0] + [30000]
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA500, expect_cont=True, opts=opts)
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA501, dyadic=False, opts=opts)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("range_pieces", [False, True])
def test_xtile_split_ranges(lhpc, gpu, dtype, xt_layout, range_pieces):
    """Row-range plan (lhpc_spmv_plan_create_split): stage once, reduce each
    range into its own buffer; long rows end at and start right after the
    split rows; the concatenation equals the whole-matrix oracle bit for bit
    (dyadic) and lhpc_spmv on the same plan gives the same bits.
    range_pieces: per-range gather pieces (a plan whose xg exceeds the
    Infinity Cache): stage gathers every range's pieces, lhpc_spmv runs
    gather k / reduce k."""
    import torch
    opts = dict(xt_layout, xtile_ranges=2 if range_pieces else 0)
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 30000 + [0, 0] + [30000]
    n_cols = 200_000
    rp, col, val = _csr_from_lengths(lengths, n_cols, 0xA700, dyadic=True)
    val = val.astype(dtype)
    rng = np.random.default_rng(0xA701)
    x = (rng.integers(-8, 9, size=n_cols) / 8.0).astype(dtype)
    n = len(lengths)
    splits = [1, 51, 57, 20000, n - 1]  # after the long first row, around the long rows, before the last
    with lhpc.SpMVPlan(rp, col, val, n_cols, flags=FAMILIES["xtile"], splits=splits, options=opts) as plan:
        assert plan.info()["kernel"] == lhpc.KERNEL_XTILE
        xd = torch.from_numpy(x).to(gpu)
        bounds = [0] + splits + [n]
        ys = [torch.full((bounds[k + 1] - bounds[k],), float("nan"), dtype=xd.dtype, device=gpu)
              for k in range(len(bounds) - 1)]
        for _ in range(2):  # twice: carries from the previous call must not leak
            plan.stage(xd)
            for k, yk in enumerate(ys):
                plan.range(k, yk)
        y = torch.cat(ys).cpu().numpy()
        yfull = plan(xd).cpu().numpy()
    _, yr, _ = S.spmv_oracle(rp, col, val, x)
    assert np.array_equal(y, yr)
    assert np.array_equal(yfull, yr)


@pytest.mark.parametrize("ranges", [2, 3, 5])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_cache_ranges(lhpc, gpu, dtype, ranges, xt_layout):
    """Cache-sized ranges (options.xtile_ranges = K, the default for large fp32
    plans): gather k and reduce k in turn over K nnz-balanced row ranges,
    each range's gather pieces rounded up to 8-entry bounds inside a tile (its
    first ≤ 7 entries come from the previous range's gather), one fix-up for
    every range's cut rows.  Long rows crossing chunks, a tiny piece size (so
    ranges hold several pieces per tile), two calls in a row; bit-exact."""
    import torch
    opts = dict(xt_layout, xtile_ranges=ranges)
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 30000 + [0, 0] + [30000]
    n_cols = 200_000
    rp, col, val = _csr_from_lengths(lengths, n_cols, 0xA900 + ranges, dyadic=True)
    val = val.astype(dtype)
    rng = np.random.default_rng(0xA9F0 + ranges)
    x = (rng.integers(-8, 9, size=n_cols) / 8.0).astype(dtype)
    _, yr, _ = S.spmv_oracle(rp, col, val, x)
    for piece in (0, 1000):
        opts["xtile_range_piece"] = piece
        with lhpc.SpMVPlan(rp, col, val, n_cols, flags=FAMILIES["xtile"], options=opts) as plan:
            info = plan.info()
            assert info["kernel"] == lhpc.KERNEL_XTILE
            assert info["launches"] == 2 * ranges + (1 if info["n_long_rows"] else 0)
            xd = torch.from_numpy(x).to(gpu)
            for _ in range(2):  # carries from the previous call must not leak
                y = plan(xd).cpu().numpy()
                assert np.array_equal(y, yr)


@pytest.mark.parametrize("ranges", [2, 3, 5])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_xg_ring(lhpc, gpu, dtype, ranges):
    """The xg ring of cache-sized ranges (round 6, options.xtile_ring auto):
    one range-sized xg buffer that every range's gather rewrites, each
    range's part of each tile at its own ring offset, the 8-entry groups two
    ranges share gathered by both.  Bit-identical to the one-slot-per-entry
    layout (xtile_ring = 1) and to the oracle — dyadic and uniform values,
    tiny gather pieces (many pieces per (range, tile)), two calls in a row —
    with less HBM held; a ring plan refuses lhpc_spmv_stage."""
    import torch
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 30000 + [0, 0] + [30000]
    n_cols = 200_000
    for dyadic in (True, False):
        rp, col, val = _csr_from_lengths(lengths, n_cols, 0xB100 + ranges, dyadic=dyadic)
        val = val.astype(dtype)
        rng = np.random.default_rng(0xB1F0 + ranges)
        x = ((rng.integers(-8, 9, size=n_cols) / 8.0) if dyadic else rng.uniform(-1, 1, n_cols)).astype(dtype)
        xd = torch.from_numpy(x).to(gpu)
        _, yr, asum = S.spmv_oracle(rp, col, val, x)
        for piece in (0, 200):
            ys, nbytes = [], []
            for ring_off in (0, 1):
                opts = {"xtile_reduce": 2, "xtile_ranges": ranges, "xtile_range_piece": piece, "xtile_ring": ring_off}
                with lhpc.SpMVPlan(rp, col, val, n_cols, flags=FAMILIES["xtile"], options=opts) as plan:
                    info = plan.info()
                    assert info["kernel"] == lhpc.KERNEL_XTILE
                    nbytes.append(info["device_bytes"])
                    for _ in range(2):
                        y = plan(xd)
                    ys.append(y.cpu().numpy())
                    if ring_off == 0:
                        with pytest.raises(lhpc.LhpcError) as e:
                            plan.stage(xd)
                        assert e.value.status == -5
            assert np.array_equal(ys[0], ys[1]), (dyadic, piece)
            if dyadic:
                assert np.array_equal(ys[0], yr)
            else:
                S.assert_spmv_close(ys[0], yr, asum)
            nnz = int(col.size)
            assert nbytes[0] < nbytes[1] - (ranges - 1) / ranges * 0.9 * nnz * val.itemsize


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_xg_ring_user_ranges(lhpc, gpu, dtype):
    """options.xtile_ring = 2: a plan with user row ranges whose ranges are
    gathered one by one (forced here by xtile_ranges) shares one xg ring
    across them, as the per-rank plans of lhpc_dist_spmv do.  A whole call is
    bit-identical to the one-slot-per-entry plan (xtile_ring = 1) and to the
    oracle, twice in a row, user ranges without nonzeros included; the ring plan
    refuses lhpc_spmv_stage and lhpc_spmv_range."""
    import torch
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 30000 + [0, 0] + [30000]
    n_cols = 200_000
    rp, col, val = _csr_from_lengths(lengths, n_cols, 0xB300, dyadic=True)
    val = val.astype(dtype)
    x = (np.random.default_rng(0xB301).integers(-8, 9, size=n_cols) / 8.0).astype(dtype)
    xd = torch.from_numpy(x).to(gpu)
    _, yr, _ = S.spmv_oracle(rp, col, val, x)
    splits = [55, 56, 9000, 30057, 30059]  # rows 55 and 30057-30058: ranges with no nonzeros
    ys, nbytes = [], []
    for ring in (2, 1):
        opts = {"xtile_reduce": 2, "xtile_ranges": 2, "xtile_ring": ring}
        with lhpc.SpMVPlan(rp, col, val, n_cols, flags=FAMILIES["xtile"], options=opts, splits=splits) as plan:
            info = plan.info()
            assert info["kernel"] == lhpc.KERNEL_XTILE
            nbytes.append(info["device_bytes"])
            for _ in range(2):
                y = plan(xd)
            ys.append(y.cpu().numpy())
            if ring == 2:
                with pytest.raises(lhpc.LhpcError) as e:
                    plan.stage(xd)
                assert e.value.status == -5
    assert np.array_equal(ys[0], ys[1])
    assert np.array_equal(ys[0], yr)
    assert nbytes[0] < nbytes[1] - 0.3 * int(col.size) * val.itemsize, nbytes


def test_split_plan_unsupported_without_xtile(lhpc, gpu):
    """A matrix that does not select XTILE (small x) refuses a row-range plan."""
    rp, col, val = _csr_from_lengths([5] * 1000, 1000, 0xA800, dyadic=True)
    with pytest.raises(lhpc.LhpcError):
        lhpc.SpMVPlan(rp, col, val.astype(np.float32), 1000, splits=[500])


def test_xtile_is_auto_choice_without_locality(lhpc, gpu):
    """x > 8 MB with uniform random columns selects XTILE; options.spmv_no_xtile gives XSLICE."""
    n = 3_000_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 4, dtype=lhpc.F32, dist=1, seed=0xA500)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0xA501)
    y, info = _run(lhpc, gpu, rp, col, val, x, n, 0)
    assert info["kernel"] == lhpc.KERNEL_XTILE
    assert info["launches"] in (2, 3)
    _, yr, _ = S.spmv_oracle(rp, col, val, x)
    assert np.array_equal(y, yr)
    y2, info2 = _run(lhpc, gpu, rp, col, val, x, n, 0, options={"spmv_no_xtile": 1})
    assert info2["kernel"] == lhpc.KERNEL_XSLICE
    assert np.array_equal(y2, yr)


@pytest.mark.parametrize("lanes,rows", [(4, 4), (16, 8), (64, 1)])
def test_rowgroup_shape_option(lhpc, gpu, lanes, rows):
    """options.rowgroup_lanes/rows pin the ROWGROUP shape (same bits on
    dyadic inputs); a shape the library does not instantiate is refused."""
    rp, col, val = lhpc.gen_powerlaw_csr(20_000, 20_000, lmax=300, dtype=lhpc.F32, dist=1, seed=0xA600)
    x = lhpc.gen_values(lhpc.F32, 1, 20_000, 0xA601)
    y, info = _run(lhpc, gpu, rp, col, val, x, 20_000, FAMILIES["rowgroup"],
                   options={"rowgroup_lanes": lanes, "rowgroup_rows": rows})
    assert info["lanes_per_row"] == lanes and info["rows_per_group"] == rows
    _, yr, _ = S.spmv_oracle(rp, col, val, x)
    assert np.array_equal(y, yr)
    with pytest.raises(lhpc.LhpcError):
        lhpc.SpMVPlan(rp, col, val, 20_000, flags=FAMILIES["rowgroup"],
                      options={"rowgroup_lanes": 8, "rowgroup_rows": 8})


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("cap", [40_000, 100_003])
def test_xtile_row_parts(lhpc, gpu, dtype, cap, xt_layout):
    """XTILE row parts (lhpc_options.xtile_part_nnz): the plan cuts the rows
    into nnz-balanced parts of ≤ cap nonzeros, one XTILE plan each, run in
    turn on the same x — the path a matrix takes when its tile stream
    outgrows the int32 offsets (nnz + 8·tiles ≥ 2^31), here forced at small
    size.  Long rows (up to 30000 nonzeros, i.e. most of a part) and empty
    rows sit next to the cuts.  Dyadic: bit-exact; random: within the bound;
    the host-buffer path too.  More launches than a single plan."""
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 3000 + [0, 0] + [30000] + [7] * 4000
    opts = dict(xt_layout, xtile_part_nnz=cap)
    info = _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA900, opts=opts)
    single = _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA900, opts=xt_layout)
    assert info["launches"] > single["launches"]
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xA901, dyadic=False, opts=opts)
    rp, col, val = _csr_from_lengths(lengths, 200_000, 0xA902, True)
    val = val.astype(dtype)
    x = (np.random.default_rng(7).integers(-8, 9, size=200_000) / 8.0).astype(dtype)
    yh, _ = _run(lhpc, gpu, rp, col, val, x, 200_000, FAMILIES["xtile"], device_buffers=False, options=opts)
    assert np.array_equal(yh, S.spmv_oracle(rp, col, val, x)[1])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("blocks", [2, 3, 5])
def test_xtile_col_blocks(lhpc, gpu, dtype, blocks, xt_layout):
    """XTILE column blocks (lhpc_options.xtile_col_blocks): the plan cuts the
    columns into B blocks, one XTILE plan each over x's column range, run in
    turn, every block after the first adding into y — the path a matrix takes
    when x spans many tiles (lhpc_spmv.hip xtile_col_blocks_for), here forced
    at small size.  Long rows cut by chunk ends (the fix-up adds under the
    accumulation), empty rows, short rows with no entry in some blocks.
    Dyadic: bit-exact; random: within the bound; with row parts on top; the
    host-buffer path; a y full of NaN beforehand does not leak through."""
    import torch
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 3000 + [0, 0] + [30000] + [7] * 4000
    opts = dict(xt_layout, xtile_col_blocks=blocks)
    info = _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xAB00, opts=opts)
    single = _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xAB00, opts=dict(xt_layout, xtile_col_blocks=1))
    assert info["launches"] > single["launches"]
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xAB01, dyadic=False, opts=opts)
    _check_xtile(lhpc, gpu, lengths, 200_000, dtype, 0xAB02, opts=dict(opts, xtile_part_nnz=40_000))
    rp, col, val = _csr_from_lengths(lengths, 200_000, 0xAB03, True)
    val = val.astype(dtype)
    x = (np.random.default_rng(9).integers(-8, 9, size=200_000) / 8.0).astype(dtype)
    yr = S.spmv_oracle(rp, col, val, x)[1]
    yh, _ = _run(lhpc, gpu, rp, col, val, x, 200_000, FAMILIES["xtile"], device_buffers=False, options=opts)
    assert np.array_equal(yh, yr)
    with lhpc.SpMVPlan(rp, col, val, 200_000, flags=FAMILIES["xtile"], options=opts) as plan:
        y = torch.full((len(lengths),), float("nan"), dtype=torch.from_numpy(x).dtype, device=gpu)
        plan(torch.from_numpy(x).to(gpu), y)
        assert np.array_equal(y.cpu().numpy(), yr)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("lo,hi", [(0, 60_000), (120_000, 200_000), (0, 200_000)])
def test_xtile_col_blocks_empty_blocks(lhpc, gpu, dtype, lo, hi):
    """Column blocks with no nonzeros are left out, and the first non-empty
    block stores every row (columns only in the first 30% / the last 40% of
    x, four blocks of 50000 columns; the full range as the control)."""
    rng = np.random.default_rng(0xAC00 + lo)
    lengths = rng.integers(0, 40, size=5000)
    rp = np.zeros(lengths.size + 1, dtype=np.int32)
    np.cumsum(lengths, out=rp[1:])
    col = np.concatenate([np.sort(rng.choice(np.arange(lo, hi), size=int(n), replace=False)) for n in lengths])
    col = col.astype(np.int32)
    val = (rng.integers(-8, 9, size=col.size) / 8.0).astype(dtype)
    x = (rng.integers(-8, 9, size=200_000) / 8.0).astype(dtype)
    y, info = _run(lhpc, gpu, rp, col, val, x, 200_000, FAMILIES["xtile"], options={"xtile_col_blocks": 4})
    assert info["kernel"] == lhpc.KERNEL_XTILE
    assert np.array_equal(y, S.spmv_oracle(rp, col, val, x)[1])


@pytest.mark.parametrize("dtype,blocks", [(np.float32, 2), (np.float64, 3)])
def test_xtile_col_blocks_auto(lhpc, gpu, dtype, blocks):
    """The automatic choice: x of 40M columns (977 fp32 / 1954 fp64 tiles,
    past the 768 one block keeps) with 100 nonzeros per row gives 2 (fp32) /
    3 (fp64) column blocks — as many launches as that many single plans, and
    the same y as one block, bit for bit on dyadic values."""
    import torch
    n_cols, n_rows = 40_000_000, 300
    rng = np.random.default_rng(0xAD00)
    rp = np.arange(0, 100 * (n_rows + 1), 100, dtype=np.int32)
    col = np.concatenate([np.sort(rng.choice(n_cols, size=100, replace=False)) for _ in range(n_rows)]).astype(np.int32)
    val = (rng.integers(-8, 9, size=col.size) / 8.0).astype(dtype)
    x = torch.from_numpy((rng.integers(-8, 9, size=n_cols) / 8.0).astype(dtype)).to(gpu)
    with lhpc.SpMVPlan(rp, col, val, n_cols) as auto, \
            lhpc.SpMVPlan(rp, col, val, n_cols, options={"xtile_col_blocks": 1}) as one:
        ia, i1 = auto.info(), one.info()
        assert ia["kernel"] == i1["kernel"] == lhpc.KERNEL_XTILE
        assert ia["launches"] == blocks * i1["launches"]
        ya, y1 = auto(x).cpu().numpy(), one(x).cpu().numpy()
    assert np.array_equal(ya, y1)
    assert np.array_equal(ya, S.spmv_oracle(rp, col, val, x.cpu().numpy())[1])


def test_xtile_row_parts_row_past_cap(lhpc, gpu):
    """A single row longer than the part cap cannot be cut into parts: the
    plan leaves XTILE (as the int32 limit did before parts existed) and the
    result is still exact."""
    lengths = [3] * 100 + [50_000] + [3] * 100
    rp, col, val = _csr_from_lengths(lengths, 100_000, 0xAA00, True)
    val = val.astype(np.float32)
    x = (np.random.default_rng(8).integers(-8, 9, size=100_000) / 8.0).astype(np.float32)
    y, info = _run(lhpc, gpu, rp, col, val, x, 100_000, FAMILIES["xtile"], options={"xtile_part_nnz": 10_000})
    assert info["kernel"] != lhpc.KERNEL_XTILE
    assert np.array_equal(y, S.spmv_oracle(rp, col, val, x)[1])


@pytest.mark.slow
def test_xtile_parts_past_int32(lhpc, gpu):
    """Past the int32 tile stream: n = 20M rows and columns, 108 uniform
    nonzeros per row (nnz = 2.16e9 > 2^31, int64 row_ptr, fp32, dyadic
    values).  Before row parts this plan fell to XSLICE; now it stays XTILE
    (two row parts over the same 512 tiles).  10^5 sampled rows bit-exact
    against fp64 numpy (exact on dyadic data), the whole y equal run to run,
    and GFLOP/s printed (per part the same kernels and segment lengths as
    C2, so C2-level rates are expected)."""
    import torch
    n, per_row = 20_000_000, 108
    rp, col, val = lhpc.gen_uniform_csr(n, n, per_row, dtype=lhpc.F32, dist=1, seed=0x15000)
    assert rp.dtype == np.int64 and int(rp[-1]) > 2**31
    x = lhpc.gen_values(lhpc.F32, 1, n, 0x15001)
    with lhpc.SpMVPlan(rp, col, val, n) as plan:
        info = plan.info()
        assert info["kernel"] == lhpc.KERNEL_XTILE and info["nnz"] == per_row * n
        xd = torch.from_numpy(x).to(gpu)
        y1 = plan(xd).clone()
        y2 = plan(xd)
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(5):
            plan(xd, y2)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / 5
        print(f"\nXTILE row parts, nnz {per_row * n}: {ms:.3f} ms/call, {2 * per_row * n / ms / 1e6:.1f} GFLOP/s, "
              f"launches {info['launches']}")
        y = y1.cpu().numpy()
        del xd, y1, y2
    rows, y64, _ = S.sampled_rows_fp64(rp, col, val, x, 100_000)
    assert np.array_equal(y[rows].astype(np.float64), y64)


@pytest.mark.slow
def test_xslice_dispatch_past_2p32_work_items(lhpc, gpu):
    """A dispatch holds < 2^32 work-items: the XSLICE stream kernel's logical
    grid (slices × 64-row chunks, 256 threads each) passes that at S · n >
    2^32 (S = 256 slices, n = 17M rows here; C2 at n = 80M is 64 · 80M), and
    the kernel strides over its logical blocks.  Before the stride the
    truncated dispatch left rows unwritten (bench --n 80000000 with XSLICE
    failed its sampled check).  Dyadic values: 10^5 sampled rows exact."""
    import torch
    n = 17_000_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 2, dtype=lhpc.F32, dist=1, seed=0x17000)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0x17001)
    with lhpc.SpMVPlan(rp, col, val, n, flags=FAMILIES["xslice"], options={"xslice_slices": 256}) as plan:
        info = plan.info()
        assert info["kernel"] == lhpc.KERNEL_XSLICE and info["slices"] * n > 2**32
        y = plan(torch.from_numpy(x).to(gpu)).cpu().numpy()
    rows, y64, _ = S.sampled_rows_fp64(rp, col, val, x, 100_000)
    assert np.array_equal(y[rows].astype(np.float64), y64)


def _digests_host_vs_device(lhpc, gpu, rp, col, val, n_cols, flags=0, options=None, splits=None):
    import torch
    kw = dict(flags=flags, options=options, splits=splits)
    # the host build (options.xtile_host_build) against the device builds:
    # from device arrays, and from host arrays uploaded by the library
    with lhpc.SpMVPlan(rp, col, val, n_cols, flags=flags, splits=splits,
                       options=dict(options or {}, xtile_host_build=1)) as ph:
        dh, ih = ph.layout_digest(), ph.info()
    with lhpc.SpMVPlan(rp, col, val, n_cols, **kw) as pu:
        assert pu.layout_digest() == dh and pu.info() == ih
    drp, dcol, dval = (torch.from_numpy(np.ascontiguousarray(a)).to(gpu) for a in (rp, col, val))
    with lhpc.SpMVPlan(drp, dcol, dval, n_cols, **kw) as pd:
        dd, idev = pd.layout_digest(), pd.info()
        if splits is None:
            x = (np.random.default_rng(5).integers(-8, 9, size=n_cols) / 8.0).astype(val.dtype)
            y = pd(torch.from_numpy(x).to(gpu)).cpu().numpy()
            assert np.array_equal(y, S.spmv_oracle(rp, col, val, x)[1])
    assert ih == idev
    return dh, dd


@pytest.mark.parametrize("case", ["uniform_f32", "uniform_f64", "powerlaw_f32", "perm_f32", "ranges_f32",
                                  "splits_f64", "rp64_f32", "colblocks_f32", "powerlaw_colblocks_f64",
                                  "parts_f32", "parts_colblocks_f32"])
def test_device_input_layout_matches_host(lhpc, gpu, case):
    """LHPC_PLAN_DEVICE_INPUT: an XTILE plan built on the GPU from device
    row_ptr / col_idx / val (k_xt_counts → host offsets → k_xt_scatter →
    k_xt_permute_blocks) has the host build's layout byte for byte (FNV-1a
    digests of row_ptr, col16, perm/iperm, val runs, chunk descriptors, cr,
    the segment table, the gather pieces and cont), the same plan info, and
    gives the oracle's y bit for bit (dyadic).  Cases: uniform fp32 / fp64
    (iperm reduce), power-law rows crossing chunks (cont, fix-up), the perm
    reduce, cache-sized ranges (per-range pieces), a row-range split plan
    (fp64), int64 row_ptr input, and plans of parts built part by part on the
    GPU (column blocks cut by k_colblock_count / k_colblock_scatter, row
    parts, both), whose digests fold the parts' in order."""
    n = 3_000_000
    dt = lhpc.F64 if "f64" in case else lhpc.F32
    if case.startswith("powerlaw"):
        rp, col, val = lhpc.gen_powerlaw_csr(n, n, lmax=5000, dtype=dt, dist=1, seed=0xDE00)
    else:
        rp, col, val = lhpc.gen_uniform_csr(n, n, 7, dtype=dt, dist=1, seed=0xDE01, narrow=case != "rp64_f32")
    opts, splits = None, None
    if case == "perm_f32":
        opts = {"xtile_reduce": lhpc.XTILE_REDUCE_PERM}
    elif case == "ranges_f32":
        opts = {"xtile_ranges": 3}
    elif case == "splits_f64":
        splits = [n // 3, n // 2 + 7]
    elif case == "colblocks_f32":
        opts = {"xtile_col_blocks": 3}
    elif case == "powerlaw_colblocks_f64":
        opts = {"xtile_col_blocks": 2}
    elif case == "parts_f32":
        opts = {"xtile_part_nnz": 8_000_000}
    elif case == "parts_colblocks_f32":
        opts = {"xtile_part_nnz": 6_000_000, "xtile_col_blocks": 2}
    if case == "rp64_f32":
        assert rp.dtype == np.int64
    dh, dd = _digests_host_vs_device(lhpc, gpu, rp, col, val, n, options=opts, splits=splits)
    assert dh == dd, [i for i, (a, b) in enumerate(zip(dh, dd)) if a != b]


def test_device_input_checks_and_fallbacks(lhpc, gpu):
    """Device input that does not select XTILE (x fits L2: SELL here) goes
    through the host path and is exact; malformed device CSR is refused on
    the GPU with LHPC_ERR_BAD_CSR (a column out of range, a decreasing
    row_ptr)."""
    import torch
    n = 50_000
    rp, col, val = lhpc.gen_uniform_csr(n, n, 5, dtype=lhpc.F32, dist=1, seed=0xDE10)
    x = lhpc.gen_values(lhpc.F32, 1, n, 0xDE11)
    dev = [torch.from_numpy(np.ascontiguousarray(a)).to(gpu) for a in (rp, col, val)]
    with lhpc.SpMVPlan(*dev, n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_SELL  # 5 nonzeros per row: SELL (test_gpu_sell.py)
        assert np.array_equal(p(torch.from_numpy(x).to(gpu)).cpu().numpy(), S.spmv_oracle(rp, col, val, x)[1])
    bad_col = dev[1].clone()
    bad_col[123] = n
    with pytest.raises(lhpc.LhpcError) as e:
        lhpc.SpMVPlan(dev[0], bad_col, dev[2], n)
    assert e.value.status == -2
    bad_rp = dev[0].clone()
    bad_rp[7] = bad_rp[9] + 1
    with pytest.raises(lhpc.LhpcError) as e:
        lhpc.SpMVPlan(bad_rp, dev[1], dev[2], n)
    assert e.value.status == -2


def test_coo_to_csr_to_spmv_stays_on_device(lhpc, gpu):
    """SURVEY §8f chain without a host round trip for A: COO triples on the
    device → lhpc_coo_to_csr (GPU radix sort) → device CSR → an XTILE plan
    built on the GPU from it (LHPC_PLAN_DEVICE_INPUT) → y = A·x, against the
    oracle on the same triples (dyadic, duplicates summed)."""
    import torch
    n, m = 2_500_000, 12_000_000
    rng = np.random.default_rng(0xDE20)
    r = rng.integers(0, n, m).astype(np.int32)
    c = rng.integers(0, n, m).astype(np.int32)
    v = (rng.integers(-8, 9, m) / 8.0).astype(np.float32)
    want_rp, want_col, want_val = S.coo_oracle(n, n, r, c, v)
    rp, col, val = lhpc.coo_to_csr(n, n, *(torch.from_numpy(a).to(gpu) for a in (r, c, v)), row_ptr_bits=32)
    with lhpc.SpMVPlan(rp, col, val, n) as p:
        assert p.info()["kernel"] == lhpc.KERNEL_XTILE
        x = lhpc.gen_values(lhpc.F32, 1, n, 0xDE21)
        y = p(torch.from_numpy(x).to(gpu)).cpu().numpy()
    assert np.array_equal(y, S.spmv_oracle(want_rp, want_col, want_val, x)[1])


@pytest.mark.parametrize("ranges", [1, 3])
@pytest.mark.parametrize("tiles", [3, 256])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_xtile_phase_tables(lhpc, gpu, dtype, ranges, tiles):
    """The iperm reduce from the plan's per-chunk phase-A tables
    (options.xtile_pretable = 2: batch rank terms and segment bases copied to
    LDS by LDS-DMA instead of the segment scan) gives the scanning reduce's y
    bit for bit and the oracle's on dyadic data — one range and three ring
    ranges, long rows across chunks and empty rows, 3 and 256 tiles."""
    import torch
    lengths = [20000] + [3] * 50 + [5000, 4096, 4095, 1, 0, 9000] + [15] * 30000 + [0, 0] + [30000]
    n_cols = (40960 if dtype == np.float32 else 20480) * tiles - 7
    for dyadic in (True, False):
        rp, col, val = _csr_from_lengths(lengths, n_cols, 0xB500 + tiles, dyadic=dyadic)
        val = val.astype(dtype)
        rng = np.random.default_rng(0xB5F0)
        x = ((rng.integers(-8, 9, size=n_cols) / 8.0) if dyadic else rng.uniform(-1, 1, n_cols)).astype(dtype)
        xd = torch.from_numpy(x).to(gpu)
        ys = []
        for pre in (2, 1):
            opts = {"xtile_reduce": 2, "xtile_ranges": ranges, "xtile_pretable": pre}
            with lhpc.SpMVPlan(rp, col, val, n_cols, flags=FAMILIES["xtile"], options=opts) as plan:
                assert plan.info()["kernel"] == lhpc.KERNEL_XTILE
                for _ in range(2):
                    y = plan(xd)
                ys.append(y.cpu().numpy())
        assert np.array_equal(ys[0], ys[1]), dyadic
        _, yr, asum = S.spmv_oracle(rp, col, val, x)
        if dyadic:
            assert np.array_equal(ys[0], yr)
        else:
            S.assert_spmv_close(ys[0], yr, asum)
