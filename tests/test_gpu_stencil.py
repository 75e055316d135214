"""GPU parity for the ghost-cell stencils through the C ABI.

blur_x / blur_y must be BIT-EXACT against (a) the golden fixtures produced by
the reference's own HPCHighDimensionFlatArray + BM_x_blur/BM_y_blur loop
(oracle/_ref/ref_probe, tests/golden/make_golden.py) and (b) the C oracle at
other shapes, up to the reference's 8192² grid.  stencil7 is bit-exact
against the oracle (both evaluate the same order without contraction).
"""
import glob
import os

import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu

GOLDEN_BLUR = sorted(glob.glob(os.path.join(S.GOLDEN, "blur_*.npz")))


def _dev(gpu, a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


@pytest.mark.parametrize("buffers", ["device", "host"])
@pytest.mark.parametrize("path", GOLDEN_BLUR, ids=lambda p: os.path.basename(p)[:-4])
def test_blur_golden_bit_exact(lhpc, gpu, path, buffers):
    g = S.load_golden(os.path.basename(path))
    ny, nx, ghost, nb = (int(g[k]) for k in ("ny", "nx", "ghost", "nblur"))
    fn = lhpc.blur_y if os.path.basename(path).startswith("blur_y") else lhpc.blur_x
    if buffers == "device":
        import torch
        b = torch.empty(ny * nx, dtype=torch.float32, device=gpu)
        out = fn(_dev(gpu, g["a"]), b, ny, nx, ghost, nb).cpu().numpy()
    else:
        out = fn(g["a"].copy(), np.empty(ny * nx, dtype=np.float32), ny, nx, ghost, nb)
    assert np.array_equal(out, g["b"])


SHAPES = [(1, 1, 8), (3, 5, 8), (17, 33, 8), (64, 1000, 8), (257, 131, 12), (100, 96, 8),
          (33, 64, 3), (512, 1024, 8)]


@pytest.mark.parametrize("ny,nx,ghost", SHAPES)
@pytest.mark.parametrize("ydir", [False, True])
def test_blur_shapes_vs_oracle(lhpc, gpu, ny, nx, ghost, ydir):
    import torch
    nb = min(8, ghost)
    a = S.random_padded(((ny + 2 * ghost) * (nx + 2 * ghost),), seed=ny * 7919 + nx)
    want = S.blur_oracle(a, ny, nx, ghost, nb, ydir)
    b = torch.empty(ny * nx, dtype=torch.float32, device=gpu)
    fn = lhpc.blur_y if ydir else lhpc.blur_x
    got = fn(_dev(gpu, a), b, ny, nx, ghost, nb).cpu().numpy()
    assert np.array_equal(got, want)


@pytest.mark.slow
@pytest.mark.parametrize("ydir", [False, True])
def test_blur_reference_grid_8192(lhpc, gpu, ydir):
    """The reference benchmark's own size: 8192², ghost 8, nblur 8."""
    import torch
    n, g = 8192, 8
    a = S.random_padded(((n + 2 * g) ** 2,), seed=8192 + ydir)
    want = S.blur_oracle(a, n, n, g, 8, ydir)
    b = torch.empty(n * n, dtype=torch.float32, device=gpu)
    got = (lhpc.blur_y if ydir else lhpc.blur_x)(_dev(gpu, a), b, n, n, g, 8).cpu().numpy()
    assert np.array_equal(got, want)


def test_blur_rejects_narrow_ghost(lhpc):
    a = np.zeros((4 + 4) * (4 + 4), dtype=np.float32)
    with pytest.raises(lhpc.LhpcError):
        lhpc.blur_x(a, np.zeros(16, dtype=np.float32), 4, 4, 2, 8)


@pytest.mark.parametrize("nz,ny,nx", [(1, 1, 1), (2, 3, 5), (16, 17, 65), (33, 64, 64), (64, 96, 130),
                                      (4, 5, 512), (5, 9, 517), (3, 7, 1100)])  # ≥ 512: the 1 × 8 default tile
def test_stencil7_vs_oracle(lhpc, gpu, nz, ny, nx):
    g = 1
    shape = (nz + 2, ny + 2, nx + 2)
    u = S.random_padded(shape, seed=nz * 131 + nx, zero_ghost=False).reshape(-1)
    out0 = S.random_padded(shape, seed=99).reshape(-1)  # ghosts of `out` must survive
    want = S.stencil7_oracle(u, nz, ny, nx, g, -6.0, 1.0, out=out0.copy())
    got = lhpc.stencil7(_dev(gpu, u), _dev(gpu, out0), nz, ny, nx, g, -6.0, 1.0).cpu().numpy()
    assert np.array_equal(got, want)
    # host-buffer path
    got_h = lhpc.stencil7(u.copy(), out0.copy(), nz, ny, nx, g, -6.0, 1.0)
    assert np.array_equal(got_h, want)


def test_stencil7_planes_compose(lhpc, gpu):
    """Computing z-plane ranges separately (the halo-overlap schedule) gives
    exactly the full sweep."""
    nz, ny, nx = 40, 30, 70
    shape = (nz + 2, ny + 2, nx + 2)
    u = _dev(gpu, S.random_padded(shape, seed=5).reshape(-1))
    full = lhpc.stencil7(u, _dev(gpu, np.zeros(np.prod(shape), np.float32)), nz, ny, nx, 1, -6.0, 1.0)
    part = _dev(gpu, np.zeros(np.prod(shape), np.float32))
    for z0, z1 in ((0, 1), (1, 17), (17, 39), (39, 40)):
        lhpc.stencil7_planes(u, part, nz, ny, nx, 1, -6.0, 1.0, z0, z1)
    import torch
    assert torch.equal(full, part)


@pytest.mark.slow
def test_stencil7_c5_size(lhpc, gpu):
    """BASELINE configs[4] grid (512³, Dirichlet-0 ghosts, c0=-6, c1=1)."""
    n, g = 512, 1
    shape = (n + 2,) * 3
    u = S.random_padded(shape, seed=0x5EED0005, zero_ghost=True, ghost=1).reshape(-1)
    want = S.stencil7_oracle(u, n, n, n, g, -6.0, 1.0)
    got = lhpc.stencil7(_dev(gpu, u), _dev(gpu, np.zeros_like(u)), n, n, n, g, -6.0, 1.0).cpu().numpy()
    assert np.array_equal(got, want)


S7_IMPLS = ["buf", "buf:1,8,0,2", "buf:1,4,128,3", "buf:1,8,5,3", "buf:1,8,16", "buf:1,8,32", "buf:1,4,32",
            "buf:1,8,4", "simple",
            # tuning-build tiles (their kernels spill SGPRs): LHPC_ERR_UNSUPPORTED in the product library
            "buf:2,8,0,2", "buf:4,4,128,3", "buf:2,8,32", "buf:2,4,32", "buf:4,8,32"]


def _s7_in_product(name, cfg):
    """The tiles the product library compiles (lhpc_stencil.hip s7_launch):
    one row per wave, or the x4 ring's LDS-shared 2 rows × 4 blocks."""
    if name == "simple" or not cfg:
        return True
    ry, nj = (int(v) for v in cfg.split(",")[:2])
    return nj in (4, 8) and (ry == 1 or (name == "buf4lds" and ry == 2 and nj == 4))


def _s7_options(lhpc, name, cfg, store):
    """lhpc_options fields for a stencil7 variant: impl name, "RY,NJ,ZC[,PF]", store policy."""
    o = {"stencil7_impl": {"buf": lhpc.S7_RING, "buf4": lhpc.S7_RING_X4, "buf4lds": lhpc.S7_RING_X4_LDS,
                           "simple": lhpc.S7_SIMPLE}[name],
         "stencil7_store": {"nt": lhpc.STORE_NT, "plain": lhpc.STORE_PLAIN, "staged": lhpc.STORE_STAGED}[store]}
    if cfg:
        for k, v in zip(("stencil7_ry", "stencil7_nj", "stencil7_zc", "stencil7_pf"), cfg.split(",")):
            o[k] = int(v)
    return o


@pytest.mark.parametrize("impl", S7_IMPLS)
@pytest.mark.parametrize("store", ["nt", "plain", "staged"])
def test_stencil7_every_impl(lhpc, gpu, impl, store):
    """Every stencil7 implementation / tiling / store mode selectable through
    lhpc_options.stencil7_* ("simple": the thread-per-column kernel the launcher
    falls back to when a row's byte offset does not fit a buffer voffset) is
    bit-exact against the oracle on ragged shapes: nx
    spanning several 512-wide x tiles with a partial last one, ny and nz not
    multiples of the row / z-chunk tiles, ghost widths 1 and 2."""
    name, _, cfg = impl.partition(":")
    opts = _s7_options(lhpc, name, cfg, store)
    if not _s7_in_product(name, cfg):
        with pytest.raises(lhpc.LhpcError) as e:
            u = np.zeros(5 * 6 * 7, np.float32)
            lhpc.stencil7(_dev(gpu, u), _dev(gpu, u.copy()), 3, 4, 5, 1, -6.0, 1.0, options=opts)
        assert e.value.status == -5
        return
    for (nz, ny, nx, g) in ((37, 45, 1100, 1), (9, 19, 130, 2), (3, 2, 1, 1)):
        shape = (nz + 2 * g, ny + 2 * g, nx + 2 * g)
        u = S.random_padded(shape, seed=nz * 7 + nx + g, zero_ghost=False).reshape(-1)
        out0 = S.random_padded(shape, seed=1234 + g).reshape(-1)
        want = S.stencil7_oracle(u, nz, ny, nx, g, -6.0, 1.0, out=out0.copy())
        got = lhpc.stencil7(_dev(gpu, u), _dev(gpu, out0), nz, ny, nx, g, -6.0, 1.0, options=opts).cpu().numpy()
        assert np.array_equal(got, want), (impl, store, nz, ny, nx, g)


S7_BUF4 = ["1,8,16", "1,8,0", "1,4,0", "1,8,0,3", "1,4,7,1", "2,4,7", "2,4,0", "2,8,0", "4,8,32", "4,4,32"]


@pytest.mark.parametrize("cfg", S7_BUF4)
@pytest.mark.parametrize("store", ["nt", "plain"])
@pytest.mark.parametrize("impl", ["buf4", "buf4lds"])
def test_stencil7_buf4(lhpc, gpu, cfg, store, impl):
    """The x4 ring (stencil7_impl = S7_RING_X4, 4 consecutive x per lane,
    dwordx4 loads/stores at 4-B alignment) is bit-exact against the oracle on
    shapes whose nx is a multiple of its tile width — one and several x tiles,
    ny / nz ragged against the row and z-chunk tiles, ghost widths 1 to 3 (so
    rows start at every 4-B phase of a 16-B line) — and on ragged nx, where the
    last x tile is partial (dword loads and stores past nx, every lane phase
    of the last x4: nx % 4 = 0..3, nx < 4)."""
    opts = _s7_options(lhpc, impl, cfg, store)
    if not _s7_in_product(impl, cfg):  # tuning-build tile: refused by the product library
        with pytest.raises(lhpc.LhpcError) as e:
            u = np.zeros(5 * 6 * 7, np.float32)
            lhpc.stencil7(_dev(gpu, u), _dev(gpu, u.copy()), 3, 4, 5, 1, -6.0, 1.0, options=opts)
        assert e.value.status == -5
        return
    for (nz, ny, nx, g) in ((37, 45, 1024, 1), (9, 19, 512, 2), (3, 2, 1536, 3), (5, 9, 512, 1),
                            (37, 45, 1100, 1), (9, 19, 130, 2), (3, 2, 1, 1), (5, 7, 517, 3), (2, 3, 1541, 1),
                            (4, 5, 768, 2), (3, 4, 258, 1), (6, 3, 3, 2)):
        shape = (nz + 2 * g, ny + 2 * g, nx + 2 * g)
        u = S.random_padded(shape, seed=nz * 7 + nx + g, zero_ghost=False).reshape(-1)
        out0 = S.random_padded(shape, seed=1234 + g).reshape(-1)
        want = S.stencil7_oracle(u, nz, ny, nx, g, -6.0, 1.0, out=out0.copy())
        got = lhpc.stencil7(_dev(gpu, u), _dev(gpu, out0), nz, ny, nx, g, -6.0, 1.0, options=opts).cpu().numpy()
        assert np.array_equal(got, want), (cfg, store, nz, ny, nx, g)


@pytest.mark.parametrize("rows", [1, 2, 4, 8, 16, 32])
def test_blur_x_every_impl(lhpc, gpu, rows):
    """The wave-private blur_x at every rows-per-wave setting (options.blur_x_rows)
    is bit-exact against the oracle on vector-eligible ragged shapes: nx not a
    multiple of the 256-float segment, ny not a multiple of the row group.
    (Unaligned shapes take the block-LDS kernel: test_blur_shapes_vs_oracle.)"""
    import torch
    for ny, nx, ghost in ((37, 260, 8), (5, 1300, 8), (70, 2048, 12), (1, 4, 8)):
        a = S.random_padded(((ny + 2 * ghost) * (nx + 2 * ghost),), seed=ny * 31 + nx)
        want = S.blur_oracle(a, ny, nx, ghost, 8, False)
        b = torch.empty(ny * nx, dtype=torch.float32, device=gpu)
        got = lhpc.blur_x(_dev(gpu, a), b, ny, nx, ghost, 8, options={"blur_x_rows": rows}).cpu().numpy()
        assert np.array_equal(got, want), (rows, ny, nx, ghost)
