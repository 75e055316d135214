"""GPU radix sort and COO→CSR against the oracle and
the reference's own sorted output.  Bit-exact: sorted keys are unique, and
the sort is stable so (key, value) pairs are too."""
import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 2, 63, 64, 65, 4095, 4096, 4097, 8191, 8192, 8193, 16383, 16384, 16385, 20479, 20480, 20481,
         2 * 20480 + 3, 3 * 20480 + 5, 24575, 24576, 24577, 100_003, (1 << 20) + 7]  # sub-tiles: 20480 u32 keys
                                                                                   # (prefetched), 16384 pairs


def _dev(gpu, a):
    import torch
    return torch.from_numpy(a).to(gpu)


def _u32_view(t):
    return t.cpu().numpy().view(np.uint32)


def _keys(n, kind, seed, kt=np.uint32):
    rng = np.random.default_rng(seed)
    hi = np.iinfo(kt).max
    if kind == "uniform":
        return rng.integers(0, hi, size=n, dtype=kt, endpoint=True)
    if kind == "equal":
        return np.full(n, kt(0xDEADBEEF), dtype=kt)
    if kind == "few":
        return rng.choice(np.array([0, 1, 255, 256, hi], dtype=kt), size=n)
    if kind == "sorted":
        return np.sort(rng.integers(0, hi, size=n, dtype=kt, endpoint=True))
    if kind == "reversed":
        return np.sort(rng.integers(0, hi, size=n, dtype=kt, endpoint=True))[::-1].copy()
    raise ValueError(kind)


@pytest.mark.parametrize("n", SIZES)
def test_sort_u32_device_sizes(lhpc, gpu, n):
    keys = _keys(n, "uniform", n)
    t = _dev(gpu, keys.view(np.int32))
    lhpc.radix_sort(t)
    assert np.array_equal(_u32_view(t), np.sort(keys))


@pytest.mark.parametrize("kind", ["equal", "few", "sorted", "reversed"])
def test_sort_u32_distributions(lhpc, gpu, kind):
    keys = _keys(300_001, kind, 3)
    t = _dev(gpu, keys.view(np.int32))
    lhpc.radix_sort(t)
    assert np.array_equal(_u32_view(t), S.sort_oracle(keys))


@pytest.mark.parametrize("off", [1, 2, 3])
@pytest.mark.parametrize("n", [100_003, (1 << 20) + 7])
def test_sort_u32_offset_pointer(lhpc, gpu, n, off):
    """Keys whose device pointer is 4-B but not 16-B aligned (a slice t[off:]):
    the upsweep's 16-B loads are used only on 16-B aligned keys;
    the keys around the slice stay untouched."""
    import torch
    keys = _keys(n + off + 5, "uniform", n + off)
    t = _dev(gpu, keys.view(np.int32))
    sl = t[off:off + n]
    assert sl.data_ptr() % 16 != 0
    vals = torch.arange(n, dtype=torch.int32, device=gpu)
    lhpc.radix_sort_pairs(sl, vals, 0, 32)
    wk, wv = S.sort_oracle(keys[off:off + n], np.arange(n, dtype=np.uint32), 0, 32)
    got = _u32_view(t)
    assert np.array_equal(got[off:off + n], wk) and np.array_equal(_u32_view(vals), wv)
    assert np.array_equal(got[:off], keys[:off]) and np.array_equal(got[off + n:], keys[off + n:])
    t2 = _dev(gpu, keys.view(np.int32))
    lhpc.radix_sort(t2[off:off + n])
    assert np.array_equal(_u32_view(t2)[off:off + n], np.sort(keys[off:off + n]))


def test_sort_u32_host_path(lhpc, gpu):
    keys = _keys(77_777, "uniform", 5)
    got = lhpc.radix_sort(keys.copy())
    assert np.array_equal(got, np.sort(keys))


@pytest.mark.parametrize("name", ["sort_ref_gpu_keys_5000.npz", "sort_ref_cpu_keys_4097.npz"])
def test_sort_matches_reference_golden(lhpc, gpu, name):
    g = S.load_golden(name)
    t = _dev(gpu, g["keys"].view(np.int32))
    lhpc.radix_sort(t)
    assert np.array_equal(_u32_view(t), g["sorted"])


@pytest.mark.parametrize("begin,end", [(0, 12), (4, 28), (8, 16), (3, 3), (31, 32)])
def test_sort_u32_bit_range(lhpc, gpu, begin, end):
    keys = _keys(50_000, "uniform", begin * 100 + end)
    vals = np.arange(keys.size, dtype=np.uint32)
    kt, vt = _dev(gpu, keys.view(np.int32)), _dev(gpu, vals.view(np.int32))
    lhpc.radix_sort_pairs(kt, vt, begin, end)
    wk, wv = S.sort_oracle(keys, vals, begin, end)
    assert np.array_equal(_u32_view(kt), wk) and np.array_equal(_u32_view(vt), wv)


@pytest.mark.parametrize("n", [1, 65, 16383, 16384, 16385, 3 * 16384 + 5, 300_001])
def test_sort_pairs_u32_stable(lhpc, gpu, n):
    """32-bit pairs across the 16384-key sub-tile boundaries, a third of the
    keys equal (stability is observable through the values)."""
    rng = np.random.default_rng(0x9A1 + n)
    keys = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    keys[::3] = keys[0]
    vals = np.arange(n, dtype=np.uint32)
    kt, vt = _dev(gpu, keys.view(np.int32)), _dev(gpu, vals.view(np.int32))
    lhpc.radix_sort_pairs(kt, vt, 0, 32)
    wk, wv = S.sort_oracle(keys, vals, 0, 32)
    assert np.array_equal(_u32_view(kt), wk) and np.array_equal(_u32_view(vt), wv)


@pytest.mark.parametrize("n", [1, 65, 4097, 16383, 16384, 16385, 3 * 16384 + 5, 70_001, 1 << 20])
@pytest.mark.parametrize("bits", [64, 47, 20])
def test_sort_pairs_u64_stable(lhpc, gpu, n, bits):
    import torch
    rng = np.random.default_rng(n + bits)
    keys = rng.integers(0, 1 << bits, size=n, dtype=np.uint64) if bits < 64 else \
        rng.integers(0, np.iinfo(np.uint64).max, size=n, dtype=np.uint64, endpoint=True)
    keys[::3] = keys[0]  # duplicates: stability is observable through the values
    vals = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    kt = _dev(gpu, keys.view(np.int64))
    vt = _dev(gpu, vals.view(np.int32))
    lhpc.radix_sort_pairs(kt, vt, 0, bits)
    wk, wv = S.sort_oracle(keys, vals, 0, bits)
    assert np.array_equal(kt.cpu().numpy().view(np.uint64), wk)
    assert np.array_equal(vt.cpu().numpy().view(np.uint32), wv)
    torch.cuda.synchronize()


@pytest.mark.parametrize("off", [0, 1])
def test_sort_pairs_u64_offset_pointer(lhpc, gpu, off):
    """64-bit keys 8 B past a 16-B boundary (a slice t[1:]): the upsweep's
    16-B loads are used only on 16-B aligned keys, one key per load
    otherwise; the same stable order either way."""
    rng = np.random.default_rng(0x64 + off)
    n = 3 * 16384 + 77
    keys = rng.integers(0, 1 << 40, size=n, dtype=np.uint64)
    keys[::5] = keys[1]
    vals = np.arange(n, dtype=np.uint32)
    kt = _dev(gpu, np.concatenate([np.zeros(off, np.uint64), keys]).view(np.int64))[off:]
    vt = _dev(gpu, np.concatenate([np.zeros(off, np.uint32), vals]).view(np.int32))[off:]
    lhpc.radix_sort_pairs(kt, vt, 0, 40)
    wk, wv = S.sort_oracle(keys, vals, 0, 40)
    assert np.array_equal(kt.cpu().numpy().view(np.uint64), wk)
    assert np.array_equal(vt.cpu().numpy().view(np.uint32), wv)


def test_sort_pairs_u64_host_path(lhpc, gpu):
    rng = np.random.default_rng(9)
    keys = rng.integers(0, 1 << 40, size=33_333, dtype=np.uint64)
    vals = np.arange(keys.size, dtype=np.uint32)
    k, v = lhpc.radix_sort_pairs(keys.copy(), vals.copy(), 0, 40)
    wk, wv = S.sort_oracle(keys, vals, 0, 40)
    assert np.array_equal(k, wk) and np.array_equal(v, wv)


def test_sort_rejects_bad_args(lhpc, gpu):
    with pytest.raises(lhpc.LhpcError):
        lhpc.radix_sort(np.zeros(4, np.uint32), 0, 33)
    with pytest.raises(lhpc.LhpcError):
        lhpc.radix_sort(np.zeros(4, np.uint32), 9, 8)


@pytest.mark.slow
def test_sort_reference_test_size(lhpc, gpu):
    """The reference GPU test's own case (tests/test_radixsort_gpu/test_radixsort_gpu_v4.cc:7-21):
    100M keys from its generator, checked sorted — and here also equal to np.sort."""
    keys = S.ref_gpu_test_keys(100_000_000)
    if keys is None:
        rng = np.random.default_rng(0)
        keys = rng.integers(100, np.iinfo(np.uint32).max - 100, size=100_000_000, dtype=np.uint32)
    t = _dev(gpu, keys.view(np.int32))
    lhpc.radix_sort(t)
    got = _u32_view(t)
    del t
    assert np.all(got[1:] >= got[:-1])
    keys.sort()
    assert np.array_equal(got, keys)


# ------------------------------------------------------------ COO → CSR
def _coo(n_rows, n_cols, nnz, seed, dt, dup=True):
    rng = np.random.default_rng(seed)
    rows = rng.integers(0, max(n_rows, 1), nnz).astype(np.int32)
    cols = rng.integers(0, max(n_cols, 1), nnz).astype(np.int32)
    if dup and nnz > 200:
        rows[50:150] = rows[0]
        cols[50:150] = rng.integers(0, min(4, n_cols), 100)
    vals = rng.uniform(-1, 1, nnz).astype(dt)
    return rows, cols, vals


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(1000, 1000, 20_000), (1, 1, 5), (7, 100_000, 3000), (100_000, 3, 50_000),
                                   (5000, 5000, 0), (300_000, 300_000, 1_000_003)])
def test_coo_to_csr_vs_oracle(lhpc, gpu, dt, shape):
    n_rows, n_cols, nnz = shape
    rows, cols, vals = _coo(n_rows, n_cols, nnz, nnz + n_rows, dt)
    want = S.coo_oracle(n_rows, n_cols, rows, cols, vals)
    for rpb in (64, 32):
        got = lhpc.coo_to_csr(n_rows, n_cols, rows, cols, vals, row_ptr_bits=rpb)
        assert np.array_equal(got[0].astype(np.int64), want[0])
        assert np.array_equal(got[1], want[1]) and np.array_equal(got[2], want[2])
    d = lhpc.coo_to_csr(n_rows, n_cols, _dev(gpu, rows), _dev(gpu, cols), _dev(gpu, vals))
    assert np.array_equal(d[0].cpu().numpy(), want[0])
    assert np.array_equal(d[1].cpu().numpy(), want[1]) and np.array_equal(d[2].cpu().numpy(), want[2])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("off", [0, 1, 2])
def test_coo_to_csr_device_offsets(lhpc, gpu, dt, off):
    """Device COO arrays starting 0 / 4 / 8 B past a 16-B boundary (slices
    t[off:]): the key pass takes four entries per thread with 16-B loads only
    when rows, cols and (fp32) values are all 16-B aligned, one per thread
    otherwise; the same CSR either way, nnz not a multiple of 4."""
    n_rows, n_cols, nnz = 3000, 5000, 40_003
    rows, cols, vals = _coo(n_rows, n_cols, nnz, 0xC00 + off, dt)
    want = S.coo_oracle(n_rows, n_cols, rows, cols, vals)

    def pad(a):
        return _dev(gpu, np.concatenate([np.zeros(off, a.dtype), a]))[off:]
    d = lhpc.coo_to_csr(n_rows, n_cols, pad(rows), pad(cols), pad(vals))
    assert np.array_equal(d[0].cpu().numpy(), want[0])
    assert np.array_equal(d[1].cpu().numpy(), want[1]) and np.array_equal(d[2].cpu().numpy(), want[2])


def test_coo_to_csr_feeds_spmv(lhpc, gpu):
    """Round trip: a generated CSR → COO (shuffled) → coo_to_csr gives back the
    same CSR, and the SpMV plan built from it reproduces y."""
    rp, col, val = lhpc.gen_uniform_csr(20_000, 20_000, 9, dtype=lhpc.F32, seed=0xC0C0)
    rows = np.repeat(np.arange(20_000, dtype=np.int32), np.diff(rp).astype(np.int64))
    perm = np.random.default_rng(1).permutation(rows.size)
    got = lhpc.coo_to_csr(20_000, 20_000, rows[perm], col[perm], val[perm], row_ptr_bits=32)
    assert np.array_equal(got[0], rp.astype(np.int32)) and np.array_equal(got[1], col)
    assert np.array_equal(got[2], val)


def test_coo_to_csr_rejects_out_of_range(lhpc, gpu):
    with pytest.raises(lhpc.LhpcError):
        lhpc.coo_to_csr(4, 4, np.array([0, 4], np.int32), np.array([0, 0], np.int32), np.ones(2, np.float32))
    with pytest.raises(lhpc.LhpcError):
        lhpc.coo_to_csr(4, 4, np.array([0, 1], np.int32), np.array([-1, 0], np.int32), np.ones(2, np.float64))


def test_sort_u32_reference_100m(lhpc, gpu):
    """The reference's largest GPU radix-sort test size, 100,000,000 keys
    (tests/test_radixsort_gpu_local_count/src/test_radix_local_count.cu:199-201),
    uniform 32-bit keys: the device sort equals numpy's sort bit for bit."""
    keys = _keys(100_000_000, "uniform", 0x5EED100)
    t = _dev(gpu, keys.view(np.int32))
    lhpc.radix_sort(t)
    got = _u32_view(t)
    del t
    keys.sort(kind="stable")
    assert np.array_equal(got, keys)


def test_sort_u32_past_2_31(lhpc, gpu):
    """2^31 + 4099 keys (8.6 GB): sub-tile bases and output positions past
    2^31 (int64 tile offsets, u32 positions up to 2^32).  Checked on the
    device: sorted as unsigned, the same 65536-bin histogram of the top 16
    bits and the same sum as the input (a permutation), and the last partial
    sub-tile's keys in place."""
    import torch
    n = (1 << 31) + 4099
    g = torch.Generator(device=gpu)
    g.manual_seed(0x2E31)
    t = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=gpu, generator=g)
    t[-3:] = torch.tensor([-1, 0, 12345], dtype=torch.int32, device=gpu)  # max, min, a marker in the tail sub-tile

    def summary(x):
        u = x.to(torch.int64) & 0xFFFFFFFF
        return torch.bincount(u >> 16, minlength=65536), int(u.sum().item())
    h0, s0 = summary(t)
    lhpc.radix_sort(t)
    torch.cuda.synchronize()
    h1, s1 = summary(t)
    assert torch.equal(h0, h1) and s0 == s1
    u = t.to(torch.int64) & 0xFFFFFFFF
    assert bool((u[1:] >= u[:-1]).all())
    assert int(u[0]) == 0 and int(u[-1]) == 0xFFFFFFFF


@pytest.mark.parametrize("poison", [0x00, 0xA5, 0xFF])
def test_coo_to_csr_poisoned_pool(lhpc, gpu, poison):
    """Regression for the round-2 host-path race: the on-device
    sort / scan / COO→CSR still take their scratch from the stream-ordered
    pool (lhpc_sort.hip DevBuf: the library's own scratch pool).  Every
    scratch buffer must be fully written before it is read, so results must
    not depend on what the pool hands back: the pool is left filled with
    0x00 / 0xA5 / 0xFF before each call (lhpc_scratch_poison, on the call's
    stream), for the
    4-entry symmetric Matrix Market case that failed, tiny and ragged COO
    inputs with duplicates and empty rows, and the sorts they run."""
    import torch
    P = lhpc.lib
    st = torch.cuda.current_stream(gpu)
    cases = [(3, 3, np.array([0, 1, 0, 2]), np.array([0, 0, 1, 2]), np.array([2.0, -1.5, -1.5, 4.0]))]
    rng = np.random.default_rng(0x9015 + poison)
    for n_rows, n_cols, nnz in ((1, 1, 1), (5, 7, 2), (64, 65, 300), (1000, 50, 5000), (3, 100_000, 4099)):
        cases.append((n_rows, n_cols, rng.integers(0, n_rows, nnz), rng.integers(0, n_cols, nnz),
                      rng.integers(-8, 9, nnz) / 8.0))
    for n_rows, n_cols, r, c, v in cases:
        r, c, v = r.astype(np.int32), c.astype(np.int32), v.astype(np.float64)
        want = S.coo_oracle(n_rows, n_cols, r, c, v)
        for _ in range(3):
            assert P.lhpc_scratch_poison(1 << 24, poison, st.cuda_stream) == 0
            rp, col, val = lhpc.coo_to_csr(n_rows, n_cols, _dev(gpu, r), _dev(gpu, c), _dev(gpu, v), stream=st)
            torch.cuda.synchronize()
            assert np.array_equal(rp.cpu().numpy(), want[0]), (n_rows, n_cols, r.size)
            assert np.array_equal(col.cpu().numpy(), want[1]) and np.array_equal(val.cpu().numpy(), want[2])
    keys = rng.integers(0, 1 << 32, 5000, dtype=np.uint64).astype(np.uint32)
    for _ in range(3):
        assert P.lhpc_scratch_poison(1 << 24, poison, st.cuda_stream) == 0
        kd = _dev(gpu, keys.view(np.int32))
        lhpc.radix_sort(kd, stream=st)
        torch.cuda.synchronize()
        assert np.array_equal(_u32_view(kd), np.sort(keys))
