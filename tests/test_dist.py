"""Multi-rank SpMV path on CPU: world_size 2 (and 3) with the gloo backend.

Exercises libhpc_amd.dist exactly as bench.py uses it on N GPUs (nnz-balanced
row cuts, rebased local CSR, padded all_gather_into_tensor, assembly), with
the oracle as the local product.  The assembled y must equal the
unpartitioned oracle y bit-for-bit (each row is summed by the same code on
the same data — SURVEY §8c "partition identity").
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, q):
    try:
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import libhpc_amd as L
        from libhpc_amd.dist import DistSpMV, row_block
        from tests import _support as S
        n = 20_011
        if kind == "powerlaw":
            rp, col, val = L.gen_powerlaw_csr(n, n, lmax=2000, dtype=L.F64, seed=0xD157)
        else:
            rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=L.F32, seed=0xD158)
        x = L.gen_values(L.F64 if kind == "powerlaw" else L.F32, 0, n, 0xD159)
        blk = row_block(rp, col, val, rank, world)

        def local(xt, yt):  # oracle as the local product (CPU test only)
            _, yr, _ = S.spmv_oracle(blk.row_ptr, blk.col_idx, blk.val, xt.numpy())
            yt.copy_(torch.from_numpy(yr))

        xt = torch.from_numpy(x)
        d = DistSpMV(blk, local, like=xt)
        d.step(xt)
        y = d.assemble().numpy()
        _, want, _ = S.spmv_oracle(rp, col, val, x)
        ok = np.array_equal(y, want)
        nnz_local = int(blk.row_ptr[-1])
        dist.destroy_process_group()
        q.put((rank, ok, nnz_local, int(rp[-1])))
    except Exception as e:  # report, never hang the parent
        q.put((rank, repr(e), -1, -1))


@pytest.mark.parametrize("world,kind", [(2, "uniform"), (3, "powerlaw"), (2, "powerlaw")])
def test_distributed_spmv_gloo(world, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    res.sort()
    for rank, ok, _, _ in res:
        assert ok is True, f"rank {rank}: {ok}"
    total = res[0][3]
    assert sum(r[2] for r in res) == total
    # nnz balance: each block within one max-row of total/world
    assert max(r[2] for r in res) - min(r[2] for r in res) <= 10_000


def _worker_overlap(rank, world, port, K, q, balanced=False):
    try:
        import torch
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import libhpc_amd as L
        from libhpc_amd.dist import DistSpMVOverlap, InterleavedBlocks
        from tests import _support as S
        n = 10_007
        rp, col, val = L.gen_powerlaw_csr(n, n, lmax=500, dtype=L.F32, seed=0xD160)
        x = L.gen_values(L.F32, 0, n, 0xD161)
        ib = InterleavedBlocks(n, world, K, row_ptr=rp if balanced else None)
        fns = []
        for k in range(K):
            lrp, lc, lv = ib.local_csr(rp, col, val, rank, k)

            def f(xt, yt, lrp=lrp, lc=lc, lv=lv):  # oracle as the local product (CPU test only)
                _, yr, _ = S.spmv_oracle(lrp, lc, lv, xt.numpy())
                yt.copy_(torch.from_numpy(yr))
            fns.append(f)
        d = DistSpMVOverlap(ib, fns, like=torch.from_numpy(x))
        y = d.step(torch.from_numpy(x)).numpy()
        _, want, _ = S.spmv_oracle(rp, col, val, x)
        dist.destroy_process_group()
        q.put((rank, bool(np.array_equal(y, want))))
    except Exception as e:
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world,K,balanced", [(2, 3, False), (3, 4, False), (4, 1, False), (2, 3, True),
                                              (3, 4, True), (4, 2, True)])
def test_overlapped_allgather_gloo(world, K, balanced):
    """The torch-collective form of the overlapped SpMV: equal-row or
    nnz-balanced interleaved blocks (the latter padded for all_gather and
    compacted), assembled y bit-identical to the unpartitioned oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_overlap, args=(r, world, port, K, q, balanced)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    for rank, ok in res:
        assert ok is True, f"rank {rank}: {ok}"


@pytest.mark.parametrize("world,K,rank", [(2, 2, 0), (2, 2, 1), (3, 4, 2), (8, 2, 7)])
def test_local_csr_all_concatenates_chunks(world, K, rank):
    """InterleavedBlocks.local_csr_all (the row-range plan's input) is the
    rank's K chunk CSRs stacked, with splits at multiples of B."""
    from libhpc_amd.dist import InterleavedBlocks
    rng = np.random.default_rng(world * 100 + K * 10 + rank)
    n = 1003
    lens = rng.integers(0, 9, size=n)
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=rp[1:])
    col = rng.integers(0, n, size=int(rp[-1])).astype(np.int32)
    val = rng.standard_normal(int(rp[-1])).astype(np.float32)
    ib = InterleavedBlocks(n, world, K)
    lrp, lc, lv, splits = ib.local_csr_all(rp, col, val, rank)
    assert splits == [k * ib.B for k in range(1, K)]
    assert lrp.shape[0] == K * ib.B + 1 and lrp[0] == 0 and lrp[-1] == lc.shape[0] == lv.shape[0]
    for k in range(K):
        prp, pc, pv = ib.local_csr(rp, col, val, rank, k)
        seg = lrp[k * ib.B:(k + 1) * ib.B + 1]
        assert np.array_equal(seg - seg[0], prp.astype(np.int64))
        assert np.array_equal(lc[seg[0]:seg[-1]], pc) and np.array_equal(lv[seg[0]:seg[-1]], pv)


@pytest.mark.parametrize("world,K", [(2, 2), (3, 4), (8, 2), (4, 1)])
def test_interleaved_cuts_are_nnz_balanced(world, K):
    """cuts by binary search on row_ptr for the nnz targets
    b·nnz/(world·K) — every block within one row's length of the target."""
    import libhpc_amd as L
    from libhpc_amd.dist import InterleavedBlocks
    n = 50_021
    rp, _, _ = L.gen_powerlaw_csr(n, n, lmax=3000, dtype=L.F32, seed=0xD170)
    ib = InterleavedBlocks(n, world, K, row_ptr=rp)
    assert np.array_equal(ib.cuts, L.interleaved_cuts(rp, world, K))
    nnz, P = int(rp[-1]), world * K
    lens = np.diff(rp)
    for b in range(1, P):
        target = -(-b * nnz // P)
        c = int(ib.cuts[b])
        assert rp[c] >= target and (c == 0 or rp[c - 1] < target)
    blk = np.diff(rp[ib.cuts])
    assert blk.max() - blk.min() <= 2 * lens.max()


def _local_rows(rp, col, val, x, world, K, cuts):
    """Every rank's y before the exchange: rank r's stacked local CSR
    (interleaved_local_csr, the input of lhpc_dist_spmv_plan_create) reduced
    with the oracle into its blocks' rows; every other row NaN."""
    import libhpc_amd as L
    from tests import _support as S
    ys = [np.full(rp.shape[0] - 1, np.nan, dtype=val.dtype) for _ in range(world)]
    for r in range(world):
        lrp, lc, lv = L.interleaved_local_csr(rp, col, val, cuts, world, K, r)
        _, yl, _ = S.spmv_oracle(lrp, lc, lv, x)
        at = 0
        for k in range(K):
            b0, b1 = int(cuts[k * world + r]), int(cuts[k * world + r + 1])
            ys[r][b0:b1] = yl[at:at + b1 - b0]
            at += b1 - b0
    return ys


def _run_schedules(ys, cuts, world, K, exchange, broadcast=False):
    """Execute, on the CPU, the transfers every rank's lhpc_dist_spmv issues
    (lhpc_dist_exchange_schedule — the same host function the device path
    walks) with RCCL / peer-store semantics, checking on the way that the
    ranks' collectives match (same calls, same order: a mismatch would hang
    RCCL) and that each in-place all-gather sends from its own slot."""
    import libhpc_amd as L
    sched = [L.dist_exchange_schedule(cuts, world, K, r, exchange, broadcast) for r in range(world)]
    for k in range(K):
        per = [[e for e in sched[r] if e["chunk"] == k] for r in range(world)]
        if exchange == L.DIST_EXCHANGE_RCCL:
            sig = [[(e["kind"], e["root"], e["group"], e["offset"], e["count"]) for e in per[r]] for r in range(world)]
            assert all(sg == sig[0] for sg in sig), f"chunk {k}: collectives differ between ranks"
            for j in range(len(per[0])):
                e0 = per[0][j]
                if e0["kind"] == L.XFER_ALLGATHER:
                    off, cnt = e0["offset"], e0["count"]
                    parts = []
                    for r in range(world):
                        assert per[r][j]["send_offset"] == off + r * cnt, "in-place all-gather slot"
                        parts.append(ys[r][off + r * cnt:off + (r + 1) * cnt].copy())
                    for r in range(world):
                        for q in range(world):
                            ys[r][off + q * cnt:off + (q + 1) * cnt] = parts[q]
                else:
                    assert e0["kind"] == L.XFER_BROADCAST and e0["group"] == 1
                    off, cnt, root = e0["offset"], e0["count"], e0["root"]
                    data = ys[root][off:off + cnt].copy()
                    for r in range(world):
                        ys[r][off:off + cnt] = data
        else:
            for r in range(world):
                for e in per[r]:
                    assert e["kind"] == L.XFER_PUSH and e["root"] == r
                    off, cnt = e["offset"], e["count"]
                    b = k * world + r
                    assert (off, off + cnt) == (int(cuts[b]), int(cuts[b + 1])), "a rank pushes exactly its block"
                    for q in range(world):
                        if q != r:
                            ys[q][off:off + cnt] = ys[r][off:off + cnt]
    return sched


@pytest.mark.parametrize("world,K", [(2, 2), (3, 3), (8, 2), (1, 2), (8, 1)])
@pytest.mark.parametrize("kind", ["powerlaw", "uniform", "tiny"])
@pytest.mark.parametrize("exchange", ["rccl", "rccl_bcast", "p2p"])
def test_native_dist_exchange_schedule(world, K, kind, exchange):
    """The native path's data layout (lhpc_dist_spmv_plan_create input) and
    its exchange schedule (lhpc_dist_exchange_schedule, the function
    broadcast/push issuing walks), run on the CPU for every rank: unequal
    nnz-balanced blocks (power-law rows: broadcast groups), equal blocks
    (uniform rows: one in-place all-gather per chunk), and a matrix with
    fewer rows than blocks (empty blocks); every rank ends with the
    unpartitioned y bit for bit (dyadic values), and the local stacked CSRs
    cover A exactly once (SURVEY §8c partition identity)."""
    import libhpc_amd as L
    from tests import _support as S
    if kind == "powerlaw":
        n = 30_011
        rp, col, val = L.gen_powerlaw_csr(n, n, lmax=2000, dtype=L.F32, dist=1, seed=0xD180)
    elif kind == "uniform":
        n = 4_096 * world * K
        rp, col, val = L.gen_uniform_csr(n, n, 5, dtype=L.F64, dist=1, seed=0xD182)
    else:
        n = 5
        rp, col, val = L.gen_uniform_csr(n, n, 2, dtype=L.F64, dist=1, seed=0xD183)
    x = L.gen_values(L.F32 if val.dtype == np.float32 else L.F64, 1, n, 0xD181)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    cuts = L.interleaved_cuts(rp, world, K)
    assert sum(int(L.interleaved_local_csr(rp, col, val, cuts, world, K, r)[0][-1]) for r in range(world)) == rp[-1]
    ys = _local_rows(rp, col, val, x, world, K, cuts)
    xk = L.DIST_EXCHANGE_P2P if exchange == "p2p" else L.DIST_EXCHANGE_RCCL
    sched = _run_schedules(ys, cuts, world, K, xk, broadcast=exchange == "rccl_bcast")
    for r, y in enumerate(ys):
        assert np.array_equal(y, want), f"rank {r}"
    kinds = {e["kind"] for s in sched for e in s}
    if exchange == "p2p":
        assert kinds <= {L.XFER_PUSH}
    elif exchange == "rccl_bcast" or (kind == "powerlaw" and world > 1):
        assert kinds <= {L.XFER_BROADCAST}
    elif kind == "uniform":
        assert kinds == {L.XFER_ALLGATHER}


def test_exchange_schedule_rejects_bad_input():
    import libhpc_amd as L
    with pytest.raises(L.LhpcError):
        L.dist_exchange_schedule([0, 5, 3, 8, 9], 2, 2, 0)  # cuts not ascending
    with pytest.raises(L.LhpcError):
        L.dist_exchange_schedule([0, 1, 2, 3, 4], 2, 2, 2)  # rank out of range


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("K", [1, 2, 3, 4])
@pytest.mark.parametrize("kind", ["uniform", "powerlaw", "empty"])
@pytest.mark.parametrize("tile_width", [1, 7, 4096, 39063])
def test_chain_parts_schedule(world, K, kind, tile_width):
    """The cross-step overlap's schedule (lhpc_dist_chain_parts, the host rule
    the chained stage of lhpc_dist_spmv_begin follows): tile t's gather
    waits for exchange part[t].  Exchanges land in chunk order and chunk j
    delivers rows [cuts[j·N], cuts[(j+1)·N]) of y = those columns of the next
    x.  Every column a tile reads must have landed (it lies below
    cuts[(part+1)·N]), the part is the earliest such chunk (the tile waits no
    longer than it must), and the parts never decrease along x."""
    import libhpc_amd as L
    if kind == "powerlaw":
        n = 30_011
        rp, _, _ = L.gen_powerlaw_csr(n, n, lmax=2000, dtype=L.F32, dist=1, seed=0xD190)
    elif kind == "uniform":
        n = 4_096 * world * K + 13
        rp, _, _ = L.gen_uniform_csr(n, n, 5, dtype=L.F32, dist=1, seed=0xD191)
    else:
        n = 5  # fewer rows than blocks: empty chunks
        rp, _, _ = L.gen_uniform_csr(n, n, 2, dtype=L.F32, dist=1, seed=0xD192)
    cuts = L.interleaved_cuts(rp, world, K)
    part = L.dist_chain_parts(cuts, world, K, n, tile_width)
    landed = [int(cuts[(j + 1) * world]) for j in range(K)]  # columns complete after exchange j
    for t, j in enumerate(part):
        last = min((t + 1) * tile_width, n)  # exclusive end of the tile's columns
        assert 0 <= j < K and landed[j] >= last, (t, j)
        assert j == 0 or landed[j - 1] < last, (t, j)
    assert np.all(np.diff(part) >= 0)


def test_chain_parts_rejects_bad_input():
    import libhpc_amd as L
    cuts = np.array([0, 5, 10], dtype=np.int64)
    with pytest.raises(L.LhpcError):
        L.dist_chain_parts(cuts, 2, 1, 11, 4)  # the chunks do not cover x
    with pytest.raises(L.LhpcError):
        L.dist_chain_parts(np.array([0, 6, 4, 10], dtype=np.int64), 1, 3, 10, 4)  # not ascending


def _cuts_of(kind, world, K):
    import libhpc_amd as L
    if kind == "uniform":
        rp = np.arange(0, 5 * (4096 * world * K) + 1, 5, dtype=np.int64)
    elif kind == "powerlaw":
        rp, _, _ = L.gen_powerlaw_csr(30_011, 30_011, lmax=2000, dtype=L.F32, dist=1, seed=0xD190)
    else:  # fewer rows than blocks: empty blocks
        rp = np.arange(0, 2 * 5 + 1, 2, dtype=np.int64)
    return L.interleaved_cuts(rp, world, K), int(rp.shape[0] - 1)


@pytest.mark.parametrize("world,K", [(8, 1), (8, 2), (8, 4), (2, 2), (3, 4)])
@pytest.mark.parametrize("kind", ["uniform", "powerlaw", "empty"])
@pytest.mark.parametrize("dtype", ["f32", "f64"])
@pytest.mark.parametrize("broadcast", [False, True])
def test_rccl_call_arguments(world, K, kind, dtype, broadcast):
    """the exact RCCL argument lists the device paths
    issue (lhpc_dist_rccl_calls = the records lhpc_dist.hip and lhpc_multi.hip
    walk, lhpc_rccl.hpp), for every rank: matching collectives on every rank
    (op, count, datatype, root, group brackets, recvbuff — a mismatch hangs
    RCCL), the in-place all-gather contract sendbuff == recvbuff + rank·count,
    in-place broadcasts of exactly the root's block, balanced group brackets,
    buffers inside y; then the calls are executed on byte buffers with RCCL
    semantics and every rank must end with the whole y."""
    import libhpc_amd as L
    dt = L.F32 if dtype == "f32" else L.F64
    tsz, npdt, ncdt = (4, np.float32, 7) if dt == L.F32 else (8, np.float64, 8)
    cuts, n = _cuts_of(kind, world, K)
    calls = [L.dist_rccl_calls(cuts, world, K, r, dt, broadcast) for r in range(world)]
    full = np.arange(n, dtype=npdt) + 1
    ys = []
    for r in range(world):
        y = np.full(n, np.nan, dtype=npdt)
        for k in range(K):
            b = k * world + r
            y[cuts[b]:cuts[b + 1]] = full[cuts[b]:cuts[b + 1]]
        ys.append(y.view(np.uint8))
    for k in range(K):
        per = [[c for c in calls[r] if c["chunk"] == k] for r in range(world)]
        sig = [[(c["op"], c["count"], c["datatype"], c["root"], c["group_begin"], c["group_end"],
                 c["recv_byte_offset"]) for c in per[r]] for r in range(world)]
        assert all(s == sig[0] for s in sig), f"chunk {k}: ranks issue different collectives"
        b0 = k * world
        blocks = [(int(cuts[b0 + q]), int(cuts[b0 + q + 1])) for q in range(world)]
        nonempty = [q for q, (a, e) in enumerate(blocks) if e > a]
        depth = 0
        for j in range(len(per[0])):
            c0 = per[0][j]
            assert c0["datatype"] == ncdt and c0["count"] > 0
            depth += c0["group_begin"]
            assert depth in (0, 1), "nested or unbalanced group"
            if c0["op"] == L.RCCL_ALLGATHER:
                cnt, recv = c0["count"], c0["recv_byte_offset"]
                assert not broadcast and c0["root"] == -1 and len(per[0]) == 1
                assert all(e - a == cnt for a, e in blocks), "all-gather needs equal blocks"
                assert recv == blocks[0][0] * tsz and recv + world * cnt * tsz == blocks[-1][1] * tsz <= n * tsz
                parts = []
                for r in range(world):
                    send = per[r][j]["send_byte_offset"]
                    assert send == recv + r * cnt * tsz, "in-place all-gather: sendbuff = recvbuff + rank*count"
                    parts.append(ys[r][send:send + cnt * tsz].copy())
                for r in range(world):
                    for q in range(world):
                        ys[r][recv + q * cnt * tsz:recv + (q + 1) * cnt * tsz] = parts[q]
            else:
                assert c0["op"] == L.RCCL_BROADCAST and 0 <= c0["root"] < world
                root, cnt, recv = c0["root"], c0["count"], c0["recv_byte_offset"]
                assert (recv, recv + cnt * tsz) == (blocks[root][0] * tsz, blocks[root][1] * tsz), "root's block"
                for r in range(world):
                    assert per[r][j]["send_byte_offset"] == recv, "in-place broadcast"
                data = ys[root][recv:recv + cnt * tsz].copy()
                for r in range(world):
                    ys[r][recv:recv + cnt * tsz] = data
            depth -= c0["group_end"]
            assert depth in (0, 1)
        assert depth == 0, "a group left open"
        ops = {c["op"] for c in per[0]}
        if ops == {L.RCCL_BROADCAST}:
            assert sorted(c["root"] for c in per[0]) == nonempty, "one broadcast per non-empty block"
        elif nonempty:
            assert ops == {L.RCCL_ALLGATHER}
    for r in range(world):
        assert np.array_equal(ys[r].view(npdt), full), f"rank {r}"


def test_rccl_calls_reject_bad_input():
    import libhpc_amd as L
    with pytest.raises(L.LhpcError):
        L.dist_rccl_calls([0, 5, 3, 8, 9], 2, 2, 0)
    with pytest.raises(L.LhpcError):
        L.dist_rccl_calls([0, 1, 2, 3, 4], 2, 2, 0, dtype=7)
