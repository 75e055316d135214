"""The single-process multi-device plan (SURVEY §8b "Threading": one host
thread, hipSetDevice per device, one stream and one comm per device) through
the drop-in lhpc_spmv_plan_create(…, device_ids, n_devices, …).

The GPU box has one MI355X, so the multi-device paths run with the device
listed several times ([0, 0], [0, 0, 0, 0]): every share gets its own local
plan, stream, comm stream, events and replicas exactly as on distinct
devices; only the peer stores stay on one GPU (over xGMI they are the same
stores) and RCCL (one rank per device) is exercised at one device
(options.multi_force).  Every result is compared bit for bit with the oracle
on dyadic values (exact in any summation order)."""
import numpy as np
import pytest

from tests import _support as S

pytestmark = pytest.mark.gpu


def _problem(lhpc, n, per_row, dt, seed, powerlaw=False):
    if powerlaw:
        rp, col, val = lhpc.gen_powerlaw_csr(n, n, lmax=2000, dtype=dt, dist=1, seed=seed)
    else:
        rp, col, val = lhpc.gen_uniform_csr(n, n, per_row, dtype=dt, dist=1, seed=seed)
    x = lhpc.gen_values(dt, 1, n, seed + 1)
    return rp, col, val, x


CASES = [  # (n, per_row, dtype, powerlaw): 3M columns select XTILE (row-range local plans)
    (3_000_000, 6, "f32", False),
    (20_000, 7, "f64", False),
    (400_000, 0, "f32", True),
]


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0]])
@pytest.mark.parametrize("K", [1, 2, 3])
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}-{c[2]}{'-pl' if c[3] else ''}")
def test_multi_home_and_host_calls(lhpc, gpu, devices, K, case):
    """lhpc_spmv on a multi-device plan: x/y on device_ids[0] (x copied to
    the other shares, their blocks stored back into y) and host buffers;
    three calls each; the plan's cuts are the nnz-balanced D·K split."""
    import torch
    n, per_row, dts, pl = case
    dt = lhpc.F32 if dts == "f32" else lhpc.F64
    rp, col, val, x = _problem(lhpc, n, per_row, dt, 0xB100 + K, pl)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    with lhpc.SpMVPlan(rp, col, val, n, devices=devices, options={"multi_chunks": K}) as plan:
        mi = plan.multi_info()
        assert mi["n_devices"] == len(devices) and mi["chunks"] == K and mi["exchange"] == lhpc.DIST_EXCHANGE_P2P
        assert np.array_equal(mi["cuts"], lhpc.csr_partition_rows(rp, len(devices) * K))
        xd = torch.from_numpy(x).to(gpu)
        for _ in range(3):
            y = torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu)
            plan(xd, y)
            torch.cuda.synchronize()
            assert np.array_equal(y.cpu().numpy(), want)
        for _ in range(2):
            assert np.array_equal(plan(x), want)


@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0]])
@pytest.mark.parametrize("case", CASES[:2], ids=lambda c: f"{c[0]}-{c[2]}")
def test_multi_replicas_iterate(lhpc, gpu, devices, case):
    """lhpc_spmv_multi: full x/y replicas per share; y of call n is x of call
    n+1 (ping-pong, four calls, no host synchronisation between them: the
    READY / push events are the only ordering between the shares); every
    share's y equals the oracle's iterate bit for bit."""
    import torch
    n, per_row, dts, _ = case
    dt = lhpc.F32 if dts == "f32" else lhpc.F64
    rp, col, val, x = _problem(lhpc, n, per_row, dt, 0xB200, False)
    steps, D = 4, len(devices)
    want, cur = [], x
    for _ in range(steps):
        _, cur, _ = S.spmv_oracle(rp, col, val, cur)
        want.append(cur)
    with lhpc.SpMVPlan(rp, col, val, n, devices=devices, options={"multi_chunks": 2}) as plan:
        xd = torch.from_numpy(x).to(gpu)
        a = [xd.clone() for _ in range(D)]
        b = [torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu) for _ in range(D)]
        streams = [torch.cuda.Stream(gpu) for _ in range(D)]
        torch.cuda.synchronize()
        snaps = []
        for it in range(steps):
            src, dst = (a, b) if it % 2 == 0 else (b, a)
            plan.multi(src, dst, streams)
            # snapshot every replica on the last share's stream once every
            # share's stream has passed the call; the next call starts after
            # the snapshot (stream order only, no host synchronisation)
            for d in range(D):
                streams[D - 1].wait_stream(streams[d])
            with torch.cuda.stream(streams[D - 1]):
                snaps.append([t.clone() for t in dst])
            for d in range(D - 1):
                streams[d].wait_stream(streams[D - 1])
        torch.cuda.synchronize()
    for it in range(steps):
        for d in range(D):
            assert np.array_equal(snaps[it][d].cpu().numpy(), want[it]), (it, d)


def test_multi_own_push_before_later_writes(lhpc, gpu):
    """share d's stream passes lhpc_spmv_multi only after its
    OWN push (which reads y[d] to copy d's blocks into the peers' replicas)
    has finished, so a write to y[d] queued on that stream right after the
    call cannot corrupt the peers' replicas."""
    import torch
    n, D = 3_000_000, 3
    rp, col, val, x = _problem(lhpc, n, 6, lhpc.F32, 0xB250)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    with lhpc.SpMVPlan(rp, col, val, n, devices=[0] * D, options={"multi_chunks": 2}) as plan:
        xd = torch.from_numpy(x).to(gpu)
        a = [xd.clone() for _ in range(D)]
        streams = [torch.cuda.Stream(gpu) for _ in range(D)]
        for it in range(3):
            src = it % D  # the share whose y is overwritten
            b = [torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu) for _ in range(D)]
            torch.cuda.synchronize()
            plan.multi(a, b, streams)
            with torch.cuda.stream(streams[src]):
                b[src].fill_(-1.0)  # right after the call, on that share's stream only
            torch.cuda.synchronize()
            for d in range(D):
                if d != src:
                    assert np.array_equal(b[d].cpu().numpy(), want), (src, d)


@pytest.mark.parametrize("exchange", ["p2p", "rccl"])
@pytest.mark.parametrize("K", [1, 2])
def test_multi_one_device_forced(lhpc, gpu, exchange, K):
    """n_devices = 1 through the multi-device code path (options.multi_force):
    the P2P form and the RCCL form (ncclCommInitAll over the one device, a
    group all-gather per chunk — in place, so y must come out unchanged)."""
    import torch
    n = 3_000_000
    rp, col, val, x = _problem(lhpc, n, 5, lhpc.F32, 0xB300 + K)
    _, want, _ = S.spmv_oracle(rp, col, val, x)
    ex = lhpc.DIST_EXCHANGE_RCCL if exchange == "rccl" else lhpc.DIST_EXCHANGE_P2P
    with lhpc.SpMVPlan(rp, col, val, n, devices=[0],
                       options={"multi_force": 1, "multi_chunks": K, "multi_exchange": ex}) as plan:
        assert plan.multi_info()["exchange"] == ex
        xd = torch.from_numpy(x).to(gpu)
        y = torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu)
        plan(xd, y)
        torch.cuda.synchronize()
        assert np.array_equal(y.cpu().numpy(), want)
        y2 = torch.full((n,), float("nan"), dtype=xd.dtype, device=gpu)
        plan.multi([xd], [y2])
        torch.cuda.synchronize()
        assert np.array_equal(y2.cpu().numpy(), want)


def test_multi_rccl_needs_distinct_devices(lhpc, gpu):
    rp, col, val, x = _problem(lhpc, 1000, 5, lhpc.F32, 0xB400)
    with pytest.raises(lhpc.LhpcError) as e:
        lhpc.SpMVPlan(rp, col, val, 1000, devices=[0, 0], options={"multi_exchange": lhpc.DIST_EXCHANGE_RCCL})
    assert e.value.status == -5  # LHPC_ERR_UNSUPPORTED


def test_multi_cg_matches_single_device(lhpc, gpu):
    """lhpc_cg_solve on a two-share plan (its SpMV runs through the home
    path) converges like the single-device solve: same iteration count and x
    within 1e-8 of the fp64 oracle CG."""
    import torch
    ny = nx = 96
    rp, col, val = S.laplacian_2d(ny, nx)
    b = np.random.default_rng(0xB500).uniform(-1, 1, ny * nx)
    want_x, want_it, _ = S.cg_oracle(rp, col, val, b, tol=1e-10, max_iter=2000)
    for devices in (None, [0, 0]):
        with lhpc.SpMVPlan(rp, col, val, ny * nx, devices=devices) as plan:
            x, it, res = lhpc.cg(plan, torch.from_numpy(b).to(gpu), tol=1e-10, max_iter=2000)
            assert abs(it - want_it) <= 1 and res <= 1e-10
            x = x.cpu().numpy()
            assert np.linalg.norm(x - want_x) <= 1e-8 * np.linalg.norm(want_x)
