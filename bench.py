"""bench.py — CSR SpMV throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c2|c3|c4|c5|blur_x|blur_y|sort|cg]

N=1: BASELINE configs[1] — CSR SpMV, n=10M, nnz=150M (exactly 15 uniform
distinct sorted columns per row), fp32 values/x/y, A and x resident in HBM.
N>1 (one rank per GPU; `python bench.py --gpus N` without a launcher starts
torch.distributed.run with N ranks itself, as a child process, and refuses
when N disagrees with the launcher's WORLD_SIZE or exceeds the visible GPUs
outside the LHPC_DIST_BACKEND=gloo rehearsal — launch_decision): the SAME matrix is
split into N·K nnz-balanced interleaved row blocks, K = --chunks per rank
(strong scaling); a step is the rank's local SpMV plus the y exchange over
xGMI that makes y the next x, chunk k's exchange overlapping chunk k+1's
reduce.  The native path (lhpc_dist_*) times both exchanges in the same run —
RCCL collectives (backend "nccl" = RCCL) and direct peer stores into every
rank's registered y window — plus SpMV-only and exchange-only steps, and
reports the faster exchange whose y equals the RCCL one.

One step = one y = A·x over the whole matrix.  W untimed warmup steps, then
exactly K timed steps between barrier + device synchronize; the max over ranks
is reported.  value = 2·nnz·K / time (GFLOP/s, whole job).

Extra objects on the JSON line:
  roofline      the SpMV call on rank 0 (XTILE for C2-C4 = k_xtile_gather +
                k_xtile_reduce (+ k_xtile_fixup)):
                achieved = algorithmic bytes per call (nnz·(4+4) + (n+1)·4 +
                2·n·4 for fp32, x counted once) ÷ average call time from HIP
                events on the launch stream; peak 8.0 TB/s; traffic = PMC
                fabric bytes per call from profiles/traffic.json (or null);
                layout = the same call against the bytes the XTILE layout
                streams.
  cpu_baseline  rank 0, N=1 only: the AVX2 + OpenMP CSR SpMV of oracle/ (the
                reference has no CPU SpMV) on the same matrix, timed
                for ~10 s on the box's host cores (OpenMP placement and host
                CPU / NUMA nodes recorded in the object).

--workload sort (not the headline): the reference's only
published GPU number — radix sort of 500M uint32 keys (README.md:52, ~360 ms
on an RTX 3080 Ti Laptop = 1.39 G keys/s) — on lhpc_radix_sort_u32; each step
sorts a fresh copy of the same random keys (the restore copy is outside the
timed events); cpu_baseline = the reference's own CPU radix sort
(oracle/_ref/libref_sort.so, kind "reference").

--workload cg: conjugate gradient on the 4096² 2-D
Laplacian in fp64 (16.8M rows, 83.9M nnz); a step = one CG iteration
(SpMV + 2 all-reduced dots + the fused vector updates).  N=1 runs the
native lhpc_cg_solve (10-iteration blocks replayed as HIP graphs); N>1 over
RCCL runs the native lhpc_dist_cg_solve (K chunks per rank, p's exchange
chained into the next q = A·p), and the torch.distributed DistCG only under
gloo or LHPC_DIST_TORCH=1.
"""
import argparse
import json
import os
import sys
import time

# CPU-baseline thread placement: set before anything loads an
# OpenMP runtime, so the oracle's libgomp reads it at initialisation
os.environ.setdefault("OMP_PROC_BIND", "close")
os.environ.setdefault("OMP_PLACES", "cores")


def _process_cpus():
    """The process's CPU set, read from /proc/self/status before any OpenMP
    runtime loads: once libgomp has bound the master thread (OMP_PROC_BIND),
    sched_getaffinity(0) reports that thread's place, not the process's set."""
    try:
        for line in open("/proc/self/status"):
            if line.startswith("Cpus_allowed_list:"):
                cpus = set()
                for part in line.split(":", 1)[1].strip().split(","):
                    if part:
                        lo, _, hi = part.partition("-")
                        cpus.update(range(int(lo), int(hi or lo) + 1))
                return sorted(cpus)
    except OSError:
        pass
    try:
        return sorted(os.sched_getaffinity(0))
    except AttributeError:
        return list(range(os.cpu_count() or 1))


PROCESS_CPUS = _process_cpus()

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import step_model  # noqa: E402  (tools/step_model.py: the N > 1 step model, pure Python)

METRIC = "CSR SpMV GFLOP/s + achieved HBM GB/s, n=10M nnz=150M, at 1/2/4/8 MI355X"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def parse_options(text):
    """--spmv-options: a JSON dict, or k=v[,k=v] (integers) — the form that
    survives shell quoting in tools/gpu.sh steps."""
    if text is None or text.strip().startswith("{"):
        return json.loads(text) if text else None
    return {k.strip(): int(v) for k, v in (kv.split("=", 1) for kv in text.split(",") if kv.strip())}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "blur_x", "blur_y", "sort", "cg"])
    ap.add_argument("--n", "--n-rows", dest="n", type=int, default=10_000_000,
                    help="rows = columns (--n-rows under torch.distributed.run, whose parser takes --n as a prefix)")
    ap.add_argument("--per-row", type=int, default=15)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--chunks", type=int, default=0,
                    help="N>1: row chunks per rank K (exchange overlap).  0 (default): the native path measures "
                         "K = 1, 2, 4 and reports the fastest (the step model, tools/step_model.py, puts K = 4 "
                         "first at 64 GB/s per xGMI link, DESIGN.md §6.3); other paths use 4")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="N=1: run the step back to back for this long before the W warmup steps (0: off) — the "
                         "device's clocks ramp over the first ~10-15 ms of sustained load after an idle gap "
                         "(round 5: C2 call 479-483 -> 462-465 us on one box, 462 -> 435 on another, profiles/r05/ramp*.jsonl; 40 ms "
                         "of settle left part of it, 100 ms all of it); reported as `settle`")
    ap.add_argument("--no-alt-kernels", action="store_true",
                    help="skip the other kernel families' C2-C4 times (alt_kernels: ADAPTIVE, ROWGROUP, XSLICE)")
    ap.add_argument("--spmv-options", default=None, type=parse_options,
                    help="lhpc_options fields for the 1-GPU SpMV plan (measured alternatives, DESIGN.md §4): a JSON "
                         "dict or k=v[,k=v] with integer values")
    ap.add_argument("--dtype", default="auto", choices=["auto", "f32", "f64"],
                    help="SpMV value type (auto: the config's own — fp64 for c1/c3, fp32 for c2/c4; "
                         "SURVEY §8d also runs C4 in fp64)")
    return ap.parse_args()


def cpu_threads():
    """OMP_NUM_THREADS (the box sets 16), capped at the process's CPU set:
    more threads than CPUs would only time-slice."""
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() and int(env) > 0 else len(PROCESS_CPUS)
    return max(1, min(n, len(PROCESS_CPUS)))


def load_traffic(kernel_tag):
    """PMC-measured HBM bytes per call, committed under profiles/ by
    tools/pmc_traffic.py (FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected)."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get(kernel_tag, {}).get("bytes_per_call")
    except Exception:
        return None


def settle(fn, torch, ms, end=None):
    """Keep the device busy with `fn` (one step) for `ms` milliseconds before
    the warmup, so the timed steps do not straddle the clock ramp that
    follows an idle gap (host-side setup: data generation, plan builds,
    layout checks).  Untimed; the W warmup and K timed steps are unchanged.
    N = 1 only (a time-based loop would give ranks different step counts);
    the N > 1 paths time their exchange candidates just before the headline
    loop, which keeps the devices under load."""
    if ms <= 0:
        return {"ms": 0.0, "steps": 0}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    while (time.perf_counter() - t0) * 1e3 < ms:
        fn()
        n += 1
        if n % 16 == 0:
            torch.cuda.synchronize()  # keep the host within a few steps of the device
    if end is not None:
        end()
    torch.cuda.synchronize()
    return {"ms": (time.perf_counter() - t0) * 1e3, "steps": n,
            "why": "device clocks ramp over the first ~10-15 ms of sustained load after an idle gap "
                   "(DESIGN.md §5, profiles/r05/ramp.jsonl); untimed, before the W warmup steps"}


def launch_decision(gpus, env, visible, argv, port=0):
    """What `bench.py --gpus N` does in this process, decided before any GPU
    call:  ("run", None) — this process is a rank (or N = 1);
    ("spawn", cmd) — N > 1 with no launcher: start torch.distributed.run with
    N ranks as a CHILD process running the same arguments (never exec: the
    parent has imported torch); ("refuse", message) — N disagrees with the
    launcher's WORLD_SIZE, or N exceeds the visible GPUs outside the gloo
    rehearsal (LHPC_DIST_BACKEND=gloo: ranks may share a GPU)."""
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "refuse", f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks"
        return "run", None
    if gpus <= 1:
        return "run", None
    if gpus > visible and env.get("LHPC_DIST_BACKEND", "nccl") != "gloo":
        return "refuse", (f"bench.py: --gpus {gpus} but {visible} GPU(s) visible; one rank per GPU "
                          "(set LHPC_DIST_BACKEND=gloo to rehearse ranks sharing a GPU)")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py")] + list(argv)
    return "spawn", cmd


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    args = parse()
    import torch
    # N > 1 without a launcher: N ranks through torch.distributed.run, as a
    # child process (device_count() does not initialise the GPU on this image)
    action, what = launch_decision(args.gpus, os.environ, torch.cuda.device_count(), sys.argv[1:], free_port())
    if action == "refuse":
        print(what, file=sys.stderr, flush=True)
        raise SystemExit(2)
    if action == "spawn":
        import subprocess
        env = dict(os.environ)
        if env.get("LHPC_DIST_BACKEND") == "gloo":
            env.setdefault("LHPC_DIST_P2P", "1")  # the native peer-store path, as on a node
        print(f"bench.py: --gpus {args.gpus}: {' '.join(what)}", file=sys.stderr, flush=True)
        rc = subprocess.run(what, env=env).returncode  # rank 0 prints the JSON line to our stdout
        raise SystemExit(rc)
    import torch.distributed as dist
    import libhpc_amd as L

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; the modulo only matters for the 1-GPU rehearsal of the
    # N>1 path (LHPC_DIST_BACKEND=gloo, ranks sharing cuda:0) — identity on a full node
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # LHPC_DIST_NATIVE=1 under torch.distributed.run with one process: the
    # native N > 1 path at world 1 (the rehearsal a 1-GPU box allows; RCCL
    # cannot place two ranks on one GPU)
    force_native = os.environ.get("LHPC_DIST_NATIVE", "0") == "1" and "RANK" in os.environ
    if world > 1 or force_native:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = os.environ.get("LHPC_DIST_BACKEND", "nccl")  # nccl = RCCL over xGMI
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    stream = torch.cuda.current_stream(dev)
    # N > 1 over RCCL: the native lhpc_dist_* path (one RCCL communicator and
    # comm stream per process, created from rank 0's unique id); the
    # torch.distributed form serves the gloo rehearsal or LHPC_DIST_TORCH=1.
    # The native path times both y exchanges (RCCL collectives and direct
    # xGMI peer stores into every rank's registered y window) in the same
    # run, plus SpMV-only and exchange-only steps, and reports the faster
    # exchange as the headline.  With the gloo backend (ranks
    # sharing one GPU in a rehearsal) only the peer exchange exists, over an
    # RCCL-free local communicator.
    native_dist = (world > 1 or force_native) and (
        dist.get_backend() == "nccl" and os.environ.get("LHPC_DIST_TORCH", "0") != "1"
        or os.environ.get("LHPC_DIST_P2P", "0") == "1")

    def timed(fn, steps, warmup):
        """max-over-ranks seconds per step of fn: W untimed calls, then
        `steps` calls bracketed by barrier + synchronize."""
        for _ in range(warmup):
            fn()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        barrier()
        el = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el / steps
    wl = args.workload
    result = {}
    step_end = None  # chained N > 1 steps: the call that waits for the last exchange
    if wl in ("c1", "c2", "c3", "c4"):
        dt = L.F64 if wl in ("c1", "c3") else L.F32
        if args.dtype != "auto":
            dt = L.F64 if args.dtype == "f64" else L.F32
        dtag = "" if dt == (L.F64 if wl in ("c1", "c3") else L.F32) else ("f64" if dt == L.F64 else "f32")
        tsz = 8 if dt == L.F64 else 4
        n = 100_000 if wl == "c1" else args.n
        t0 = time.time()
        if wl == "c4":
            rp, col, val = L.gen_powerlaw_csr(n, n, dtype=dt)
        else:
            rp, col, val = L.gen_uniform_csr(n, n, 10 if wl == "c1" else args.per_row, dtype=dt)
        x = L.gen_values(dt, 0, n, L.SEED_X)
        nnz = int(col.shape[0])
        t_gen = time.time() - t0
        from libhpc_amd.dist import DistSpMVOverlap, InterleavedBlocks
        xd = torch.from_numpy(x).to(dev)
        t0 = time.time()
        if world == 1 and not native_dist:
            plans = [L.SpMVPlan(rp, col, val, n,
                                options=args.spmv_options)]
            local_nnz, local_rows = nnz, n
            y_local = torch.empty(n, dtype=xd.dtype, device=dev)

            def step():
                plans[0](xd, y_local, stream=stream)
        elif native_dist:
            # native path behind the C ABI (lhpc_dist_spmv): nnz-balanced
            # interleaved blocks, K chunks per rank; chunk k is reduced into
            # the rank's rows of y and exchanged on the comm stream while
            # chunk k+1 is reduced.  One plan per exchange kind (the kind is
            # a plan option), each over the same local rows.
            has_rccl = dist.get_backend() == "nccl"
            comm = L.DistComm.from_torch(local) if has_rccl else L.DistComm.local(world, rank, local)
            xnotes = {}
            y_p2p = torch.empty(n, dtype=xd.dtype, device=dev)
            y_p2p_b = torch.empty(n, dtype=xd.dtype, device=dev)  # second window: chained ping-pong
            y_full = torch.empty(n, dtype=xd.dtype, device=dev)
            y_full_b = torch.empty(n, dtype=xd.dtype, device=dev)
            ybuf = {"rccl": y_full, "p2p": y_p2p, "none": y_full}
            ybuf_b = {"rccl": y_full_b, "p2p": y_p2p_b}

            def agree(ok):  # every rank takes the same branch (no half-set-up exchange)
                f = torch.tensor([1 if ok else 0], dtype=torch.int32,
                                 device=dev if dist.get_backend() == "nccl" else "cpu")
                dist.all_reduce(f, op=dist.ReduceOp.MIN)
                return bool(f.item())
            # the peer windows (y buffers registered on every rank) serve every K
            p2p_ok = False
            if world > 1:
                try:
                    comm.p2p_setup_torch(y_p2p)  # collective-safe: raises on every rank or none
                    comm.p2p_setup_torch(y_p2p_b)
                    p2p_ok = True
                except Exception as e:  # e.g. no IPC between the ranks' devices
                    xnotes["p2p"] = f"unavailable: {e}"
                p2p_ok = agree(p2p_ok)

            def timed_chain(dp, ya, yb, steps, warmup):
                """Iterative use (y of step n is x of step n+1, ping-pong
                buffers): lhpc_dist_spmv_begin per step, so each step's tile
                gather starts by column part as soon as the exchange that
                delivers it has landed (cross-step overlap); one end per run,
                inside the timed region."""
                bufs = [ya, yb]
                ya.copy_(xd)
                cur = [0]

                def one():
                    dp.begin(bufs[cur[0]], bufs[cur[0] ^ 1], stream=stream)
                    cur[0] ^= 1
                for _ in range(warmup):
                    one()
                dp.end(stream=stream)
                barrier()
                t0 = time.perf_counter()
                for _ in range(steps):
                    one()
                dp.end(stream=stream)
                barrier()
                el = time.perf_counter() - t0
                if world > 1:
                    tt = torch.tensor([el], dtype=torch.float64, device=dev)
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                    el = float(tt.item())
                return el / steps

            def measure_k(K):
                """Plans over K chunks per rank (one per exchange kind: the kind
                is a plan option) and their times: end-to-end (plain and
                chained), exchange-only, SpMV-only."""
                cuts = L.interleaved_cuts(rp, world, K)
                lrp, lc, lv = L.interleaved_local_csr(rp, col, val, cuts, world, K, rank)
                dpl, notes = {}, {}
                if has_rccl:
                    dpl["rccl"] = L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv,
                                                 options={"dist_exchange": L.DIST_EXCHANGE_RCCL,
                                                          "dist_world1": 1 if world == 1 else 0})
                if p2p_ok:
                    # the peer exchange is an optimisation: if a short probe fails
                    # on any rank (a flag wait timing out), every rank drops it and
                    # the RCCL exchange is still measured.  The probe calls hold no
                    # collective, and every flag wait is bounded, so all ranks
                    # reach the agreement.
                    pp, ok = None, True
                    try:
                        pp = L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv,
                                            options={"dist_exchange": L.DIST_EXCHANGE_P2P})
                        for _ in range(3):
                            pp(xd, y_p2p, stream=stream)
                        torch.cuda.synchronize()
                        ok = comm.p2p_status() == 0
                        if not ok:
                            notes["p2p"] = "probe: a flag wait timed out"
                    except Exception as e:
                        ok, notes["p2p"] = False, f"probe failed: {e}"
                    if agree(ok):
                        dpl["p2p"] = pp
                    else:
                        notes.setdefault("p2p", "probe failed on another rank")
                        torch.cuda.synchronize()
                        if pp is not None:
                            pp.close()
                dpl["none"] = L.DistSpMVPlan(comm, n, n, K, cuts, lrp, lc, lv,
                                             options={"dist_exchange": L.DIST_EXCHANGE_NONE})
                xt = {}
                for kx in [k for k in ("rccl", "p2p") if k in dpl]:
                    dp, yb = dpl[kx], ybuf[kx]
                    e2e = timed(lambda dp=dp, yb=yb: dp(xd, yb, stream=stream), args.steps, args.warmup)
                    xo = timed(lambda dp=dp, yb=yb: dp.exchange(yb, stream=stream), args.steps, args.warmup)
                    ch = timed_chain(dp, yb, ybuf_b[kx], args.steps, args.warmup)
                    # chained calls must give what two plain calls give (every rank
                    # agrees); the plan's own y buffers (P2P plans need windows)
                    ybb = ybuf_b[kx]
                    dp(xd, yb, stream=stream)
                    dp(yb, ybb, stream=stream)
                    ref2 = ybb.clone()
                    ybb.copy_(xd)
                    dp.begin(ybb, yb, stream=stream)
                    dp.begin(yb, ybb, stream=stream)
                    dp.end(stream=stream)
                    same = torch.tensor([1 if torch.equal(ref2, ybb) else 0], dtype=torch.int32, device=dev)
                    if world > 1:
                        dist.all_reduce(same, op=dist.ReduceOp.MIN)
                    xt[kx] = {"step_ms": e2e * 1e3, "exchange_only_ms": xo * 1e3,
                              "gflops": 2.0 * nnz / e2e / 1e9, "chained_step_ms": ch * 1e3,
                              "chained_gflops": 2.0 * nnz / ch / 1e9, "chained_same_y": bool(same.item())}
                so = timed(lambda: dpl["none"](xd, y_full, stream=stream), args.steps, args.warmup)
                # the peer exchange competes only with a y identical on every rank
                # to the RCCL one (read on the device, through this GPU's caches)
                if "p2p" in xt and "rccl" in xt:
                    dpl["rccl"](xd, y_full, stream=stream)
                    dpl["p2p"](xd, y_p2p, stream=stream)
                    same = torch.tensor([1 if torch.equal(y_full, y_p2p) else 0], dtype=torch.int32, device=dev)
                    dist.all_reduce(same, op=dist.ReduceOp.MIN)
                    xt["p2p"]["same_y_as_rccl"] = bool(same.item())
                    if not same.item():
                        xt["p2p"]["excluded"] = "y differs from the RCCL exchange"
                # per exchange: the faster of plain and chained (chained only when
                # it gave the plain calls' y)
                best = None
                for kx, r in xt.items():
                    if "excluded" in r:
                        continue
                    for mode in ("plain", "chained"):
                        if mode == "chained" and not r["chained_same_y"]:
                            continue
                        t = r["chained_step_ms" if mode == "chained" else "step_ms"]
                        if best is None or t < best[2]:
                            best = (kx, mode == "chained", t)
                return {"K": K, "plans": dpl, "xtimes": xt, "notes": notes, "spmv_only_ms": so * 1e3,
                        "best": best, "local": (lrp, lc, lv)}

            # K (chunks per rank) is measured, not assumed: the exchange overlap
            # it buys against the per-chunk launch cost depends on the link rate
            # (tools/step_model.py); --chunks N fixes it
            kcands = [args.chunks] if args.chunks > 0 else [1, 2, 4]

            def strip(r):
                return {k: v for k, v in r.items() if k not in ("plans", "local")}
            top, others = None, []
            for K in kcands:
                r = measure_k(K)
                torch.cuda.synchronize()
                if top is None or (r["best"] is not None and (top["best"] is None or r["best"][2] < top["best"][2])):
                    if top is not None:  # the new fastest K: the previous one's plans go
                        for dp in top["plans"].values():
                            dp.close()
                        others.append(strip(top))
                    top = r
                else:
                    for dp in r["plans"].values():
                        dp.close()
                    others.append(strip(r))
            n_chunks = top["K"]
            dplans, xtimes = top["plans"], top["xtimes"]
            xnotes.update(top["notes"])
            lrp, lc, lv = top["local"]
            spmv_only = top["spmv_only_ms"] * 1e-3
            chosen, chained = (top["best"][0], top["best"][1]) if top["best"] else ("none", False)
            dplan = dplans[chosen]
            y_out_buf = ybuf[chosen]
            # the same local rows as one plan: the live kernel-only call timing below
            plans = [L.SpMVPlan(lrp, lc, lv, n)]
            local_nnz, local_rows = int(lc.shape[0]), int(lrp.shape[0] - 1)
            exchange_report = {"chosen": chosen, "chained": chained, "chunks_per_rank": n_chunks,
                               "spmv_only_ms": spmv_only * 1e3, **xtimes, **xnotes,
                               "other_chunk_counts": [{"K": r["K"], "spmv_only_ms": r["spmv_only_ms"],
                                                       "best": r["best"], **r["xtimes"]} for r in others],
                               "note": "step = local SpMV + y exchange (lhpc_dist_spmv); chained = iterative use, "
                                       "y of step n is x of step n+1, lhpc_dist_spmv_begin (next step's gather by "
                                       "column part as each exchange lands); exchange_only = lhpc_dist_exchange "
                                       "alone; spmv_only = exchange NONE; max over ranks; chunks_per_rank = the "
                                       "fastest of the measured K (other_chunk_counts)"}
            if world > 1 and chosen in xtimes:
                # the step model (tools/step_model.py) at this run's own numbers:
                # measured receive / per-link rate from the exchange-only time, and
                # the step it predicts beside the measured one.
                # The stage (the x tile gather) alone, from a two-range plan of
                # the same local rows; 0.45 of the local call when that plan
                # cannot be built (not XTILE)
                stage_ms, stage_src = 0.45 * spmv_only * 1e3, "0.45 of spmv_only (no split plan)"
                if local_rows >= 2:
                    try:
                        with L.SpMVPlan(lrp, lc, lv, n, splits=[local_rows // 2]) as sp:
                            stage_ms = timed(lambda: sp.stage(xd, stream=stream), args.steps, args.warmup) * 1e3
                            stage_src = "measured (lhpc_spmv_stage of the rank's rows)"
                    except L.LhpcError:
                        pass
                xr = xtimes[chosen]
                exchange_report["model"] = dict(
                    step_model.exchange_model(world, n_chunks, chained, n, tsz, stage_ms, spmv_only * 1e3,
                                              xr["exchange_only_ms"],
                                              xr["chained_step_ms" if chained else "step_ms"]),
                    stage_source=stage_src, exchange=chosen)

            class _Native:
                def step(self, xv):
                    return dplan(xv, y_out_buf, stream=stream)
            dsp = _Native()
            if chained:
                ch_bufs = [y_out_buf, ybuf_b[chosen]]
                ch_bufs[0].copy_(xd)
                ch_cur = [0]

                def step():
                    dplan.begin(ch_bufs[ch_cur[0]], ch_bufs[ch_cur[0] ^ 1], stream=stream)
                    ch_cur[0] ^= 1

                def step_end():
                    dplan.end(stream=stream)
            else:
                def step():
                    dplan(xd, y_out_buf, stream=stream)
        else:
            # torch.distributed form (gloo rehearsal, LHPC_DIST_TORCH=1):
            # interleaved nnz-balanced row blocks, K chunks per rank; chunk
            # k's all-gather overlaps the SpMV of chunk k+1 (libhpc_amd/dist.py)
            n_chunks = args.chunks if args.chunks > 0 else 4
            ib = InterleavedBlocks(n, world, n_chunks, row_ptr=rp)
            plans, local_nnz, fns = [], 0, None
            if n_chunks > 1:
                # one row-range plan over the rank's K chunks: x is staged once
                # (one XTILE tile gather), then chunk k is reduced and its
                # all-gather starts; falls back to a plan per chunk when the
                # matrix does not select XTILE
                lrp, lc, lv, splits = ib.local_csr_all(rp, col, val, rank)
                try:
                    sp = L.SpMVPlan(lrp, lc, lv, n, splits=splits)
                except L.LhpcError:
                    sp = None
                if sp is not None:
                    plans, local_nnz = [sp], int(lc.shape[0])

                    def first(xv, yv, pl=sp):
                        pl.stage(xv, stream=stream)
                        pl.range(0, yv, stream=stream)
                    fns = [first] + [lambda xv, yv, k=k, pl=sp: pl.range(k, yv, stream=stream)
                                     for k in range(1, n_chunks)]
            if fns is None:
                for k in range(n_chunks):
                    lrp, lc, lv = ib.local_csr(rp, col, val, rank, k)
                    plans.append(L.SpMVPlan(lrp, lc, lv, n))
                    local_nnz += int(lc.shape[0])
                fns = [lambda xv, yv, pl=pl: pl(xv, yv, stream=stream) for pl in plans]
            local_rows = ib.B * n_chunks
            dsp = DistSpMVOverlap(ib, fns, like=xd)

            def step():
                dsp.step(xd)
        t_plan = time.time() - t0
        info = plans[0].info()
        t_plan_dev = None
        if world == 1 and not native_dist and info["kernel"] == L.KERNEL_XTILE and wl in ("c2", "c3", "c4"):
            # the same plan from device-resident CSR (LHPC_PLAN_DEVICE_INPUT:
            # the XTILE layout built on the GPU), timed beside the host build
            drp, dcol, dval = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))
            torch.cuda.synchronize()
            t0 = time.time()
            pdev = L.SpMVPlan(drp, dcol, dval, n,
                              options=args.spmv_options)
            t_plan_dev = time.time() - t0
            try:
                same = pdev.layout_digest() == plans[0].layout_digest()
            except L.LhpcError:  # row-part plans (nnz past the int32 stream) have no single layout
                same = None
            pdev.close()
            del drp, dcol, dval
            torch.cuda.empty_cache()

        if step_end is None:
            step_end = lambda: None  # noqa: E731
        settled = settle(step, torch, args.settle_ms if world == 1 else 0.0, step_end)
        for _ in range(args.warmup):
            step()
        step_end()
        barrier()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t_wall0 = time.perf_counter()
        ev0.record(stream)
        for i in range(args.steps):
            step()
        step_end()  # chained steps: the last exchange, inside the timed region
        ev1.record(stream)
        barrier()
        t_wall = time.perf_counter() - t_wall0
        # the per-step distribution (median of per-rep timings) in a
        # second pass with an event at every step boundary, outside the timed
        # region: a timing event between two calls leaves the GPU idle ≈ 6 µs
        # (rocprof trace, round 5), which the headline run must not carry
        sev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
        for i in range(args.steps):
            sev[i].record(stream)
            step()
        step_end()
        sev[args.steps].record(stream)
        barrier()
        step_ms = np.array([sev[i].elapsed_time(sev[i + 1]) for i in range(args.steps)])
        t_ev = ev0.elapsed_time(ev1) * 1e-3
        elapsed = max(t_wall, t_ev)
        timing = {"wall_s": t_wall, "events_s": t_ev, "value_from": "wall" if t_wall >= t_ev else "events"}
        if world > 1:
            tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        per_step = elapsed / args.steps
        gflops = 2.0 * nnz / per_step / 1e9
        alg_bytes = nnz * (tsz + 4) + (n + 1) * 4 + 2 * n * tsz
        # live SpMV-call timing on rank 0's launch stream (kernel-only, no collective)
        kev0 = torch.cuda.Event(enable_timing=True)
        kev1 = torch.cuda.Event(enable_timing=True)
        reps = max(args.steps, 10)
        barrier()
        ysc = torch.empty(max(pl.n_rows for pl in plans), dtype=xd.dtype, device=dev)
        kev0.record(stream)
        for _ in range(reps):
            for pl in plans:
                pl(xd, ysc[:pl.n_rows], stream=stream)
        kev1.record(stream)
        torch.cuda.synchronize()
        call_loop_s = kev0.elapsed_time(kev1) * 1e-3 / reps
        # N = 1: the call time is the timed region's own (HIP events on the
        # launch stream around exactly the K timed steps); N > 1 steps hold the
        # exchange too, so there the kernel-only loop above gives the call
        call_s = t_ev / args.steps if (world == 1 and not native_dist) else call_loop_s
        local_alg = local_nnz * (tsz + 4) + (local_rows + len(plans)) * 4 + (n + local_rows) * tsz
        achieved = local_alg / call_s / 1e9
        kname = {L.KERNEL_XSLICE: "xslice", L.KERNEL_ROWGROUP: "rowgroup", L.KERNEL_ADAPTIVE: "adaptive",
                 L.KERNEL_XTILE: "xtile", L.KERNEL_SELL: "sell"}[info["kernel"]]
        kernels = {"xslice": "k_spmv_xslice+k_xslice_reduce", "rowgroup": "k_spmv_rowgroup",
                   "adaptive": "k_spmv_adaptive", "sell": "k_spmv_sell",
                   "xtile": "k_xtile_gather+k_xtile_reduce" + ("+k_xtile_fixup" if info["n_long_rows"] else "")}[kname]
        traffic = load_traffic(f"{wl}{dtag}_{kname}") if world == 1 else None
        result.update(
            metric=METRIC if wl != "c1" else "CSR SpMV GFLOP/s, n=100k nnz=1M fp64 (BASELINE configs[0])",
            value=gflops, unit="GFLOP/s", n_gpus=world, steps=args.steps,
            warmup=args.warmup, ms_per_step=per_step * 1e3, higher_is_better=True,
            scaling="strong", vs_baseline=None, dtype="f64" if dt == L.F64 else "f32",
            data="synthetic: deterministic splitmix64 CSR (SURVEY §8d seeds), A/x resident in HBM",
            config={"workload": {"c1": "BASELINE configs[0]: CSR SpMV n=100k nnz=1M fp64 uniform 10/row (CPU config; "
                                       "GPU time beside the 1-thread SIMD baseline)",
                                 "c2": "BASELINE configs[1]: CSR SpMV n=10M nnz=150M fp32 uniform 15/row",
                                 "c3": "BASELINE configs[2] matrix: CSR SpMV n=10M nnz=150M fp64 uniform 15/row",
                                 "c4": "BASELINE configs[3]: power-law CSR (1..1e4 nnz/row) fp32"}[wl]
                    + (f" (run in {dtag})" if dtag else ""),
                    "n_rows": n, "n_cols": n, "nnz": nnz, "kernel": kname, "slices": info["slices"],
                    "parallelism": f"row-block x{world}" + (
                        f" (interleaved nnz-balanced, {n_chunks} chunks/rank) + "
                        + ("direct xGMI peer stores of y chunks (lhpc_dist_p2p windows)" if chosen == "p2p" else
                           "native RCCL exchange of y chunks (in-place all-gather for equal blocks, else "
                           "broadcasts)" if chosen == "rccl" else "no exchange")
                        + (" (lhpc_dist_spmv_begin, chained: y of step n is x of step n+1, next gather by column "
                           "part under the exchange)" if chained else " (lhpc_dist_spmv)")
                        + " overlapped; faster of the measured exchanges" if native_dist else
                        f" (interleaved nnz-balanced, {n_chunks} chunks/rank) + torch.distributed all_gather(y) "
                        "overlapped" if world > 1 else "")},
            achieved_GBps=alg_bytes / per_step / 1e9,
            roofline={"bound": "hbm", "kernel": kernels, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                      "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS, "traffic": traffic,
                      "alg_bytes_per_call": local_alg, "call_us": call_s * 1e6,
                      "call_us_source": "HIP events over the timed region" if (world == 1 and not native_dist)
                      else "kernel-only loop of the rank's local calls", "call_us_kernel_loop": call_loop_s * 1e6},
            timing=timing, settle=settled,
            step_ms={"median": float(np.median(step_ms)), "p10": float(np.percentile(step_ms, 10)),
                     "p90": float(np.percentile(step_ms, 90)),
                     "source": "rank 0 HIP events per step, in a second untimed pass of the same K steps"},
            setup_s={"generate": t_gen, "plan": t_plan,
                     **({"plan_device_input": t_plan_dev, "device_layout_identical": same} if t_plan_dev else {})},
        )
        # correctness of the timed output, outside the timed region: y of the
        # last step on 10^5 sampled rows against an fp64 numpy evaluation,
        # |dy| <= 1e-6·Σ|a·x| per row (the parity bar of tests/_support.py)
        if native_dist:
            result["exchange"] = exchange_report
        y_out = dsp.step(xd) if (world > 1 or native_dist) else y_local  # every rank: the step holds collectives
        if rank == 0:
            result["check"] = sampled_y_check(rp, col, val, x, y_out.cpu().numpy(), 100_000)
        if kname == "xslice" and rank == 0:
            result["roofline"]["gather"] = gather_ceiling(L, torch, dev, stream, local_nnz, call_s)
        if kname == "xtile":
            # bytes the XTILE layout streams per call: gather reads
            # col16 (2 B) + x tiles, writes xg (T); reduce reads xg (T) + perm (2 B) +
            # val (T) + row_ptr, writes y.  The x-gathers themselves are LDS reads.
            stream_b = local_nnz * (2 + 2 * tsz + 2 + tsz) + (local_rows + len(plans)) * 4 + (n + local_rows) * tsz
            result["roofline"]["layout"] = {"stream_bytes_per_call": stream_b,
                                            "achieved": stream_b / call_s / 1e9,
                                            "frac": stream_b / call_s / 1e9 / HBM_PEAK_GBPS}
        if rank == 0 and world == 1:
            # the attainable rate for the bytes this call streams (the layout's
            # for XTILE, else the algorithmic ones), measured live
            lay = result["roofline"].get("layout")
            moved = lay["stream_bytes_per_call"] if lay else local_alg
            result["roofline"]["copy"] = copy_ceiling(L, torch, dev, stream, int(moved), moved / call_s / 1e9)
        if rank == 0 and world == 1 and not native_dist and not args.no_alt_kernels and wl in ("c2", "c3", "c4"):
            result["alt_kernels"] = alt_kernels(L, torch, dev, stream, rp, col, val, xd, n, nnz, args)
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_spmv_baseline(rp, col, val, x, nnz, args.cpu_seconds,
                                                       threads=1 if wl == "c1" else None)
        for pl in plans:
            pl.close()
        if native_dist:  # the plans before their communicator
            for dp in dplans.values():
                dp.close()
            comm.close()
    elif wl == "sort":
        result.update(sort_bench(args, L, torch, dev, stream, barrier, world, rank))
    elif wl == "cg":
        result.update(cg_bench(args, L, torch, dev, stream, barrier, world, rank))
    else:
        result.update(stencil_bench(args, L, torch, dev, stream, barrier))
        if rank == 0 and world == 1 and not args.no_cpu_baseline and wl in ("blur_x", "blur_y", "c5"):
            result["cpu_baseline"] = result.pop("_cpu", None)
        result.pop("_cpu", None)
    if rank == 0:
        # which library ran: the product build has flags 0 (lhpc_build_flags)
        result["library"] = {"path": os.path.relpath(L.LIB_PATH, ROOT), "build_flags": L.BUILD_FLAGS}
        print(json.dumps(result), flush=True)
    if world > 1 or force_native:
        dist.barrier()
        dist.destroy_process_group()


def alt_kernels(L, torch, dev, stream, rp, col, val, xd, n, nnz, args):
    """The same matrix through the other kernel families, each forced by its
    plan flag and timed like the headline call (HIP events over 10 calls on
    the bench stream): ADAPTIVE and ROWGROUP are the wavefront-per-row CSR
    kernels BASELINE configs[1] names (report both), XSLICE the
    column-sliced one.  Reported beside the default (XTILE), not as `value`."""
    out = {}
    flags = {"adaptive": L.PLAN_FORCE_ADAPTIVE, "rowgroup": L.PLAN_FORCE_ROWGROUP, "xslice": L.PLAN_FORCE_XSLICE}
    y = torch.empty(n, dtype=xd.dtype, device=dev)
    for name, fl in flags.items():
        try:
            t0 = time.time()
            pl = L.SpMVPlan(rp, col, val, n, flags=fl)
            t_plan = time.time() - t0
        except L.LhpcError as e:
            out[name] = {"error": str(e)}
            continue
        for _ in range(3):
            pl(xd, y, stream=stream)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            pl(xd, y, stream=stream)
        e1.record(stream)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e-3 / 10
        kern = {L.KERNEL_XSLICE: "xslice", L.KERNEL_ROWGROUP: "rowgroup", L.KERNEL_ADAPTIVE: "adaptive",
                L.KERNEL_XTILE: "xtile", L.KERNEL_SELL: "sell"}[pl.info()["kernel"]]
        pl.close()
        out[name] = {"gflops": 2.0 * nnz / t / 1e9, "call_us": t * 1e6, "kernel": kern, "plan_s": t_plan}
    del y
    torch.cuda.empty_cache()
    return out


def probe_lib_path(L):
    """liblhpc_probe.so (measurement kernels, not on the ABI): next to the
    loaded liblhpc.so, else the in-tree build (A/B builds ship only liblhpc.so)."""
    p = os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so")
    return p if os.path.exists(p) else os.path.join(ROOT, "libhpc_amd", "_lib", "liblhpc_probe.so")


def copy_ceiling(L, torch, dev, stream, nbytes, achieved_gbps):
    """Attainable rates for the same bytes (a measured copy
    bandwidth beside the 8 TB/s peak), timed live on the bench stream with the
    probes of liblhpc_probe.so (not on the ABI):
      copy  a 16-B/lane copy of nbytes/2 in and nbytes/2 out, non-temporal
            loads and stores, one 16-KB tile per 1024-thread block (the
            fastest of the round-5 calibration sweep, tools/probe_calib.py,
            profiles/r05/probe_calib.jsonl: 6.38 TB/s at this size against
            MI355X_MICROARCH.md's 6.29 TB/s float4 copy); 512-thread blocks
            with 2 loads in flight are timed too and the faster is `copy`;
      read  the same bytes read only (non-temporal, same tiling): the ceiling
            of a read-dominated kernel such as the XTILE reduce;
      copy_gridstride  the round-1..4 probe (grid-stride, 16384 blocks of
            256), kept for continuity.
    `frac` puts achieved_gbps against `copy`."""
    import ctypes as C
    P = C.CDLL(probe_lib_path(L))
    half = (nbytes // 2) // 16 * 16
    src = torch.empty(half // 4, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    n16 = half // 16
    s = C.c_void_p(stream.cuda_stream)

    def rate(fn, moved):
        for _ in range(3):
            fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(10):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return moved / (e0.elapsed_time(e1) * 1e-3 / 10) / 1e9

    def cu(buf_in, buf_out, block, unroll, mode):
        grid = (n16 + block * unroll - 1) // (block * unroll)
        rc = P.lhpc_probe_copy_u(C.c_void_p(buf_in.data_ptr()), C.c_void_p(buf_out.data_ptr()), C.c_int64(half),
                                 C.c_int(grid), C.c_int(block), C.c_int(unroll), C.c_int(mode), s)
        if rc != 0:
            raise RuntimeError(f"lhpc_probe_copy_u: {rc}")
    copies = {f"{b}x{u}": rate(lambda b=b, u=u: cu(src, dst, b, u, 3), 2 * half) for b, u in ((1024, 1), (512, 2))}
    read = rate(lambda: (cu(src, dst, 1024, 1, 5), cu(dst, src, 1024, 1, 5)), 2 * half)
    legacy = rate(lambda: P.lhpc_probe_copy_w(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                              C.c_int64(half), C.c_int(16384), C.c_int(16), C.c_int(1), s), 2 * half)
    del src, dst
    gbps = max(copies.values())
    return {"unit": "GB/s", "copy": gbps, "frac": achieved_gbps / gbps, "read": read,
            "frac_of_read": achieved_gbps / read, "copy_tiles": copies, "copy_gridstride": legacy,
            "bytes": 2 * half,
            "note": "live 16-B/lane probes over the same bytes: copy (nt loads + stores, one 16-KB tile per "
                    "block; the faster of 1024x1 / 512x2), read (nt, read only), copy_gridstride (rounds 1-4)"}


def gather_ceiling(L, torch, dev, stream, nnz, call_s):
    """The binding limit of uniform-random SpMV on MI355X is the L2 request
    rate of 4-byte x gathers, not HBM bandwidth.  Measured
    live: the same number of random gathers from a 4 MB (L2-resident) table
    with the probe kernel (liblhpc_probe.so, not part of the ABI), against the
    SpMV's own gathers per second."""
    import ctypes as C
    P = C.CDLL(probe_lib_path(L))
    m = int(nnz)
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0007)
    idx = torch.randint(0, 1 << 20, (m,), dtype=torch.int32, device=dev, generator=g)
    table = torch.rand(1 << 20, device=dev, generator=g)
    out = torch.empty(m, device=dev)

    def run():
        P.lhpc_probe_gather(C.c_void_p(idx.data_ptr()), C.c_void_p(table.data_ptr()), C.c_void_p(out.data_ptr()),
                            C.c_int64(m), C.c_void_p(stream.cuda_stream))
    for _ in range(3):
        run()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(10):
        run()
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) * 1e-3 / 10
    ceil_gps = m / t
    got = m / call_s
    return {"unit": "G gathers/s", "achieved": got / 1e9, "ceiling": ceil_gps / 1e9, "frac": got / ceil_gps,
            "note": "ceiling = the same number of 4-B random gathers from an L2-resident 4 MB table (probe kernel)"}


def sampled_y_check(rp, col, val, x, y, m, seed=0x5EED00C1):
    """y vs an fp64 numpy evaluation on m seeded rows (no oracle/ code)."""
    n = rp.shape[0] - 1
    rows = np.sort(np.random.default_rng(seed).choice(n, size=min(m, n), replace=False))
    lo, hi = rp[rows].astype(np.int64), rp[rows + 1].astype(np.int64)
    lens = hi - lo
    idx = np.repeat(lo - np.concatenate(([0], np.cumsum(lens)[:-1])), lens) + np.arange(lens.sum())
    prod = val[idx].astype(np.float64) * x[col[idx]].astype(np.float64)
    seg = np.repeat(np.arange(rows.size), lens)
    y64 = np.bincount(seg, weights=prod, minlength=rows.size)
    asum = np.bincount(seg, weights=np.abs(prod), minlength=rows.size)
    err = np.abs(y[rows].astype(np.float64) - y64)
    ratio = float(np.max(err / (1e-6 * asum + 1e-30))) if rows.size else 0.0
    return {"rows": int(rows.size), "nnz": int(lens.sum()), "max_err_over_bound": ratio, "pass": ratio <= 1.0,
            "bound": "|dy| <= 1e-6*sum|a*x| per row vs fp64 numpy"}


def host_info(threads=None):
    """Which host produced a CPU baseline: CPU model, the CPUs this process may
    run on (PROCESS_CPUS, read before OpenMP loaded), the NUMA nodes those CPUs
    belong to, and the threads the baseline ran (bound close, one per core,
    inside that set)."""
    info = {"cpu_model": None, "affinity_cpus": None, "numa_nodes": None, "threads": threads}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        cpus = PROCESS_CPUS
        info["affinity_cpus"] = len(cpus)
        mine, nodes = set(cpus), set()
        base = "/sys/devices/system/node"
        for d in os.listdir(base):
            if not (d.startswith("node") and d[4:].isdigit()):
                continue
            node_cpus = set()
            for part in open(os.path.join(base, d, "cpulist")).read().strip().split(","):
                if part:
                    lo, _, hi = part.partition("-")
                    node_cpus.update(range(int(lo), int(hi or lo) + 1))
            if node_cpus & mine:
                nodes.add(int(d[4:]))
        info["numa_nodes"] = sorted(nodes) or None
    except OSError:
        pass
    return info


def cpu_spmv_baseline(rp, col, val, x, nnz, seconds, threads=None):
    """C1 is quoted single-thread.  C2-C4 run two legs on the
    box's host: OMP_NUM_THREADS (the box sets 16: its CPU share per GPU) and
    the process CPU set's size (`$(nproc)`, SURVEY §8d / BASELINE.md §3);
    `value` is the faster leg and `cores` the thread count it used, `legs`
    holds both.  Each leg gets half of `seconds`."""
    from tests import _support as S  # oracle/ is test infrastructure: baseline leg only
    counts = [threads] if threads else sorted({cpu_threads(), len(PROCESS_CPUS)})
    legs = []
    for th in counts:
        y, used = S.spmv_cpu_simd(rp, col, val, x, threads=th)  # warm
        times = []
        t_end = time.perf_counter() + seconds / len(counts)
        while len(times) < 3 or (time.perf_counter() < t_end and len(times) < 200_000):
            t0 = time.perf_counter()
            S.spmv_cpu_simd(rp, col, val, x, threads=th)
            times.append(time.perf_counter() - t0)
        legs.append({"threads": used, "value": 2.0 * nnz / min(times) / 1e9, "passes": len(times),
                     "seconds": sum(times)})
    best = max(legs, key=lambda g: g["value"])
    return {"value": best["value"], "unit": "GFLOP/s", "cores": best["threads"], "kind": "port",
            "legs": legs,
            "sample": f"full matrix (nnz={nnz}), best pass per leg, AVX2 gather"
                      + (" + OpenMP" if best["threads"] > 1 else ", 1 thread") + ", oracle/oracle.c cpu_spmv_simd; "
                      "legs: OMP_NUM_THREADS and the process CPU set size",
            "omp": {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OMP_PROC_BIND", "OMP_PLACES")},
            "host": host_info(best["threads"])}


def stencil_bench(args, L, torch, dev, stream, barrier):
    wl = args.workload
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if wl == "c5":
        n = 512
        g = 1
        P = n + 2
        cells = n ** 3
        name = "k_stencil7_buf4"
        force_native = os.environ.get("LHPC_DIST_NATIVE", "0") == "1" and "RANK" in os.environ
        if world == 1 and not force_native:
            u = torch.zeros(P ** 3, device=dev)
            u.view(P, P, P)[1:-1, 1:-1, 1:-1] = torch.rand(n, n, n, device=dev) * 2 - 1
            o = torch.zeros_like(u)
            fn = lambda: L.stencil7(u, o, n, n, n, g, -6.0, 1.0, stream=stream)  # noqa: E731
            workload = "BASELINE configs[4] grid: 7-point 3-D stencil 512^3 fp32, 1 GPU"
        else:
            from libhpc_amd.dist import DistStencil7, slab_bounds
            z0, z1 = slab_bounds(n, rank, world)
            nzl = z1 - z0
            u = torch.zeros((nzl + 2) * P * P, device=dev)
            u.view(nzl + 2, P, P)[1:-1, 1:-1, 1:-1] = torch.rand(nzl, n, n, device=dev) * 2 - 1
            o = torch.zeros_like(u)
            import torch.distributed as dist
            has_rccl = dist.get_backend() == "nccl" and os.environ.get("LHPC_DIST_TORCH", "0") != "1"
            if has_rccl or os.environ.get("LHPC_DIST_P2P", "0") == "1":
                # native (lhpc_dist_stencil7_f32_x): the halo planes over RCCL
                # send/recv on the comm stream, or stored straight into the
                # neighbours' ghost planes (u a registered P2P window), while
                # the interior planes run — both timed, the faster reported
                comm = L.DistComm.from_torch(torch.cuda.current_device()) if has_rccl else \
                    L.DistComm.local(world, rank, torch.cuda.current_device())
                kinds = {}
                if has_rccl:
                    kinds["rccl"] = L.DIST_EXCHANGE_RCCL
                try:
                    comm.p2p_setup_torch(u)
                    kinds["p2p"] = L.DIST_EXCHANGE_P2P
                except Exception:  # no IPC between the devices: RCCL only
                    pass
                halo_ms = {}
                for kname, kx in kinds.items():
                    f = lambda kx=kx: comm.stencil7(u, o, nzl, n, n, 1, -6.0, 1.0, stream=stream,  # noqa: E731
                                                    exchange=kx)
                    for _ in range(3):
                        f()
                    barrier()
                    t0 = time.perf_counter()
                    for _ in range(20):
                        f()
                    barrier()
                    tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                                      device=dev if has_rccl else "cpu")
                    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                    halo_ms[kname] = float(tt.item()) / 20 * 1e3
                best = min(halo_ms, key=halo_ms.get)
                fn = lambda: comm.stencil7(u, o, nzl, n, n, 1, -6.0, 1.0, stream=stream,  # noqa: E731
                                           exchange=kinds[best])
                how = (f"native {'RCCL send/recv' if best == 'rccl' else 'P2P peer-store'} halo "
                       f"(lhpc_dist_stencil7_f32_x; measured ms/step {halo_ms})")
            else:
                ds = DistStencil7(nzl, n, n, rank, world, lambda ut, ot, zb, ze: L.stencil7_planes(
                    ut, ot, nzl, n, n, 1, -6.0, 1.0, zb, ze, stream=stream))
                fn = lambda: ds.step(u, o)  # noqa: E731
                how = "torch.distributed halo"
            workload = f"BASELINE configs[4]: 7-point 3-D stencil 512^3 fp32, z-slabs x{world} + {how}"
    else:
        n, g = 8192, 8
        a = torch.rand((n + 2 * g) ** 2, device=dev) * 2 - 1
        b = torch.empty(n * n, device=dev)
        f = L.blur_x if wl == "blur_x" else L.blur_y
        fn = lambda: f(a, b, n, n, g, 8, stream=stream)  # noqa: E731
        cells = n * n
        name = "k_blur_x" if wl == "blur_x" else "k_blur_y"
        workload = f"reference BM_{wl} grid: 8192^2 fp32, ghost 8, 17 taps"
    settled = settle(fn, torch, args.settle_ms if world == 1 else 0.0)
    for _ in range(args.warmup):
        fn()
    barrier()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        fn()
    e1.record(stream)
    barrier()
    per = e0.elapsed_time(e1) * 1e-3 / args.steps
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([per], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        per = float(tt.item())
    ach = 8.0 * cells / per / 1e9 / world
    copy = copy_ceiling(L, torch, dev, stream, int(8 * cells // world), ach) if rank == 0 else None
    out = dict(metric=f"{wl} Gcell/s (8 B/cell algorithmic)", value=cells / per / 1e9, unit="Gcell/s",
               n_gpus=world, steps=args.steps, warmup=args.warmup, ms_per_step=per * 1e3,
               higher_is_better=True, scaling="strong" if wl == "c5" else "weak", vs_baseline=None, dtype="f32",
               settle=settled,
               data="synthetic U[-1,1)", config={"workload": workload},
               roofline={"bound": "hbm", "kernel": name, "achieved": ach, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": ach / HBM_PEAK_GBPS,
                         "traffic": load_traffic(wl) if world == 1 else None, "copy": copy})
    if wl == "c5" and world == 1 and not args.no_cpu_baseline:
        from tests import _support as S
        lib = S.load_oracle()
        uh = u.cpu().numpy()
        oh = np.zeros_like(uh)
        th = cpu_threads()
        ts = []
        t_end = time.perf_counter() + args.cpu_seconds
        while len(ts) < 2 or (time.perf_counter() < t_end and len(ts) < 5000):
            t0 = time.perf_counter()
            lib.oracle_stencil7(uh.ctypes.data, oh.ctypes.data, n, n, n, g, -6.0, 1.0, th)
            ts.append(time.perf_counter() - t0)
        out["_cpu"] = {"value": cells / min(ts) / 1e9, "unit": "Gcell/s", "cores": th, "kind": "port",
                       "sample": f"full 512^3 grid, best of {len(ts)} passes, OpenMP oracle_stencil7", "host": host_info(th)}
    if wl in ("blur_x", "blur_y") and not args.no_cpu_baseline:
        from tests import _support as S
        lib = S.load_oracle()
        ah = a.cpu().numpy()
        bh = np.empty(n * n, dtype=np.float32)
        fnc = lib.cpu_blur_x_sse if wl == "blur_x" else lib.cpu_blur_y_sse
        th = cpu_threads()
        fnc(ah.ctypes.data, bh.ctypes.data, n, n, g, th)
        ts = []
        t_end = time.perf_counter() + args.cpu_seconds
        while len(ts) < 3 or (time.perf_counter() < t_end and len(ts) < 400):
            t0 = time.perf_counter()
            fnc(ah.ctypes.data, bh.ctypes.data, n, n, g, th)
            ts.append(time.perf_counter() - t0)
        out["_cpu"] = {"value": cells / min(ts) / 1e9, "unit": "Gcell/s", "cores": th, "kind": "port",
                       "sample": f"full 8192^2 grid, best of {len(ts)} passes, reference SSE loop restated",
                       "host": host_info(th)}
    return out


def cg_bench(args, L, torch, dev, stream, barrier, world, rank):
    from libhpc_amd.dist import DistCG, HipOps, InterleavedBlocks
    nx = 4096
    rp, col, val = L.gen_laplacian_2d(nx, nx, L.F64)
    n, nnz = nx * nx, int(col.size)
    b = L.gen_values(L.F64, 0, n, L.SEED_X)
    native = world > 1 and torch.distributed.get_backend() == "nccl" and os.environ.get("LHPC_DIST_TORCH", "0") != "1"
    comm = dplan = None
    if native:
        # the native distributed CG (lhpc_dist_cg_solve): interleaved
        # nnz-balanced blocks, K chunks per rank, p exchanged over RCCL with
        # the next q = A·p's gather chained per chunk, dots as block partials
        K = min(args.chunks if args.chunks > 0 else 4, 8)
        comm = L.DistComm.from_torch(dev.index)
        cuts = L.interleaved_cuts(rp, world, K)
        dplan = L.DistSpMVPlan(comm, n, n, K, cuts, *L.interleaved_local_csr(rp, col, val, cuts, world, K, rank))
        plan = dplan
        bfull = torch.from_numpy(b).to(dev)
        pw = torch.empty(n, dtype=torch.float64, device=dev)

        def run(iters):
            x = torch.zeros(n, dtype=torch.float64, device=dev)
            return dplan.cg(bfull, x, pw, tol=0.0, max_iter=iters, check_every=iters, stream=stream)
    elif world == 1:
        # lhpc_cg_solve: the native loop, whose check_every = 10 iterations
        # between two convergence checks replay as one captured HIP graph
        # (tol 0: exactly `iters` iterations; the warmup solve captures it)
        plan = L.SpMVPlan(rp, col, val, n, options=args.spmv_options)  # SELL (spmv_no_sell=1: ADAPTIVE)
        bfull = torch.from_numpy(b).to(dev)
        cg_stream = torch.cuda.Stream(dev)

        def run(iters):
            x = torch.zeros(n, dtype=torch.float64, device=dev)
            with torch.cuda.stream(cg_stream):
                out = L.cg(plan, bfull, x, tol=0.0, max_iter=iters, check_every=10, stream=cg_stream)
            cg_stream.synchronize()
            return out
    else:
        ib = InterleavedBlocks(n, world, 1)
        r0, r1 = ib.rows(rank, 0)
        plan = L.SpMVPlan(*ib.local_csr(rp, col, val, rank, 0), n)
        bd = torch.zeros(ib.B, dtype=torch.float64, device=dev)
        bd[:r1 - r0] = torch.from_numpy(b[r0:r1]).to(dev)
        solver = DistCG(ib, rank, lambda pf, qb: plan(pf, qb, stream=stream), HipOps(stream), like=bd,
                        local_spmv_dot=lambda pf, qb, wb, out: L.spmv_dot(plan, pf, qb, wb, out, stream=stream))

        def run(iters):
            x = torch.zeros_like(bd)
            return solver.solve(bd, x, tol=0.0, max_iter=iters, check_every=iters)  # tol 0: exactly `iters` iterations

    settled = settle(lambda: run(10), torch, args.settle_ms if world == 1 else 0.0)
    run(max(10, args.warmup))
    barrier()
    t0 = time.perf_counter()
    _, it, res = run(args.steps)
    barrier()
    per = (time.perf_counter() - t0) / args.steps
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([per], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        per = float(tt.item())
    spmv_b = nnz * (8 + 4) + (n + 1) * 4 + 2 * n * 8
    # p·q in the SpMV epilogue (w = p read again: n), r update (read r q, write r: 3n),
    # x/p update (read x p r, write x p: 5n) — k_cg_r + k_cg_xp
    vec_b = 9 * n * 8
    alg = (spmv_b + vec_b) / world
    kid = dplan.local_info()["kernel"] if native else plan.info()["kernel"]
    kname = {L.KERNEL_ROWGROUP: "rowgroup", L.KERNEL_ADAPTIVE: "adaptive", L.KERNEL_XSLICE: "xslice",
             L.KERNEL_XTILE: "xtile", L.KERNEL_SELL: "sell"}[kid]
    out = dict(metric="CG iterations/s, 2-D Laplacian 4096^2 fp64 (SURVEY 8f rank 3)", value=1.0 / per,
               unit="iter/s", n_gpus=world, steps=args.steps, warmup=args.warmup, ms_per_step=per * 1e3,
               higher_is_better=True, scaling="strong", vs_baseline=None, dtype="f64", settle=settled,
               data="synthetic: 5-point Laplacian, b = U[-1,1) (SEED_X)",
               config={"workload": f"CG, 2-D Laplacian {nx}^2 fp64, n={n}, nnz={nnz}, {world} GPU(s)",
                       "iterations": it, "relres": res,
                       "kernel": kid, "kernel_name": kname,
                       "solver": "lhpc_dist_cg_solve (native, RCCL, chained stages)" if native else
                                 ("lhpc_cg_solve (native loop, 10-iteration HIP graph blocks)" if world == 1 else
                                  "DistCG over torch.distributed")},
               roofline={"bound": "hbm",
                         "kernel": "k_spmv_sell_cg + k_cg_r" if kname == "sell" and world == 1 else
                                   f"spmv_dot (k_spmv_{kname}) + k_cg_r + k_cg_xp",
                         "achieved": alg / per / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": alg / per / 1e9 / HBM_PEAK_GBPS,
                         # PMC bytes per iteration (profiles/traffic.json "cg_sell")
                         "traffic": load_traffic("cg_sell") if kname == "sell" and world == 1 else None,
                         "alg_bytes_per_iter": alg})
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from tests import _support as S
        lib = S.load_oracle()
        import ctypes as C
        k = 0
        ts = []
        t_end = time.perf_counter() + args.cpu_seconds
        while len(ts) < 1 or (time.perf_counter() < t_end and len(ts) < 5):
            x = np.zeros(n)
            res_c = C.c_double(0.0)
            t0 = time.perf_counter()
            k = lib.oracle_cg_f64(n, rp.ctypes.data, 64, col.ctypes.data, val.ctypes.data, b.ctypes.data,
                                  x.ctypes.data, 0.0, 5, C.byref(res_c))
            ts.append((time.perf_counter() - t0) / max(k, 1))
        out["cpu_baseline"] = {"value": 1.0 / min(ts), "unit": "iter/s", "cores": 1, "kind": "port",
                               "sample": f"{k} iterations of the fp64 CG restatement (oracle.c), best of {len(ts)}",
                               "host": host_info(1)}
    plan.close()
    if comm is not None:
        comm.close()
    return out


SORT_N = 500_000_000
SORT_REF_GKEYS = 500e6 / 0.360 / 1e9  # reference README.md:52: 500M keys in ~360 ms


def sort_bench(args, L, torch, dev, stream, barrier, world, rank):
    n = SORT_N
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0006 + rank)
    src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev, generator=g)
    keys = torch.empty_like(src)

    def one_sort():
        keys.copy_(src)
        L.radix_sort(keys, stream=stream)
    settled = settle(one_sort, torch, args.settle_ms if world == 1 else 0.0)
    for _ in range(args.warmup):
        one_sort()
    barrier()
    total = 0.0
    for _ in range(args.steps):
        keys.copy_(src)  # restore the unsorted batch (outside the timed events)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        L.radix_sort(keys, stream=stream)
        e1.record(stream)
        e1.synchronize()
        total += e0.elapsed_time(e1) * 1e-3
    barrier()
    per = total / args.steps
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([per], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        per = float(tt.item())
    ok = bool((keys[1:].to(torch.int64) & 0xFFFFFFFF).ge(keys[:-1].to(torch.int64) & 0xFFFFFFFF).all())
    value = world * n / per / 1e9
    alg = 32.0 * n  # 4 passes x (read + write) x 4 B per key
    out = dict(metric="radix sort G keys/s, 500M uint32 keys (reference README.md:52)", value=value,
               unit="Gkeys/s", n_gpus=world, steps=args.steps, warmup=args.warmup, ms_per_step=per * 1e3,
               higher_is_better=True, scaling="weak", vs_baseline=value / world / SORT_REF_GKEYS, dtype="u32",
               settle=settled,
               data="synthetic uniform uint32 (torch generator)",
               config={"workload": "reference README radix-sort config: 500M uint32 keys, 1 GPU"
                       + (f" x{world} replicas" if world > 1 else ""), "sorted": ok},
               roofline={"bound": "hbm", "kernel": "k_radix_upsweep+k_radix_scan+k_radix_downsweep x4",
                         "achieved": alg / per / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": alg / per / 1e9 / HBM_PEAK_GBPS,
                         "traffic": load_traffic("sort") if world == 1 else None})
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_sort_baseline(keys, src, args.cpu_seconds)
    return out


def cpu_sort_baseline(keys, src, seconds):
    """The reference's own CPU radix sort (radix_sort_cache_thread_v2<256>, OpenMP) on a
    bounded 50M-key sample of the same keys; the C restatement if the reference build is absent."""
    from tests import _support as S
    m = 50_000_000
    base = src[:m].cpu().numpy().view(np.uint32).copy()
    ref = S.load_ref_sort()
    if ref is not None:
        fn, kind = (lambda a: ref.ref_radix_sort_u32(a.ctypes.data, a.size)), "reference"
    else:
        lib = S.load_oracle()
        fn, kind = (lambda a: lib.oracle_radix_sort_u32(a.ctypes.data, None, a.size, 0, 32)), "port"
    ts = []
    t_end = time.perf_counter() + seconds
    while len(ts) < 2 or (time.perf_counter() < t_end and len(ts) < 50):
        a = base.copy()
        t0 = time.perf_counter()
        fn(a)
        ts.append(time.perf_counter() - t0)
    assert np.all(a[1:] >= a[:-1])
    return {"value": m / min(ts) / 1e9, "unit": "Gkeys/s", "cores": cpu_threads(), "kind": kind,
            "sample": f"50M of the same keys, best of {len(ts)} sorts"
                      + (" (reference radix_sort, OpenMP)" if kind == "reference" else " (C LSD restatement)"),
            "host": host_info(cpu_threads())}


if __name__ == "__main__":
    main()
