"""Where the ≈ 6 µs between two lhpc_spmv calls comes from (round 5): the C2
call timed back to back (a) through SpMVPlan.__call__, (b) through the raw
ctypes entry point with precomputed arguments, (c) with a host-side pause
before the loop so the queue is full, and (d) as a captured HIP graph of one
call, replayed.  Prints per-call µs (HIP events) and the host enqueue time."""
import ctypes as C
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
n = 10_000_000
rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=L.F32)
x = torch.from_numpy(L.gen_values(L.F32, 0, n, L.SEED_X)).to(dev)
y = torch.empty(n, dtype=torch.float32, device=dev)
plan = L.SpMVPlan(rp, col, val, n)
s = torch.cuda.Stream(dev)
N = 30


def timed(label, fn, pre=None):
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        if pre:
            pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        h0 = time.perf_counter()
        for _ in range(N):
            fn()
        h1 = time.perf_counter()
        e1.record(s)
        torch.cuda.synchronize()
    print(json.dumps({"variant": label, "us_per_call": e0.elapsed_time(e1) * 1e3 / N,
                      "host_enqueue_us_per_call": (h1 - h0) * 1e6 / N}), flush=True)


timed("plan_call", lambda: plan(x, y, stream=s))
h, xp, yp, sp = plan._h, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), C.c_void_p(s.cuda_stream)
timed("ctypes_direct", lambda: L.lib.lhpc_spmv(h, xp, yp, 1, sp))


def sleepy():  # a long GPU kernel first, so every call below is enqueued before the GPU reaches it
    a = torch.empty(1 << 28, device=dev)
    for _ in range(20):
        a.mul_(1.0001)


timed("queue_full", lambda: L.lib.lhpc_spmv(h, xp, yp, 1, sp), pre=sleepy)
try:
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            L.lib.lhpc_spmv(h, xp, yp, 1, sp)
    timed("graph_replay", lambda: g.replay())
    y2 = y.clone()
    L.lib.lhpc_spmv(h, xp, yp, 1, sp)
    torch.cuda.synchronize()
    print(json.dumps({"graph_same_y": bool(torch.equal(y, y2))}), flush=True)
except Exception as e:  # capture refused
    print(json.dumps({"variant": "graph_replay", "error": str(e)}), flush=True)
