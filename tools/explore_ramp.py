"""How the C2 call time evolves over a run (round 5): after the plan build
and an idle gap, 5 × (20 back-to-back calls) timed one after another, then
one 200-call run with an event at every call; prints µs per call."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
n = 10_000_000
rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=L.F32)
x = torch.from_numpy(L.gen_values(L.F32, 0, n, L.SEED_X)).to(dev)
y = torch.empty(n, dtype=torch.float32, device=dev)
plan = L.SpMVPlan(rp, col, val, n)
s = torch.cuda.current_stream(dev)
torch.cuda.synchronize()
time.sleep(float(os.environ.get("RAMP_IDLE", "0.5")))  # an idle gap, as after host-side setup
for rep in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        plan(x, y, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    print(json.dumps({"block": rep, "calls": 20, "us_per_call": e0.elapsed_time(e1) * 1e3 / 20}), flush=True)
time.sleep(float(os.environ.get("RAMP_IDLE", "0.5")))
ev = [torch.cuda.Event(enable_timing=True) for _ in range(201)]
for i in range(200):
    ev[i].record(s)
    plan(x, y, stream=s)
ev[200].record(s)
torch.cuda.synchronize()
t = np.array([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(200)])
print(json.dumps({"per_call_us_by_10": [round(float(t[i:i + 10].mean()), 1) for i in range(0, 200, 10)]}), flush=True)
