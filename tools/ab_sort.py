"""Sort A/B timing (round 5): 500M uint32 keys (the bench's sort workload),
W warm + K timed lhpc_radix_sort_u32 calls through LHPC_LIB_PATH's library;
prints ms per sort and, unless AB_SORT_NOCHECK=1 (timing-only probe builds),
whether a 10M-key sort came out sorted.  Per-kernel times come from
rocprofv3 --stats around it."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev)
g = torch.Generator(device=dev)
g.manual_seed(0x5EED)
if os.environ.get("AB_SORT_NOCHECK") != "1":
    s = torch.randint(-2**31, 2**31 - 1, (10_000_000,), dtype=torch.int32, device=dev, generator=g)
    k = s.clone()
    L.radix_sort(k, stream=st)
    u = k.to(torch.int64) & 0xFFFFFFFF
    ok = bool((u[1:] >= u[:-1]).all()) and torch.equal(torch.sort(s.to(torch.int64) & 0xFFFFFFFF).values, u)
    print(json.dumps({"sorted_10M": ok}), flush=True)
    del s, k, u
n = 500_000_000
src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev, generator=g)
k = torch.empty_like(src)
ts = []
for i in range(8):
    k.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    L.radix_sort(k, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    if i >= 2:
        ts.append(e0.elapsed_time(e1))
print(json.dumps({"n": n, "ms_min": min(ts), "ms_med": sorted(ts)[len(ts) // 2], "Gkeys": n / min(ts) / 1e6}),
      flush=True)
