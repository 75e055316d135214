"""Pair-sort A/B timing (round 6): through LHPC_LIB_PATH's library, 150M
uint32 (key, value) pairs over 32 bits, 150M uint64 keys over 47 bits with
uint32 values (the COO→CSR sort), and COO→CSR of 150M entries (C2's shape).
Each first checks a 4M-pair sort against torch's stable sort (values =
input positions, so the check covers stability).  One JSON line per case,
min and mean ms over 5 timed calls (HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.Stream(dev)
g = torch.Generator(device=dev)
g.manual_seed(0x5A17)


def timed(prep, fn, iters=5):
    ts = []
    with torch.cuda.stream(st):
        for i in range(iters + 1):
            prep()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            e1.synchronize()
            if i:
                ts.append(e0.elapsed_time(e1))
    return min(ts), sum(ts) / len(ts)


def check(keys, bits):
    v = torch.arange(keys.numel(), dtype=torch.int32, device=dev)
    k = keys.clone()
    L.radix_sort_pairs(k, v, 0, bits, stream=st)
    st.synchronize()
    wide = keys.to(torch.int64) & ((1 << bits) - 1) if keys.dtype == torch.int32 else keys
    sv, si = torch.sort(wide, stable=True)
    kw = k.to(torch.int64) & ((1 << bits) - 1) if keys.dtype == torch.int32 else k
    return bool(torch.equal(kw, sv) and torch.equal(v.to(torch.int64), si))


n = 150_000_000
for name, dt, bits, hi in (("pairs_u32", torch.int32, 32, None), ("pairs_u64_47b", torch.int64, 47, 2**47)):
    small = (torch.randint(-2**31, 2**31 - 1, (4_000_000,), dtype=dt, device=dev, generator=g) if hi is None
             else torch.randint(0, hi, (4_000_000,), dtype=dt, device=dev, generator=g))
    ok = check(small, bits)
    ks = (torch.randint(-2**31, 2**31 - 1, (n,), dtype=dt, device=dev, generator=g) if hi is None
          else torch.randint(0, hi, (n,), dtype=dt, device=dev, generator=g))
    vs = torch.arange(n, dtype=torch.int32, device=dev)
    k, v = torch.empty_like(ks), torch.empty_like(vs)

    def prep():
        k.copy_(ks)
        v.copy_(vs)
    tmin, tavg = timed(prep, lambda: L.radix_sort_pairs(k, v, 0, bits, stream=st))
    print(json.dumps(dict(k=name, n=n, ms=tmin, ms_avg=tavg, Gpairs=n / tmin / 1e6, stable_4M=ok,
                          lib=os.path.relpath(L.LIB_PATH))), flush=True)
    del ks, vs, k, v, small
    torch.cuda.empty_cache()

n_rows = 10_000_000
rows = torch.randint(0, n_rows, (n,), dtype=torch.int32, device=dev, generator=g)
cols = torch.randint(0, n_rows, (n,), dtype=torch.int32, device=dev, generator=g)
vals = torch.rand(n, device=dev, generator=g)
tmin, tavg = timed(lambda: None, lambda: L.coo_to_csr(n_rows, n_rows, rows, cols, vals, stream=st), iters=3)
print(json.dumps(dict(k="coo_to_csr_c2", nnz=n, ms=tmin, ms_avg=tavg, Gnnz=n / tmin / 1e6)), flush=True)
