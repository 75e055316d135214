"""Radix sort / COO→CSR throughput sweep on one GPU (JSON lines)."""
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L

dev = torch.device("cuda:0")
st = torch.cuda.Stream()


def timed(prep, fn, iters=5):
    ts = []
    with torch.cuda.stream(st):
        for i in range(iters + 1):
            prep()
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st); fn(); e1.record(st)
            e1.synchronize()
            if i:
                ts.append(e0.elapsed_time(e1) * 1e-3)
    return min(ts), sum(ts) / len(ts)


import ctypes as C
RP = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe_rocprim.so"))


def rocprim_u32(src, out):
    nb = C.c_size_t(0)
    RP.lhpc_probe_rocprim_sort_u32(None, None, C.c_int64(src.numel()), None, C.byref(nb), None)
    tmp = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
    return lambda: RP.lhpc_probe_rocprim_sort_u32(C.c_void_p(src.data_ptr()), C.c_void_p(out.data_ptr()),
                                                  C.c_int64(src.numel()), C.c_void_p(tmp.data_ptr()),
                                                  C.byref(nb), C.c_void_p(st.cuda_stream))


for n in [int(x) for x in os.environ.get("SORT_NS", "1000000 16000000 100000000 500000000").split()]:
    src = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
    k = torch.empty_like(src)
    tmin, tavg = timed(lambda: k.copy_(src), lambda: L.radix_sort(k, stream=st))
    ok = bool(((k[1:].to(torch.int64) & 0xFFFFFFFF) >= (k[:-1].to(torch.int64) & 0xFFFFFFFF)).all()) if n < 200_000_000 else None
    print(json.dumps(dict(k="sort_u32", n=n, ms=tmin * 1e3, ms_avg=tavg * 1e3, Gkeys=n / tmin / 1e9,
                          GBps_alg=32 * n / tmin / 1e9, sorted=ok)), flush=True)
    out = torch.empty_like(src)
    fn = rocprim_u32(src, out)
    tmin, tavg = timed(lambda: None, fn)
    print(json.dumps(dict(k="rocprim_sort_u32", n=n, ms=tmin * 1e3, Gkeys=n / tmin / 1e9,
                          same=bool(torch.equal(out, k)))), flush=True)
    del out
    del src, k
    torch.cuda.empty_cache()

n = 150_000_000
ku = torch.randint(-2**31, 2**31 - 1, (n,), dtype=torch.int32, device=dev)
vu = torch.arange(n, dtype=torch.int32, device=dev)
k = torch.empty_like(ku); v = torch.empty_like(vu)
def prep_u():
    k.copy_(ku); v.copy_(vu)
tmin, tavg = timed(prep_u, lambda: L.radix_sort_pairs(k, v, 0, 32, stream=st))
print(json.dumps(dict(k="sort_pairs_u32", n=n, ms=tmin * 1e3, Gkeys=n / tmin / 1e9)), flush=True)
del ku, vu, k, v
ks = torch.randint(0, 2**47, (n,), dtype=torch.int64, device=dev)
vs = torch.arange(n, dtype=torch.int32, device=dev)
k = torch.empty_like(ks); v = torch.empty_like(vs)
def prep():
    k.copy_(ks); v.copy_(vs)
tmin, tavg = timed(prep, lambda: L.radix_sort_pairs(k, v, 0, 47, stream=st))
print(json.dumps(dict(k="sort_pairs_u64_47b", n=n, ms=tmin * 1e3, Gkeys=n / tmin / 1e9)), flush=True)
ko = torch.empty_like(ks); vo = torch.empty_like(vs)
nb = C.c_size_t(0)
RP.lhpc_probe_rocprim_sort_pairs_u64(None, None, None, None, C.c_int64(n), 47, None, C.byref(nb), None)
tmp = torch.empty(max(nb.value, 1), dtype=torch.uint8, device=dev)
tmin, tavg = timed(lambda: None, lambda: RP.lhpc_probe_rocprim_sort_pairs_u64(
    C.c_void_p(ks.data_ptr()), C.c_void_p(ko.data_ptr()), C.c_void_p(vs.data_ptr()), C.c_void_p(vo.data_ptr()),
    C.c_int64(n), 47, C.c_void_p(tmp.data_ptr()), C.byref(nb), C.c_void_p(st.cuda_stream)))
print(json.dumps(dict(k="rocprim_pairs_u64_47b", n=n, ms=tmin * 1e3, Gkeys=n / tmin / 1e9,
                      same=bool(torch.equal(ko, k) and torch.equal(vo, v)))), flush=True)
del ko, vo, tmp
del ks, vs, k, v
torch.cuda.empty_cache()

n_rows = 10_000_000
rows = torch.randint(0, n_rows, (n,), dtype=torch.int32, device=dev)
cols = torch.randint(0, n_rows, (n,), dtype=torch.int32, device=dev)
vals = torch.rand(n, device=dev)
tmin, tavg = timed(lambda: None, lambda: L.coo_to_csr(n_rows, n_rows, rows, cols, vals, stream=st), iters=3)
print(json.dumps(dict(k="coo_to_csr_c2", nnz=n, ms=tmin * 1e3, Gnnz=n / tmin / 1e9)), flush=True)
