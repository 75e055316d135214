"""Gather-rate probe: does XCD-local column slicing turn x-gathers into L2 hits?"""
import ctypes as C, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libhpc_amd as L
P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
dev = torch.device("cuda:0"); sp = torch.cuda.current_stream().cuda_stream
def timeit(fn, iters=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3
n = 150_000_000
out = torch.empty(n, device=dev)
for tot_mb, S_list in ((40, (1, 4, 8, 16)), (80, (1, 8, 16)), (20, (1, 8))):
    tn = tot_mb * 1_000_000 // 4
    table = torch.rand(tn, device=dev)
    for S in S_list:
        sl = tn // S
        idx = torch.randint(0, sl, (n,), dtype=torch.int32, device=dev)
        for nt in (0, 1):
            t = timeit(lambda: P.lhpc_probe_gather_sliced(C.c_void_p(idx.data_ptr()), C.c_void_p(table.data_ptr()),
                       C.c_void_p(out.data_ptr()), C.c_int64(n), C.c_int(S), C.c_int64(sl), C.c_int(nt), C.c_void_p(sp)))
            print(json.dumps(dict(table_MB=tot_mb, S=S, slice_MB=tot_mb / S, nt_gather=nt, Ggps=n / t / 1e9, ms=t * 1e3)), flush=True)
        del idx
    del table
