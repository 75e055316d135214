"""Copy-bandwidth probes: lane width × cache policy × access order, at the
stencil7 C5 array size (514^3 floats).  Prints JSON lines (GB/s of read+write)."""
import ctypes as C
import json
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L

P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
nbytes = 514 ** 3 * 4
src = torch.rand(nbytes // 4, device=dev)
dst = torch.empty_like(src)


def timeit(fn, iters=20):
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


for width in (4, 8, 16):
    for mode in (0, 1, 2, 3):
        for grid in (256, 1024, 4096, 16384):
            t = timeit(lambda: P.lhpc_probe_copy_w(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                                   C.c_int64(nbytes), C.c_int(grid), C.c_int(width), C.c_int(mode),
                                                   C.c_void_p(st.cuda_stream)))
            print(json.dumps(dict(width=width, nt=bool(mode & 1), chunked=bool(mode & 2), grid=grid,
                                  us=round(t * 1e6, 1), GBps=round(2 * nbytes / t / 1e9))), flush=True)
    assert torch.equal(src, dst)
t = timeit(lambda: dst.copy_(src))
print(json.dumps(dict(torch_copy=True, us=round(t * 1e6, 1), GBps=round(2 * nbytes / t / 1e9))), flush=True)
