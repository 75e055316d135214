"""FETCH_SIZE calibration on known byte counts (run under rocprofv3 --pmc FETCH_SIZE):
1 GiB read with 16 B/lane (dwordx4) and with 4 B/lane (dword) non-temporal loads."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libhpc_amd as L
P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
nb = 1 << 30
src = torch.rand(nb // 4, device="cuda")
sink = torch.empty(16, device="cuda")
sp = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    P.lhpc_probe_read(C.c_void_p(src.data_ptr()), C.c_void_p(sink.data_ptr()), C.c_int64(nb), C.c_int(2048), C.c_void_p(sp))
    P.lhpc_probe_read4(C.c_void_p(src.data_ptr()), C.c_void_p(sink.data_ptr()), C.c_int64(nb), C.c_int(2048), C.c_void_p(sp))
torch.cuda.synchronize()
print("calibration kernels done: k_read16 / k_read4 each read", nb, "bytes per launch")
