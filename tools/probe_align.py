"""What the 7-point stencil's 4-byte x offset costs a plain copy (round 5).

The stencil reads and writes 16-B vectors at (x + g)·4 bytes into padded rows
(g = 1), i.e. 4 bytes off every 16-B boundary — the ghost column makes it so,
and the out ghosts may not be written.  This probe times the calibrated
16-B/lane non-temporal copy (lhpc_probe_copy_u, 1024 × 1, mode 3) over the
stencil's bytes with src and dst both at +0, +4, +8 and +16 bytes from a
256-B aligned base.  One JSON line per offset (µs, TB/s), interleaved repeats.
"""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream(dev)
P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
n = 512
half = (8 * n ** 3 // 2) // 16 * 16  # bytes copied: the stencil's 1.07 GB moved = 537 MB read + 537 MB written
a = torch.empty(half // 4 + 64, device=dev).uniform_()
b = torch.empty_like(a)


def copy(off):
    return P.lhpc_probe_copy_u(C.c_void_p(a.data_ptr() + off), C.c_void_p(b.data_ptr() + off), C.c_int64(half),
                               C.c_int((half // 16 + 1023) // 1024), C.c_int(1024), C.c_int(1), C.c_int(3),
                               C.c_void_p(st.cuda_stream))


def timeit(off, iters=20):
    for _ in range(3):
        assert copy(off) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        copy(off)
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / iters


for rep in range(3):
    for off in (0, 4, 8, 16):
        t = timeit(off)
        print(json.dumps({"rep": rep, "offset_bytes": off, "us": t * 1e6, "TBps": 2 * half / t / 1e12}), flush=True)
