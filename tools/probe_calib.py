"""Attainable-HBM calibration: 16-B/lane probes
(liblhpc_probe.so lhpc_probe_copy_u) over grid × block × unroll × cache
policy, for copy, read-only and write-only, at the byte count of the C2 XTILE
layout (2.52 GB moved per call: 1.26 GB each way for a copy).  Prints one JSON
line per configuration: GB/s of bytes moved (read + written)."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
total = int(float(os.environ.get("PROBE_BYTES", 2.52e9)))
half = total // 2 // (1 << 16) * (1 << 16)
src = torch.rand(half // 4, device=dev)
dst = torch.empty_like(src)


def timeit(fn, iters=10):
    with torch.cuda.stream(st):
        for _ in range(2):
            fn()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


MODES = {0: "copy", 1: "copy nt-load", 2: "copy nt-store", 3: "copy nt", 4: "read", 5: "read nt",
         8: "write", 10: "write nt"}
grids = [int(g) for g in os.environ.get("PROBE_GRIDS", "256,512,1024,2048,4096,16384,65536").split(",")]
best = {}
for mode, mname in MODES.items():
    moved = half if mode in (8, 10) else 2 * half  # read-only probes read src and dst: a copy's total
    for block in (256, 512, 1024):
        for unroll in (1, 2, 4, 8):
            for grid in grids:
                if mode in (4, 5):
                    def fn():
                        for buf in (src, dst):
                            rc = P.lhpc_probe_copy_u(C.c_void_p(buf.data_ptr()), C.c_void_p(dst.data_ptr()),
                                                     C.c_int64(half), C.c_int(grid), C.c_int(block),
                                                     C.c_int(unroll), C.c_int(mode), C.c_void_p(st.cuda_stream))
                            assert rc == 0, rc
                else:
                    def fn():
                        rc = P.lhpc_probe_copy_u(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                                 C.c_int64(half), C.c_int(grid), C.c_int(block), C.c_int(unroll),
                                                 C.c_int(mode), C.c_void_p(st.cuda_stream))
                        assert rc == 0, rc
                t = timeit(fn)
                gbps = moved / t / 1e9
                rec = dict(mode=mname, block=block, unroll=unroll, grid=grid, us=round(t * 1e6, 1),
                           GBps=round(gbps, 1))
                print(json.dumps(rec), flush=True)
                if gbps > best.get(mname, {}).get("GBps", 0):
                    best[mname] = rec
    if mode in (0, 1, 2, 3):
        assert torch.equal(src, dst), mname
        dst.zero_()
# the bench's own copy_ceiling configuration, for comparison
for width in (8, 16):
    t = timeit(lambda: P.lhpc_probe_copy_w(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), C.c_int64(half),
                                           C.c_int(16384), C.c_int(width), C.c_int(1), C.c_void_p(st.cuda_stream)))
    print(json.dumps(dict(mode=f"bench copy_w width {width} nt", us=round(t * 1e6, 1),
                          GBps=round(2 * half / t / 1e9, 1))), flush=True)
t = timeit(lambda: dst.copy_(src))
print(json.dumps(dict(mode="torch copy_", us=round(t * 1e6, 1), GBps=round(2 * half / t / 1e9, 1))), flush=True)
print(json.dumps({"best": best, "bytes_each_way": half}), flush=True)
