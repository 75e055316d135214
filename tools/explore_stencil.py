"""C5 (7-point stencil, 512^3 fp32) sweep over the x4-ring tiling options
(lhpc_options.stencil7_*: rows per wave, 64-column blocks per wave, z planes
per block / target grid, prefetch depth, store policy), every result checked
bit-exact against the default, next to the calibrated copy probe over the same
bytes.  One JSON line per configuration (µs per pass, Gcell/s, fraction of the
copy)."""
import ctypes as C
import itertools
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

dev = torch.device("cuda:0")
n, g = 512, 1
P = n + 2
u = torch.zeros(P ** 3, device=dev)
u.view(P, P, P)[1:-1, 1:-1, 1:-1] = torch.rand(n, n, n, device=dev) * 2 - 1
o = torch.zeros_like(u)
ref = torch.zeros_like(u)
st = torch.cuda.current_stream(dev)
L.stencil7(u, ref, n, n, n, g, -6.0, 1.0, stream=st)


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e-3 / iters


P_ = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
half = (8 * n ** 3 // 2) // 16 * 16
a = torch.empty(half // 4, device=dev).uniform_()
b = torch.empty_like(a)
copy_t = timeit(lambda: P_.lhpc_probe_copy_u(C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), C.c_int64(half),
                                             C.c_int((half // 16 + 1023) // 1024), C.c_int(1024), C.c_int(1),
                                             C.c_int(3), C.c_void_p(st.cuda_stream)))
print(json.dumps({"copy_us": copy_t * 1e6, "copy_GBps": 2 * half / copy_t / 1e9}), flush=True)
del a, b
base = timeit(lambda: L.stencil7(u, o, n, n, n, g, -6.0, 1.0, stream=st))
print(json.dumps({"cfg": "default", "us": base * 1e6, "frac_copy": copy_t / base}), flush=True)
if len(sys.argv) > 1 and sys.argv[1] == "ab":  # interleaved repeats: default against rows × blocks options
    # (round 5 also timed 8 and 16 waves per block through a since-removed
    # stencil7_waves option: 196–236 µs, profiles/r05/stencil_ab.jsonl)
    alts = [dict(stencil7_ry=2, stencil7_nj=4), dict(stencil7_ry=1, stencil7_nj=8), dict(stencil7_ry=1, stencil7_nj=4)]
    for rep in range(5):
        t = timeit(lambda: L.stencil7(u, o, n, n, n, g, -6.0, 1.0, stream=st))
        print(json.dumps({"rep": rep, "cfg": "default", "us": t * 1e6}), flush=True)
        for cfg in alts:
            t = timeit(lambda: L.stencil7(u, o, n, n, n, g, -6.0, 1.0, stream=st, options=cfg))
            print(json.dumps({"rep": rep, "cfg": cfg, "us": t * 1e6, "same": bool(torch.equal(o, ref))}), flush=True)
    sys.exit(0)
configs = []
for ry, nj in ((2, 4), (1, 8), (4, 4), (2, 8), (1, 4)):
    for blocks in (128, 256, 384, 512, 768, 1024, 2048):
        for pf in (1, 2, 3):
            configs.append(dict(stencil7_ry=ry, stencil7_nj=nj, stencil7_blocks=blocks, stencil7_pf=pf))
for zc in (4, 8, 16, 32):
    configs.append(dict(stencil7_ry=2, stencil7_nj=4, stencil7_zc=zc, stencil7_pf=2))
for cfg in configs:
    try:
        t = timeit(lambda: L.stencil7(u, o, n, n, n, g, -6.0, 1.0, stream=st, options=cfg), iters=10)
    except L.LhpcError as e:
        print(json.dumps({"cfg": cfg, "error": str(e)}), flush=True)
        continue
    same = bool(torch.equal(o, ref))
    print(json.dumps({"cfg": cfg, "us": t * 1e6, "frac_copy": copy_t / t, "same": same}), flush=True)
