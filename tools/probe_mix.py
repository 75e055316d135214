"""Read:write mix ceilings (round 5): what HBM moves when a stream writes W
bytes per byte read, W = 1 … 4 — the XTILE gather's mix (fp32: ≈ 1 : 1.4
with the x tiles; fp64: ≈ 1 : 2.6–3) against the 1:1 calibrated copy.
lhpc_probe_fan: one 16-KB tile read (non-temporal) and W tiles written per
1024-thread block, plain or non-temporal stores, ≈ 1.5 GB moved per launch; and with 96 KB of dynamic
LDS per block and a grid of 256 blocks walking the tiles (one 1024-thread
block per CU for the whole launch, as the XTILE gather runs).
One JSON line per (W, store policy, LDS, repeat): µs, TB/s moved, TB/s written.
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
TILE = 16384
MOVED = 1_500_000_000
src = torch.empty(MOVED // 2 // 4 + TILE, device=dev).uniform_()
dst = torch.empty(MOVED // 4 + TILE, device=dev)


def run(w, nt, lds=0, iters=20):
    tiles = MOVED // (TILE * (1 + w))

    def one():
        return P.lhpc_probe_fan(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), C.c_int64(tiles),
                                C.c_int(w), C.c_int(nt), C.c_int(256 if lds else int(tiles)), C.c_int(lds),
                                C.c_void_p(st.cuda_stream))
    for _ in range(3):
        assert one() == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        one()
    e1.record(st)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) * 1e-3 / iters
    moved = tiles * TILE * (1 + w)
    return t, moved, tiles * TILE * w


for rep in range(2):
    for w in (1, 2, 3, 4):
        for nt, lds in ((1, 0), (0, 0), (1, 96 * 1024)):
            t, moved, written = run(w, nt, lds)
            print(json.dumps({"rep": rep, "write_per_read": w, "nt_store": nt, "lds_bytes": lds, "us": t * 1e6,
                              "TBps": moved / t / 1e12, "write_TBps": written / t / 1e12}), flush=True)
