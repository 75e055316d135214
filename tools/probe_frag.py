"""Fragment probe (round 6, VERDICT r5 items 1–2): the XTILE reduce's memory
access shape and occupancy without its compute (liblhpc_probe.so
lhpc_probe_frag, lhpc_probe.hip k_frag).  Per chunk of 8192 positions: one
row of the segment table (S u32), the S xg fragments of the chunk (tile-major
stream, ⌊8192/S⌋–⌈8192/S⌉ entries each, unaligned) into LDS in flat order,
and the val + iperm stream (wave-transposed, non-temporal).

  c3        fp64, S = 489, 150M positions (the C3 reduce: xg 1.2 GB from HBM),
            1024-thread blocks, the reduce's 73.9 KB of LDS (2 blocks per CU);
            fragment loads as b64 + ds_write (the reduce's form) and as 4-B
            LDS-DMA; also 1 block per CU
  c2        fp32, S = 256, 50M positions (one C2 cache-sized range: xg 200 MB),
            512-thread blocks, the reduce's 40.1 KB of LDS (4 blocks per CU):
              ic   xg written (plain stores, as the gather) right before: the
                   fragments come from the Infinity Cache
              hbm  xg written, then 1 GB of other data written: from HBM
  c3r       fp64, S = 489, 25M positions (one of C3's six ring ranges: xg 200 MB
            written right before, from the Infinity Cache), 1024-thread
            blocks at the reduce's LDS (2 per CU)
  ring      C2 call shape: three 200-MB xg writes each followed by its probe,
            into three distinct buffers (the plan's xg[total]) or one reused
            buffer; the writes and the probes timed apart (does the dirty-line
            write-back of distinct buffers cost the writes?)

One JSON line per case: µs per launch (HIP events on the launch stream),
the bytes the probe moves, TB/s.  Compare with the reduce's rocprof average
from the same session (c2_kernel_stats / c3_kernel_stats)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L  # noqa: E402

P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
dev = torch.device("cuda:0")
st = torch.cuda.Stream(dev)
M = 8192
sink = torch.zeros(1, dtype=torch.float64, device=dev)


def seg_table(S, Cn):
    fs = (np.arange(S + 1, dtype=np.int64) * M) // S
    ln = np.diff(fs)
    c = np.arange(Cn, dtype=np.int64)[:, None]
    return torch.from_numpy((Cn * fs[None, :S] + c * ln[None, :]).astype(np.uint32).reshape(-1).view(np.int32)).to(dev)


def lds_bytes(t, S):  # lhpc_spmv_xtile.hip xtile_lds_bytes_g for G = 1
    blk = 512 if t == 4 else 1024
    w, run = blk // 64, 64 // t
    rmax = blk * run // 8
    return (M + 16 // t) * t + w * run * 16 + w * 12 + 2 * M // 32 * 4 + ((rmax + 2) & ~1) * 2 + 4 * (S + 8)


class Case:
    def __init__(self, t, S, nnz):
        self.t, self.S = t, S
        self.C = (nnz + M - 1) // M
        n = self.C * M
        dt = torch.float32 if t == 4 else torch.float64
        self.seg = seg_table(S, self.C)
        self.xg = torch.rand(n, dtype=dt, device=dev)
        self.val = torch.rand(n, dtype=dt, device=dev)
        self.ip = torch.zeros(n, dtype=torch.int16, device=dev)
        self.moved = n * (2 * t + 2) + self.C * S * 4  # xg + val + iperm + segment rows

    def launch(self, f64_dma=0, lds=None, xg=None):
        xg = self.xg if xg is None else xg
        rc = P.lhpc_probe_frag(C.c_void_p(self.seg.data_ptr()), C.c_void_p(xg.data_ptr()),
                               C.c_int64(xg.numel() * self.t), C.c_void_p(self.val.data_ptr()),
                               C.c_void_p(self.ip.data_ptr()), C.c_int(self.S), C.c_int64(self.C), C.c_int(self.t),
                               C.c_int(f64_dma), C.c_int(lds or lds_bytes(self.t, self.S)),
                               C.c_void_p(sink.data_ptr()), C.c_void_p(st.cuda_stream))
        assert rc == 0, rc


def write(buf):  # 16-B/lane plain stores over buf (the gather's store policy for C2)
    rc = P.lhpc_probe_copy_u(C.c_void_p(buf.data_ptr()), C.c_void_p(buf.data_ptr()),
                             C.c_int64(buf.numel() * buf.element_size()), C.c_int(2048), C.c_int(1024), C.c_int(1),
                             C.c_int(8), C.c_void_p(st.cuda_stream))
    assert rc == 0, rc


def timed(pre, fn, iters=20):
    """mean µs of fn per iteration, pre (untimed on the events) before each"""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    with torch.cuda.stream(st):
        for _ in range(3):
            pre()
            fn()
        for a, b in ev:
            pre()
            a.record(st)
            fn()
            b.record(st)
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    return float(np.mean(ts)), ts[len(ts) // 2]


def out(**kw):
    print(json.dumps(kw), flush=True)


which = sys.argv[1:] or ["c3", "c2", "ring"]
for rep in range(2):
    if "c3" in which:
        c3 = Case(8, 489, 150_000_000)
        junk = torch.empty(256 << 18, dtype=torch.float32, device=dev)  # 1 GB
        for f64_dma in (0, 1):
            for blocks in (2, 1):
                lds = lds_bytes(8, 489) if blocks == 2 else 96 * 1024
                us, med = timed(lambda: write(junk), lambda: c3.launch(f64_dma, lds))
                out(case="c3", rep=rep, f64_dma=f64_dma, blocks_per_cu=blocks, lds=lds, us=us, us_median=med,
                    moved=c3.moved, TBps=c3.moved / us * 1e-6)
        del c3, junk
        torch.cuda.empty_cache()
    if "c3r" in which:
        c3r = Case(8, 489, 25_000_000)
        for blocks in (2, 1):
            lds = lds_bytes(8, 489) if blocks == 2 else 96 * 1024
            us, med = timed(lambda: write(c3r.xg), lambda: c3r.launch(0, lds))
            out(case="c3r", rep=rep, xg_from="ic", blocks_per_cu=blocks, lds=lds, us=us, us_median=med,
                moved=c3r.moved, TBps=c3r.moved / us * 1e-6)
        del c3r
        torch.cuda.empty_cache()
    if "c2" in which:
        c2 = Case(4, 256, 50_000_000)
        junk = torch.empty(256 << 18, dtype=torch.float32, device=dev)
        for src in ("ic", "hbm"):
            for blocks in (4, 3, 2):
                lds = {4: lds_bytes(4, 256), 3: 52 * 1024, 2: 80 * 1024}[blocks]
                pre = (lambda: write(c2.xg)) if src == "ic" else (lambda: (write(c2.xg), write(junk)))
                us, med = timed(pre, lambda: c2.launch(0, lds))
                out(case="c2", rep=rep, xg_from=src, blocks_per_cu=blocks, lds=lds, us=us, us_median=med,
                    moved=c2.moved, TBps=c2.moved / us * 1e-6)
        del junk
        if "ring" in which:
            bufs = [c2.xg, torch.empty_like(c2.xg), torch.empty_like(c2.xg)]
            for form in ("distinct", "ring"):
                tw, tp = [], []
                for _ in range(10):
                    ev = []
                    with torch.cuda.stream(st):
                        for k in range(3):
                            b = bufs[k] if form == "distinct" else bufs[0]
                            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                            e[0].record(st)
                            write(b)
                            e[1].record(st)
                            c2.launch(0, None, b)
                            e[2].record(st)
                            ev.append(e)
                    torch.cuda.synchronize()
                    tw.append(sum(e[0].elapsed_time(e[1]) for e in ev) * 1e3)
                    tp.append(sum(e[1].elapsed_time(e[2]) for e in ev) * 1e3)
                out(case="ring", rep=rep, form=form, write_us_per_call=float(np.median(tw[2:])),
                    probe_us_per_call=float(np.median(tp[2:])))
        del c2
        torch.cuda.empty_cache()
