"""GPU exploration: attainable-rate probes + SpMV / stencil kernel variants.

Run on the GPU box:  python tools/explore.py [--quick]
Prints one JSON object per measurement.  Development tool (not the bench).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    import torch
    import libhpc_amd as L
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream()
    sp = s.cuda_stream

    def timeit(fn, iters=20, warm=3):
        for _ in range(warm):
            fn()
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / iters * 1e-3  # seconds

    only = set(args.only.split(",")) if args.only else None

    # ---------------- probes
    if only is None or "probe" in only:
        P = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "liblhpc_probe.so"))
        nbytes = 1 << 30
        src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).uniform_()
        dst = torch.empty_like(src)
        for grid in (1024, 2048, 4096, 8192):
            t = timeit(lambda: P.lhpc_probe_copy(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                                 C.c_int64(nbytes), C.c_int(grid), C.c_void_p(sp)))
            emit(probe="copy16_nt", grid=grid, GBps=2 * nbytes / t / 1e9)
            t = timeit(lambda: P.lhpc_probe_read(C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()),
                                                 C.c_int64(nbytes), C.c_int(grid), C.c_void_p(sp)))
            emit(probe="read16_nt", grid=grid, GBps=nbytes / t / 1e9)
        del src, dst
        n = 150_000_000
        out = torch.empty(n, dtype=torch.float32, device=dev)
        for tbytes in (1 << 20, 4 << 20, 16 << 20, 40_000_000, 160 << 20, 400 << 20):
            tn = tbytes // 4
            table = torch.rand(tn, device=dev)
            idx = torch.randint(0, tn, (n,), dtype=torch.int32, device=dev)
            t = timeit(lambda: P.lhpc_probe_gather(C.c_void_p(idx.data_ptr()), C.c_void_p(table.data_ptr()),
                                                   C.c_void_p(out.data_ptr()), C.c_int64(n), C.c_void_p(sp)),
                       iters=10)
            emit(probe="gather4", table_MB=tbytes / 1e6, Ggather_per_s=n / t / 1e9,
                 stream_GBps=8 * n / t / 1e9, ms=t * 1e3)
            del table, idx
        del out
        torch.cuda.empty_cache()

    # ---------------- SpMV C2 (n=10M, 15/row, fp32)
    if only is None or "spmv" in only:
        for dtype_name, dt in (("f32", L.F32), ("f64", L.F64)):
            n = 1_000_000 if args.quick else 10_000_000
            t0 = time.time()
            rp, col, val = L.gen_uniform_csr(n, n, 15, dtype=dt)
            x = L.gen_values(dt, 0, n, L.SEED_X)
            emit(stage="gen", dtype=dtype_name, s=time.time() - t0)
            nnz = col.shape[0]
            tsz = 4 if dt == L.F32 else 8
            alg = nnz * (tsz + 4) + (n + 1) * 4 + 2 * n * tsz
            xd = torch.from_numpy(x).to(dev)
            yd = torch.empty(n, dtype=xd.dtype, device=dev)
            # correctness reference on a row sample (fp64)
            samp = np.random.default_rng(0).integers(0, n, 2000)
            ref = np.array([np.dot(val[rp[i]:rp[i + 1]].astype(np.float64),
                                   x[col[rp[i]:rp[i + 1]]].astype(np.float64)) for i in samp])
            configs = ["auto", "g:4", "g:16", "xs:2.5", "xs:1.25", "nb:2", "nopersist", "fast"]
            if dt == L.F64:
                configs = ["auto", "g:4", "xs:2.5", "xs:10", "nopersist"]
            for cfg in configs:
                flags = 0
                for k in ("LHPC_XSLICE_MB", "LHPC_XSLICE_LAYOUT", "LHPC_XSLICE_NB", "LHPC_XSLICE_PARTIAL",
                          "LHPC_XSLICE_FUSE", "LHPC_XSLICE_PERSIST", "LHPC_XSLICE_G"):
                    os.environ.pop(k, None)
                if cfg == "adaptive":
                    flags = L.PLAN_FORCE_ADAPTIVE
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                elif cfg.startswith("g:"):
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_G"] = cfg[2:]
                elif cfg == "nopersist":
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_PERSIST"] = "0"
                elif cfg == "nofuse":
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_FUSE"] = "0"
                elif cfg == "fast":
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    flags = L.PLAN_FAST_PARTIALS
                elif cfg == "p64":
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_PARTIAL"] = "f64"
                elif cfg == "auto":
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                elif cfg.startswith("jag:"):
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_MB"] = cfg[4:]
                    os.environ["LHPC_XSLICE_LAYOUT"] = "jagged"
                    flags = L.PLAN_FORCE_XSLICE
                elif cfg.startswith("nb:"):
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_NB"] = cfg[3:]
                    flags = L.PLAN_FORCE_XSLICE
                elif cfg.startswith("xs:"):
                    os.environ.pop("LHPC_SPMV_ROWGROUP", None)
                    os.environ["LHPC_XSLICE_MB"] = cfg[3:]
                else:
                    os.environ["LHPC_SPMV_ROWGROUP"] = cfg
                    flags = L.PLAN_FORCE_ROWGROUP
                t0 = time.time()
                plan = L.SpMVPlan(rp, col, val, n, flags=flags)
                tp = time.time() - t0
                t = timeit(lambda: plan(xd, yd, stream=s), iters=20)
                y = yd.cpu().numpy()
                err = np.max(np.abs(y[samp].astype(np.float64) - ref) / (np.abs(ref) + 1e-30))
                emit(kernel="spmv", dtype=dtype_name, cfg=cfg, info=plan.info(), us=t * 1e6,
                     GFLOPs=2 * nnz / t / 1e9, alg_GBps=alg / t / 1e9, frac8=alg / t / 8e12,
                     max_rel_err=float(err), plan_s=tp)
                plan.close()
            os.environ.pop("LHPC_SPMV_ROWGROUP", None)
            del xd, yd
            torch.cuda.empty_cache()
            # power-law
            if dt == L.F32:
                t0 = time.time()
                rp, col, val = L.gen_powerlaw_csr(n, n, dtype=dt)
                emit(stage="gen_powerlaw", s=time.time() - t0, nnz=int(col.shape[0]),
                     maxlen=int(np.max(np.diff(rp))))
                nnz = col.shape[0]
                alg = nnz * (tsz + 4) + (n + 1) * 4 + 2 * n * tsz
                xd = torch.from_numpy(x).to(dev)
                yd = torch.empty(n, dtype=xd.dtype, device=dev)
                ref = np.array([np.dot(val[rp[i]:rp[i + 1]].astype(np.float64),
                                       x[col[rp[i]:rp[i + 1]]].astype(np.float64)) for i in samp])
                for k in ("LHPC_XSLICE_MB", "LHPC_XSLICE_G", "LHPC_XSLICE_PERSIST"):
                    os.environ.pop(k, None)
                for cfg, flags in (("auto", 0), ("fast", L.PLAN_FAST_PARTIALS), ("g4", 0), ("xs2.5", 0)):
                    os.environ.pop("LHPC_XSLICE_G", None)
                    os.environ.pop("LHPC_XSLICE_MB", None)
                    if cfg == "g4":
                        os.environ["LHPC_XSLICE_G"] = "4"
                    if cfg == "xs2.5":
                        os.environ["LHPC_XSLICE_MB"] = "2.5"
                    plan = L.SpMVPlan(rp, col, val, n, flags=flags)
                    t = timeit(lambda: plan(xd, yd, stream=s), iters=10)
                    y = yd.cpu().numpy()
                    err = np.max(np.abs(y[samp].astype(np.float64) - ref) / (np.abs(ref) + 1e-30))
                    emit(kernel="spmv_powerlaw", cfg=cfg, info=plan.info(), us=t * 1e6,
                         GFLOPs=2 * nnz / t / 1e9, alg_GBps=alg / t / 1e9, frac8=alg / t / 8e12,
                         max_rel_err=float(err))
                    plan.close()
                del xd, yd
                torch.cuda.empty_cache()

    # ---------------- blur 8192² ghost 8
    if only is None or "blur" in only:
        ny = nx = 8192
        g = 8
        a = torch.rand((ny + 2 * g) * (nx + 2 * g), device=dev) * 2 - 1
        b = torch.empty(ny * nx, device=dev)
        A = a.view(ny + 2 * g, nx + 2 * g)
        for name, fn in (("blur_x", L.blur_x), ("blur_y", L.blur_y)):
            t = timeit(lambda: fn(a, b, ny, nx, g, 8, stream=s))
            # spot check 4 rows on host
            rows = [0, 1, 4095, 8191]
            Ah = A.cpu().numpy()
            bh = b.view(ny, nx).cpu().numpy()
            ok = True
            for r in rows:
                if name == "blur_x":
                    seg = Ah[r + g]
                    ref = np.zeros(nx, dtype=np.float32)
                    for k in range(-8, 9):
                        ref = ref + seg[g + k: g + k + nx]
                else:
                    ref = np.zeros(nx, dtype=np.float32)
                    for k in range(-8, 9):
                        ref = ref + Ah[r + g + k, g:g + nx]
                ok &= bool(np.array_equal(ref, bh[r]))
            emit(kernel=name, us=t * 1e6, alg_GBps=8 * ny * nx / t / 1e9,
                 frac8=8 * ny * nx / t / 8e12, bit_exact_rows=ok)
        del a, b
    if only is None or "stencil7" in only:
        n = 512
        g = 1
        P = n + 2
        u = torch.zeros(P * P * P, device=dev)
        U = u.view(P, P, P)
        U[1:-1, 1:-1, 1:-1] = torch.rand(n, n, n, device=dev) * 2 - 1
        o = torch.zeros_like(u)
        t = timeit(lambda: L.stencil7(u, o, n, n, n, 1, -6.0, 1.0, stream=s))
        # check a z-slab on host
        Uh = U[0:6].cpu().numpy().astype(np.float32)
        Oh = o.view(P, P, P)[1:5].cpu().numpy()
        c = Uh[1:5, 1:-1, 1:-1]
        ssum = (((((Uh[0:4, 1:-1, 1:-1] + Uh[2:6, 1:-1, 1:-1]) + Uh[1:5, 0:-2, 1:-1]) +
                  Uh[1:5, 2:, 1:-1]) + Uh[1:5, 1:-1, 0:-2]) + Uh[1:5, 1:-1, 2:])
        ref = np.float32(-6.0) * c + np.float32(1.0) * ssum
        emit(kernel="stencil7", us=t * 1e6, alg_GBps=8 * n ** 3 / t / 1e9,
             frac8=8 * n ** 3 / t / 8e12, Gcells=n ** 3 / t / 1e9,
             bit_exact_slab=bool(np.array_equal(ref, Oh[:, 1:-1, 1:-1])))


if __name__ == "__main__":
    main()
