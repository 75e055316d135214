"""A/B of stencil kernel variants (env knobs read per launch)."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import libhpc_amd as L
dev = torch.device("cuda:0"); st = torch.cuda.current_stream()
def timeit(fn, iters=30):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters): fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3
n, g = 8192, 8
a = torch.rand((n + 2 * g) ** 2, device=dev) * 2 - 1
bb = torch.empty(n * n, device=dev)
ref = None
for rows in os.environ.get("BX_CFGS", "2 wave:2 wave:4 wave:8 wave:16 wave:32 2").split():
    if rows.startswith("wave"):
        os.environ["LHPC_BLUR_X_IMPL"] = "wave"
        os.environ["LHPC_BLUR_X_RW"] = rows.split(":")[1]
    else:
        os.environ["LHPC_BLUR_X_IMPL"] = "lds"
        os.environ["LHPC_BLUR_X_ROWS"] = rows
    t = timeit(lambda: L.blur_x(a, bb, n, n, g, 8, stream=st))
    out = bb.clone()
    if ref is None: ref = out
    print(json.dumps(dict(k="blur_x", rows=rows, us=t * 1e6, frac=8 * n * n / t / 8e12, same=bool(torch.equal(out, ref)))), flush=True)
ref = None
for cfg in ("4,16",):
    os.environ["LHPC_BLUR_Y_CFG"] = cfg
    t = timeit(lambda: L.blur_y(a, bb, n, n, g, 8, stream=st))
    out = bb.clone()
    if ref is None: ref = out
    print(json.dumps(dict(k="blur_y", cfg=cfg, us=t * 1e6, frac=8 * n * n / t / 8e12, same=bool(torch.equal(out, ref)))), flush=True)
del a, bb
m = 512; P = m + 2
u = torch.zeros(P ** 3, device=dev); u.view(P, P, P)[1:-1, 1:-1, 1:-1] = torch.rand(m, m, m, device=dev) * 2 - 1
o = torch.zeros_like(u)
ref = None
CFGS = os.environ.get("S7_CFGS", "default wide:2,8:nt buf:2,8,128:plain buf:4,4,128:plain buf:2,8,32:plain "
                                  "buf:2,8,128:none").split()
for simple in CFGS:
    parts = simple.split(":")
    if parts[0] == "default":
        for k in ("LHPC_STENCIL7_IMPL", "LHPC_STENCIL7_BUF", "LHPC_STENCIL7_WIDE", "LHPC_STENCIL7_STORE"):
            os.environ.pop(k, None)
        t = timeit(lambda: L.stencil7(u, o, m, m, m, 1, -6.0, 1.0, stream=st))
        ref = o.clone()
        o.zero_()
        print(json.dumps(dict(k="stencil7", simple="default", us=t * 1e6, frac=8 * m ** 3 / t / 8e12, same=True)), flush=True)
        continue
    os.environ["LHPC_STENCIL7_IMPL"] = parts[0]
    os.environ["LHPC_STENCIL7_WIDE" if parts[0] == "wide" else "LHPC_STENCIL7_BUF"] = parts[1]
    os.environ["LHPC_STENCIL7_STORE"] = parts[2] if len(parts) > 2 else "plain"
    t = timeit(lambda: L.stencil7(u, o, m, m, m, 1, -6.0, 1.0, stream=st))
    out = o.clone()
    if ref is None: ref = out
    o.zero_()
    print(json.dumps(dict(k="stencil7", simple=simple, us=t * 1e6, frac=8 * m ** 3 / t / 8e12, same=bool(torch.equal(out, ref)))), flush=True)
