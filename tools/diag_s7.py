"""Diagnostic: per-index mismatches of stencil7 implementations on tiny shapes."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libhpc_amd as L
from tests import _support as S
dev = torch.device("cuda:0")
for impl in (sys.argv[1:] or ["buf", "wide"]):
    os.environ["LHPC_STENCIL7_IMPL"] = impl
    for (nz, ny, nx, g) in ((1, 1, 1, 1), (1, 1, 2, 1), (1, 2, 1, 1), (2, 1, 1, 1), (2, 3, 5, 1), (4, 8, 70, 1), (16, 17, 65, 1)):
        shape = (nz + 2 * g, ny + 2 * g, nx + 2 * g)
        u = S.random_padded(shape, seed=nz * 131 + nx, zero_ghost=False).reshape(-1)
        out0 = S.random_padded(shape, seed=99).reshape(-1)
        want = S.stencil7_oracle(u, nz, ny, nx, g, -6.0, 1.0, out=out0.copy())
        got = L.stencil7(torch.from_numpy(u).to(dev), torch.from_numpy(out0).to(dev), nz, ny, nx, g, -6.0, 1.0).cpu().numpy()
        bad = np.nonzero(got != want)[0]
        print(impl, (nz, ny, nx, g), "bad", len(bad), [(int(i), np.unravel_index(i, shape), float(got[i]), float(want[i]), float(out0[i])) for i in bad[:4]], flush=True)
