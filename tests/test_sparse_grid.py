"""The sparse-grid drop-in (include/sparse: RootGrid / HashBlock / PointerBlock /
DenseBlock) and sparse::to_csr, through tests/cpp/test_sparse_grid.

The reference's lib/sparse needs oneTBB, which is absent here, so
it cannot be built as an oracle; parity is pinned to its documented behaviour:
read/write round trips on its three benchmark layouts
(test_hpc_benchmark.cpp:859-925), its single-level foreach coordinates, and the
§2c-5 cells whose multi-level coordinates it reports wrongly ((-5,7) → (235,7),
(1000,-2000) → (1224,-1952)) and which must come back exact here."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP_DIR = os.path.join(ROOT, "tests", "cpp")
BIN = os.path.join(CPP_DIR, "_build", "test_sparse_grid")


def _bin():
    subprocess.run(["make", "-C", CPP_DIR, "_build/test_sparse_grid"], check=True, capture_output=True)
    return BIN


def test_sparse_grid_layouts_and_coordinates():
    r = subprocess.run([_bin(), "grid"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK (grid)" in r.stdout
    assert "BM_RootHashPointerDense: benchmark trajectory" in r.stdout


@pytest.mark.gpu
def test_to_csr_on_gpu(gpu):
    r = subprocess.run([_bin(), "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK (gpu)" in r.stdout
