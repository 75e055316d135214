"""Drop-in host layout: our include/hpc/HPCHighDimensionFlatArray.hpp must
place every cell exactly where the reference's lib/hpc header does.

The expected offsets in tests/golden/layout.json were printed by
oracle/_ref/ref_probe — a driver compiled against the reference header itself
(HPCHighDimensionFlatArray.hpp:161-187, at() :107-109).  The C++ test program
tests/cpp/test_cpp_api prints the same points through our header (and links two
translation units, which the reference's AlignedAlloc.hpp cannot: SURVEY §2c-1).
"""
import json
import os
import subprocess

import pytest

from tests._support import GOLDEN, REF_PROBE, ROOT

CPP_DIR = os.path.join(ROOT, "tests", "cpp")
CPP_BIN = os.path.join(CPP_DIR, "_build", "test_cpp_api")


def build_cpp():
    subprocess.run(["make", "-C", CPP_DIR], check=True, capture_output=True)
    return CPP_BIN


def test_dropin_layout_matches_reference_header():
    exe = build_cpp()
    ours = json.loads(subprocess.run([exe, "layout"], check=True, capture_output=True, text=True).stdout)
    ref = json.load(open(os.path.join(GOLDEN, "layout.json")))["cases"]
    assert ours == ref


def test_golden_layout_reproducible_from_reference_probe():
    if not os.path.exists(REF_PROBE):
        pytest.skip("oracle/_ref/ref_probe not built (needs /root/reference at build time)")
    ref = json.load(open(os.path.join(GOLDEN, "layout.json")))["cases"]
    r = subprocess.run([REF_PROBE, "layout2", "5", "7", "8"], check=True, capture_output=True, text=True)
    assert json.loads(r.stdout) == ref[0]


def test_python_padded_shape_matches(lhpc):
    assert lhpc.padded_shape((8192, 8192), 8) == (8208, 8208)
    assert lhpc.padded_shape((512, 512, 512), 1) == (514, 514, 514)


@pytest.mark.gpu
def test_cpp_api_on_gpu(gpu):
    exe = build_cpp()
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "ok" in r.stdout
