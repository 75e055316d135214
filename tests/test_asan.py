"""Host sanitizer runs (CPU, no GPU): the reference builds every Linux test
with -fsanitize=address (/root/reference/tests/CMakeLists.txt:6-9).  Device
code cannot be sanitized on the pool, so this covers the host code:
  - the plan-time CSR validation and XSLICE/XTILE re-encodings plus the file
    readers of liblhpc.so (tests/cpp/asan_plan.cpp, sources compiled in with
    ASan/UBSan), including out-of-range / negative col_idx and non-monotone
    row_ptr, which must come back as LHPC_ERR_BAD_CSR before any pass indexes
    a host array with them;
  - the sparse-grid drop-in headers (test_sparse_grid grid mode);
  - the oracle itself (oracle/asan_oracle.c)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def _make(d):
    r = subprocess.run(["make", "-C", os.path.join(ROOT, d), "asan"], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail(r.stdout[-2000:] + r.stderr[-2000:])


def _run(args, ok):
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=ENV)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert ok in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr


def test_asan_plan_builders_and_io():
    _make("tests/cpp")
    _run([os.path.join(ROOT, "tests/cpp/_build/asan/asan_plan")], "ALL OK (asan plan/io)")


def test_asan_sparse_grid():
    _make("tests/cpp")
    _run([os.path.join(ROOT, "tests/cpp/_build/asan/test_sparse_grid"), "grid"], "ALL OK (grid)")


def test_asan_oracle():
    _make("oracle")
    _run([os.path.join(ROOT, "oracle/_build/asan_oracle")], "ALL OK (asan oracle)")
