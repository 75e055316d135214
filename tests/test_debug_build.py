"""The debug build of the same C ABI (libhpc_amd/_lib_debug/liblhpc.so,
`make -C libhpc_amd/csrc debug`: -DLHPC_DEBUG_BOUNDS device traps on the
plan-built XTILE indices + -DLHPC_DEBUG_SYNC launch checks), the counterpart
of the reference's debug-only scatter bounds traps
(lib/gpu/radix_gpu/include/cuda_radix_scatter.cuh:87,174) and its synchronous
NDEBUG-off launch checks (cuda_radix_sort_v4.cu:104-107).  Valid inputs only:
a trap is a GPU fault, so no test provokes one on the device."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_SO = os.path.join(ROOT, "libhpc_amd", "_lib_debug", "liblhpc.so")


def test_debug_build_exports_same_abi():
    """CPU: the debug library exports every symbol the product library does."""
    import ctypes
    if not os.path.exists(DEBUG_SO):
        pytest.fail("debug build missing: run __graft_entry__.build() (make -C libhpc_amd/csrc debug)")
    prod = ctypes.CDLL(os.path.join(ROOT, "libhpc_amd", "_lib", "liblhpc.so"))
    dbg = ctypes.CDLL(DEBUG_SO)
    from tests.test_abi import declared_functions
    for name in declared_functions():
        getattr(prod, name)
        getattr(dbg, name)


@pytest.mark.gpu
def test_debug_build_runs_trap_free(gpu):
    env = dict(os.environ, LHPC_LIB_PATH=DEBUG_SO)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "debug_build_check.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DEBUG BUILD OK" in r.stdout
