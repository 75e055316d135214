"""C-ABI boundary checks that need no GPU: the library loads, exports every
function include/lhpc.h declares, and rejects bad arguments with the
documented status codes before touching a device."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from tests._support import ROOT

HEADER = os.path.join(ROOT, "include", "lhpc.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lhpc_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported(lhpc):
    names = declared_functions()
    assert len(names) >= 17
    for n in names:
        assert hasattr(lhpc.lib, n), f"{n} declared in lhpc.h but not exported"
    assert set(names) == set(lhpc.ABI_SYMBOLS), "python mirror's symbol list drifted from lhpc.h"


def test_nm_exports_match_header():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(ROOT, "libhpc_amd", "_lib", "liblhpc.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("lhpc_")}
    assert set(declared_functions()) <= exported


def test_no_unresolved_kernel_handles():
    """Every kernel the library launches has its host handle defined in the
    library: an undefined `lhpc::` symbol means a kernel instantiation whose
    host stub the compiler dropped (the aligned-segment reduce once lost its
    stubs to a host-pass check of a gfx950-only builtin) — the .so links, then
    fails at load or launch on the GPU box."""
    import subprocess
    for lib in ("_lib/liblhpc.so", "_lib/liblhpc_probe.so"):
        path = os.path.join(ROOT, "libhpc_amd", lib)
        if not os.path.exists(path):
            continue
        out = subprocess.run(["nm", "-C", "--undefined-only", path], capture_output=True, text=True,
                             check=True).stdout
        bad = [l.strip() for l in out.splitlines() if "lhpc::" in l]
        assert not bad, f"{lib}: unresolved: {bad[:4]}"


def test_abi_version_and_strerror(lhpc):
    assert lhpc.lib.lhpc_abi_version() == 1
    for st in (0, -1, -2, -3, -4, -5, -6):
        assert lhpc.lib.lhpc_strerror(st)
    assert b"invalid" in lhpc.lib.lhpc_strerror(-1)


def _create(lhpc, **kw):
    args = dict(dtype=0, n_rows=2, n_cols=2, nnz=2, row_ptr=np.array([0, 1, 2], np.int32), bits=32,
                col=np.array([0, 1], np.int32), val=np.ones(2, np.float32), flags=0)
    args.update(kw)
    h = C.c_void_p()
    st = lhpc.lib.lhpc_spmv_plan_create(
        C.byref(h), args["dtype"], args["n_rows"], args["n_cols"], args["nnz"],
        args["row_ptr"].ctypes.data if args["row_ptr"] is not None else None, args["bits"],
        args["col"].ctypes.data if args["col"] is not None else None,
        args["val"].ctypes.data if args["val"] is not None else None, None, 0, args["flags"])
    return st, h


@pytest.mark.parametrize("bad", [dict(dtype=7), dict(n_rows=-1), dict(bits=16), dict(row_ptr=None),
                                 dict(col=None), dict(nnz=-3)])
def test_plan_create_invalid_args(lhpc, bad):
    st, h = _create(lhpc, **bad)
    assert st == -1 and not h.value


def test_plan_create_bad_csr(lhpc):
    st, _ = _create(lhpc, row_ptr=np.array([0, 2, 1], np.int32))  # row_ptr[n] != nnz
    assert st == -2
    st, _ = _create(lhpc, row_ptr=np.array([1, 1, 2], np.int32))
    assert st == -2
    st, _ = _create(lhpc, col=np.array([0, 5], np.int32), flags=1)  # validate: col out of range
    assert st == -2


@pytest.mark.parametrize("col", [[0, 5], [0, -1], [0, 2], [-2147483648, 0]])
@pytest.mark.parametrize("flags", [0, 1 << 9, 1 << 6, 1 << 4])  # default, FORCE_XTILE, FORCE_XSLICE, FORCE_ROWGROUP
def test_plan_create_rejects_bad_columns_without_validate(lhpc, col, flags):
    """Out-of-range or negative col_idx is LHPC_ERR_BAD_CSR on every path,
    with or without LHPC_PLAN_VALIDATE: the layout builders index host
    arrays by column, so the check runs before any of them (and before the
    device is touched)."""
    st, h = _create(lhpc, col=np.array(col, np.int32), flags=flags)
    assert st == -2 and not h.value


def test_plan_create_rejects_decreasing_row_ptr_without_validate(lhpc):
    st, h = _create(lhpc, n_rows=3, row_ptr=np.array([0, 2, 1, 2], np.int32))
    assert st == -2 and not h.value
    st, h = _create(lhpc, n_rows=3, row_ptr=np.array([0, 2, 1, 2], np.int64), bits=64)
    assert st == -2 and not h.value


def test_plan_create_without_device_fails_loudly(lhpc):
    if lhpc.device_count() > 0:
        pytest.skip("a GPU is present")
    st, h = _create(lhpc)
    assert st != 0 and not h.value  # no silent CPU fallback


def test_null_plan_calls(lhpc):
    assert lhpc.lib.lhpc_spmv(None, None, None, 1, None) == -1
    assert lhpc.lib.lhpc_spmv_plan_destroy(None) == 0
    assert lhpc.lib.lhpc_blur_x_f32(None, None, 1, 1, 8, 8, 1, None) == -1
    assert lhpc.lib.lhpc_stencil7_f32(None, None, 1, 1, 1, 1, 1.0, 1.0, 1, None) == -1


def test_python_mirror_raises(lhpc):
    with pytest.raises(TypeError):
        lhpc.SpMVPlan(np.array([0, 1], np.int16), np.array([0], np.int32), np.ones(1, np.float32), 1)
    with pytest.raises(lhpc.LhpcError):
        lhpc.SpMVPlan(np.array([0, 1], np.int32), np.array([0], np.int32), np.ones(1, np.float32), -5)


def test_single_hip_runtime_with_torch():
    """liblhpc.so must share torch's HIP runtime (never two in one process)."""
    import subprocess, sys
    code = ("import sys; sys.path.insert(0, %r); import libhpc_amd, torch; "
            "m = open('/proc/self/maps').read(); "
            "print(len({l.split()[-1] for l in m.splitlines() if 'libamdhip64' in l}))" % ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True)
    assert out.stdout.strip() == "1"


def test_dist_calls_reject_bad_arguments_before_any_device_work(lhpc):
    """The multi-GPU entry points validate their arguments first (no device,
    no RCCL needed): null handles, bad ranks, a null window, foreign blobs."""
    import ctypes as C
    L = lhpc.lib
    h = C.c_void_p()
    assert L.lhpc_dist_comm_create_local(None, 2, 0, 0) == -1
    assert L.lhpc_dist_comm_create_local(C.byref(h), 0, 0, 0) == -1      # no ranks
    assert L.lhpc_dist_comm_create_local(C.byref(h), 2, 2, 0) == -1      # rank out of range
    assert L.lhpc_dist_comm_create_local(C.byref(h), 65, 0, 0) == -1     # > 64 ranks
    assert L.lhpc_dist_comm_create(C.byref(h), None, 1, 0, 0) == -1      # no unique id
    blob = (C.c_ubyte * lhpc.DIST_P2P_BLOB_BYTES)()
    assert L.lhpc_dist_p2p_export(None, None, 4, blob) == -1
    assert L.lhpc_dist_p2p_import(None, blob) == -1
    assert L.lhpc_dist_p2p_status(None) == -1
    assert L.lhpc_dist_spmv(None, None, None, None) == -1
    assert L.lhpc_dist_spmv_plan_destroy(None) == 0
    assert L.lhpc_dist_comm_destroy(None) == 0
    assert L.lhpc_dist_allreduce_sum_f64(None, None, 1, None) == -1
    assert L.lhpc_dist_stencil7_f32(None, None, None, 1, 1, 1, 1, 1.0, 1.0, None) == -1


def test_multi_device_plan_argument_checks(lhpc):
    """lhpc_spmv_plan_create's multi-device arguments are checked before any
    device is touched: n_devices > 1 needs device ids, at most 16 devices,
    and row splits are single-device only (CPU: no GPU needed)."""
    import ctypes as C
    rp = np.array([0, 1, 2], dtype=np.int32)
    col = np.array([0, 1], dtype=np.int32)
    val = np.ones(2, dtype=np.float32)
    h = C.c_void_p()
    args = (C.byref(h), lhpc.F32, 2, 2, 2, rp.ctypes.data, 32, col.ctypes.data, val.ctypes.data)
    assert lhpc.lib.lhpc_spmv_plan_create(*args, None, 2, 0) == -1  # no device ids
    assert lhpc.lib.lhpc_spmv_plan_create(*args, (C.c_int * 17)(*([0] * 17)), 17, 0) == -1  # > 16 devices
    assert lhpc.lib.lhpc_spmv_plan_create(*args, (C.c_int * 2)(0, 0), -1, 0) == -1
    sp = np.array([1], dtype=np.int64)
    assert lhpc.lib.lhpc_spmv_plan_create_opts(*args, (C.c_int * 2)(0, 0), 2, 0, 1, sp.ctypes.data, None) == -5
    assert not h.value


@pytest.mark.parametrize("py,c", [("Options", "lhpc_options"), ("PlanInfo", "lhpc_spmv_plan_info"),
                                  ("DistXfer", "lhpc_dist_xfer")])
def test_struct_mirrors_match_header(lhpc, tmp_path, py, c):
    """Every ctypes mirror of an lhpc.h struct (libhpc_amd.Options, PlanInfo,
    DistXfer) has the C struct's size and every field at the C offset: a
    probe compiled against include/lhpc.h prints sizeof and offsetof for each
    field the mirror names.  lhpc_options_init stamps struct_size = sizeof on
    the Options mirror."""
    import subprocess
    cls = getattr(lhpc, py)
    fields = [f[0] for f in cls._fields_]
    src = tmp_path / "probe.c"
    src.write_text("#include <stddef.h>\n#include <stdio.h>\n#include \"lhpc.h\"\nint main(void){\n"
                   f"printf(\"size %zu\\n\", sizeof({c}));\n"
                   + "".join(f"printf(\"{n} %zu\\n\", offsetof({c}, {n}));\n" for n in fields)
                   + "return 0;}\n")
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], capture_output=True, text=True,
                                                   check=True).stdout.splitlines())
    assert int(got["size"]) == C.sizeof(cls)
    for n in fields:
        assert int(got[n]) == getattr(cls, n).offset, n
    if py == "Options":
        o = lhpc.Options()
        lhpc.lib.lhpc_options_init(C.byref(o))
        assert o.struct_size == C.sizeof(lhpc.Options)


def test_host_allocation_failure_is_a_status_not_an_exception(lhpc):
    """No C++ exception crosses the C ABI (int status only): an
    entry point whose host work cannot allocate returns LHPC_ERR_ALLOC (-3)
    instead of terminating the caller's process.  The power-law generator
    asked for an 8-TiB length table (l_max = 2^40) fails that way before it
    writes anything."""
    import numpy as np
    rp = np.full(11, -7, dtype=np.int64)
    nnz = C.c_int64(0)
    st = lhpc.lib.lhpc_gen_powerlaw_row_ptr(10, 1 << 41, 1.8, 1, 1 << 40, 1, rp.ctypes.data, C.byref(nnz))
    assert st == -3, st
    assert (rp == -7).all()
