"""libhpc_amd — MI355X-native libHPC hot path (CSR SpMV + ghost-cell stencils).

Python mirror of the C ABI in ``include/lhpc.h`` (ctypes over the in-tree
``libhpc_amd/_lib/liblhpc.so``).  The C++ drop-in surface lives in
``include/hpc/*.hpp`` and ``include/sparse/*.hpp``; this module exists so the
tests and ``bench.py`` drive exactly the same entry points a C++ caller would.

There is deliberately no CPU fallback: if the shared library is missing this
module raises at import, and every compute call raises ``LhpcError`` when no
gfx950 device is present.  (The CPU restatement used as the checker lives in
``oracle/`` and is imported only by tests and bench's ``cpu_baseline`` leg.)

Reference anchors (read-only, /root/reference):
  * layout contract: lib/hpc/include/HPCHighDimensionFlatArray.hpp:54-57, 161-187
  * blur semantics:  tests/test_hpc_benchmark/test_hpc_benchmark.cpp:354-368, 444-457
  * error idiom:     lib/gpu/util/include/cudaHelper.cuh:10-27 (std::system_error)
  * SpMV: absent from the reference; defined in DESIGN.md.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np

__all__ = [
    "LhpcError", "lib", "F32", "F64", "device_count", "SpMVPlan",
    "csr_partition_rows", "blur_x", "blur_y", "stencil7", "stencil7_planes",
    "gen_uniform_csr", "gen_powerlaw_csr", "gen_values", "padded_shape",
    "PLAN_VALIDATE", "PLAN_FORCE_ROWGROUP", "PLAN_FORCE_ADAPTIVE", "PLAN_FORCE_XSLICE", "PLAN_FAST_PARTIALS", "PLAN_EXACT_PARTIALS",
    "PLAN_FORCE_XTILE", "PLAN_FORCE_SELL", "KERNEL_XTILE", "KERNEL_SELL",
    "KERNEL_ROWGROUP", "KERNEL_ADAPTIVE", "KERNEL_XSLICE",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# LHPC_LIB_PATH: an alternative build of the same ABI (same-box A/B runs, tools/gpu_ab.sh)
LIB_PATH = os.environ.get("LHPC_LIB_PATH") or os.path.join(_HERE, "_lib", "liblhpc.so")

F32, F64 = 0, 1
PLAN_VALIDATE = 1 << 0
PLAN_DEVICE_INPUT = 1 << 1
PLAN_FORCE_ROWGROUP = 1 << 4
PLAN_FORCE_ADAPTIVE = 1 << 5
PLAN_FORCE_XSLICE = 1 << 6
PLAN_FAST_PARTIALS = 1 << 7
PLAN_EXACT_PARTIALS = 1 << 8
PLAN_FORCE_XTILE = 1 << 9
PLAN_FORCE_SELL = 1 << 10
KERNEL_ROWGROUP, KERNEL_ADAPTIVE, KERNEL_XSLICE, KERNEL_XTILE, KERNEL_SELL = 0, 1, 2, 3, 4

# every symbol include/lhpc.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = (
    "lhpc_strerror", "lhpc_abi_version", "lhpc_build_flags", "lhpc_device_count",
    "lhpc_spmv_plan_create", "lhpc_spmv", "lhpc_spmv_plan_info_get",
    "lhpc_spmv_plan_destroy", "lhpc_csr_partition_rows",
    "lhpc_blur_x_f32", "lhpc_blur_y_f32", "lhpc_stencil7_f32",
    "lhpc_stencil7_f32_planes", "lhpc_gen_uniform_row_ptr",
    "lhpc_gen_powerlaw_row_ptr", "lhpc_gen_fill_cols", "lhpc_gen_fill_values",
    "lhpc_row_ptr_narrow", "lhpc_radix_sort_u32", "lhpc_radix_sort_pairs_u32",
    "lhpc_radix_sort_pairs_u64", "lhpc_coo_to_csr", "lhpc_csr_save", "lhpc_csr_load_header",
    "lhpc_csr_load", "lhpc_mm_read_header", "lhpc_mm_read_coo", "lhpc_cg_solve", "lhpc_vec_dot",
    "lhpc_cg_step_xr", "lhpc_cg_step_p", "lhpc_cg_step_r", "lhpc_cg_step_xp", "lhpc_spmv_dot",
    "lhpc_spmv_plan_create_split", "lhpc_spmv_stage", "lhpc_spmv_range",
    "lhpc_dist_get_unique_id", "lhpc_dist_comm_create", "lhpc_dist_comm_info", "lhpc_dist_comm_destroy",
    "lhpc_dist_allreduce_sum_f64", "lhpc_dist_spmv_plan_create", "lhpc_dist_spmv",
    "lhpc_dist_spmv_plan_destroy", "lhpc_dist_stencil7_f32", "lhpc_dist_stencil7_f32_x", "lhpc_dist_comm_create_local",
    "lhpc_dist_p2p_export", "lhpc_dist_p2p_import", "lhpc_dist_p2p_status",
    "lhpc_options_init", "lhpc_spmv_plan_create_opts", "lhpc_blur_x_f32_opts", "lhpc_blur_y_f32_opts",
    "lhpc_stencil7_f32_planes_opts", "lhpc_dist_spmv_plan_create_opts", "lhpc_dist_exchange",
    "lhpc_dist_exchange_schedule", "lhpc_dist_p2p_reset", "lhpc_dist_p2p_unmap", "lhpc_scratch_trim", "lhpc_scratch_poison",
    "lhpc_spmv_multi", "lhpc_spmv_plan_multi_info", "lhpc_dist_spmv_begin", "lhpc_dist_spmv_end",
    "lhpc_dist_chain_parts", "lhpc_dist_allgather_f64", "lhpc_dist_cg_solve", "lhpc_dist_spmv_plan_info",
    "lhpc_spmv_plan_layout_digest", "lhpc_dist_rccl_calls",
)

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"libhpc_amd: native library {LIB_PATH} is missing; build it with "
        "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")

def _bind_single_hip_runtime():
    """One HIP runtime and one RCCL per process.  PyTorch-ROCm bundles its own
    libamdhip64 and librccl (SONAMEs libamdhip64.so.7 / librccl.so.1, like
    /opt/rocm's); if ours were loaded first, torch would later load its
    copies as a second runtime (and see no GPU).  Importing torch first makes
    liblhpc.so bind to torch's copies, in torch's own load order."""
    try:
        import torch  # noqa: F401
    except Exception:  # a broken torch install must not make the C ABI unusable
        pass


_bind_single_hip_runtime()
lib = C.CDLL(LIB_PATH)
BUILD_TUNING, BUILD_DEBUG, BUILD_PROBE, BUILD_AB = 1, 2, 4, 8
BUILD_FLAGS = lib.lhpc_build_flags()
if BUILD_FLAGS & BUILD_PROBE and os.environ.get("LHPC_ALLOW_PROBE_BUILD") != "1":
    # a timing-only probe build skips work and computes wrong results: only
    # an explicit opt-in (the tools/ A/B scripts) may load it
    raise ImportError(f"{LIB_PATH} is a timing-only probe build (lhpc_build_flags = {BUILD_FLAGS}); "
                      "set LHPC_ALLOW_PROBE_BUILD=1 to time it")
_p, _i, _i64, _u, _u64, _f, _d = (C.c_void_p, C.c_int, C.c_int64, C.c_uint,
                                  C.c_uint64, C.c_float, C.c_double)


class Options(C.Structure):
    """include/lhpc.h lhpc_options: explicit variant choices (0 = automatic).
    ``Options(xtile_reduce=XTILE_REDUCE_PERM, ...)``; unknown names raise."""
    _fields_ = [("struct_size", C.c_uint32), ("spmv_no_xtile", C.c_int32), ("spmv_locality", C.c_double),
                ("rowgroup_lanes", C.c_int32), ("rowgroup_rows", C.c_int32),
                ("xtile_reduce", C.c_int32), ("xtile_ranges", C.c_int32), ("xtile_steps", C.c_int32),
                ("xtile_store", C.c_int32), ("xtile_cut", C.c_int32), ("xtile_align", C.c_int32),
                ("xtile_piece", C.c_int64), ("xtile_range_piece", C.c_int64),
                ("xslice_slices", C.c_int32), ("xslice_partial", C.c_int32), ("xslice_window", C.c_int32),
                ("xslice_reserved", C.c_int32), ("xslice_mb", C.c_double),
                ("stencil7_impl", C.c_int32), ("stencil7_store", C.c_int32), ("stencil7_ry", C.c_int32),
                ("stencil7_nj", C.c_int32), ("stencil7_zc", C.c_int32), ("stencil7_pf", C.c_int32),
                ("stencil7_blocks", C.c_int32), ("blur_x_rows", C.c_int32), ("blur_y_vec", C.c_int32),
                ("blur_y_rows", C.c_int32), ("dist_exchange", C.c_int32), ("dist_broadcast", C.c_int32),
                ("dist_world1", C.c_int32), ("xtile_part_nnz", C.c_int32), ("multi_chunks", C.c_int32),
                ("multi_exchange", C.c_int32), ("multi_force", C.c_int32), ("dist_reduce_streams", C.c_int32),
                ("xtile_col_blocks", C.c_int32), ("xtile_host_build", C.c_int32), ("spmv_no_sell", C.c_int32),
                ("xtile_ring", C.c_int32), ("xtile_pretable", C.c_int32)]

    def __init__(self, **kw):
        super().__init__()
        lib.lhpc_options_init(C.byref(self))
        names = {f[0] for f in self._fields_}
        for k, v in kw.items():
            if k not in names or k == "struct_size":
                raise TypeError(f"unknown option {k!r}")
            setattr(self, k, v)


def _opts(o):
    if o is None:
        return None
    if isinstance(o, dict):
        o = Options(**o)
    return C.byref(o)


XTILE_REDUCE_AUTO, XTILE_REDUCE_PERM, XTILE_REDUCE_IPERM = 0, 1, 2
XTILE_ALIGN_AUTO, XTILE_ALIGN_OFF, XTILE_ALIGN_UNITS = 0, 1, 2
S7_AUTO, S7_SIMPLE, S7_RING, S7_RING_X4, S7_RING_X4_LDS = 0, 1, 2, 3, 4
STORE_AUTO, STORE_PLAIN, STORE_NT, STORE_STAGED = 0, 1, 2, 3
DIST_EXCHANGE_AUTO, DIST_EXCHANGE_RCCL, DIST_EXCHANGE_P2P, DIST_EXCHANGE_NONE = 0, 1, 2, 3
XFER_ALLGATHER, XFER_BROADCAST, XFER_PUSH = 1, 2, 3


class DistXfer(C.Structure):
    _fields_ = [("chunk", C.c_int32), ("kind", C.c_int32), ("root", C.c_int32), ("group", C.c_int32),
                ("offset", C.c_int64), ("count", C.c_int64), ("send_offset", C.c_int64)]


class RcclCall(C.Structure):
    """include/lhpc.h lhpc_rccl_call: one RCCL call of the y exchange."""
    _fields_ = [("chunk", C.c_int32), ("op", C.c_int32), ("root", C.c_int32), ("datatype", C.c_int32),
                ("group_begin", C.c_int32), ("group_end", C.c_int32), ("send_byte_offset", C.c_int64),
                ("recv_byte_offset", C.c_int64), ("count", C.c_int64)]


class PlanInfo(C.Structure):
    _fields_ = [("dtype", _i), ("kernel", _i), ("lanes_per_row", _i),
                ("rows_per_group", _i), ("n_rows", _i64), ("n_cols", _i64),
                ("nnz", _i64), ("n_blocks", _i64), ("n_long_rows", _i64),
                ("device_bytes", _i64), ("device", _i), ("launches", _i),
                ("slices", _i), ("slice_width", _i64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def _sig(name, res, *args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_sig("lhpc_strerror", C.c_char_p, _i)
_sig("lhpc_abi_version", _i)
_sig("lhpc_build_flags", _i)
_sig("lhpc_device_count", _i)
_sig("lhpc_spmv_plan_create", _i, C.POINTER(_p), _i, _i64, _i64, _i64, _p, _i, _p,
     _p, _p, _i, _u)
_sig("lhpc_spmv", _i, _p, _p, _p, _i, _p)
_sig("lhpc_spmv_plan_create_split", _i, C.POINTER(_p), _i, _i64, _i64, _i64, _p, _i, _p,
     _p, _p, _i, _u, _i, _p)
_sig("lhpc_spmv_plan_create_opts", _i, C.POINTER(_p), _i, _i64, _i64, _i64, _p, _i, _p,
     _p, _p, _i, _u, _i, _p, _p)
_sig("lhpc_options_init", None, _p)
_sig("lhpc_spmv_stage", _i, _p, _p, _p)
_sig("lhpc_spmv_range", _i, _p, _i, _p, _p)
_sig("lhpc_spmv_plan_info_get", _i, _p, C.POINTER(PlanInfo))
_sig("lhpc_spmv_multi", _i, _p, _p, _p, _p)
_sig("lhpc_spmv_plan_layout_digest", _i, _p, _p, _i, C.POINTER(_i))
_sig("lhpc_spmv_plan_multi_info", _i, _p, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i), _p, _p)
_sig("lhpc_spmv_plan_destroy", _i, _p)
_sig("lhpc_csr_partition_rows", _i, _p, _i, _i64, _i, _p)
for _n in ("lhpc_blur_x_f32", "lhpc_blur_y_f32"):
    _sig(_n, _i, _p, _p, _i64, _i64, _i64, _i, _i, _p)
_sig("lhpc_stencil7_f32", _i, _p, _p, _i64, _i64, _i64, _i64, _f, _f, _i, _p)
for _n in ("lhpc_blur_x_f32_opts", "lhpc_blur_y_f32_opts"):
    _sig(_n, _i, _p, _p, _i64, _i64, _i64, _i, _i, _p, _p)
_sig("lhpc_stencil7_f32_planes_opts", _i, _p, _p, _i64, _i64, _i64, _i64, _f, _f, _i64, _i64, _p, _p)
_sig("lhpc_stencil7_f32_planes", _i, _p, _p, _i64, _i64, _i64, _i64, _f, _f, _i64,
     _i64, _p)
_sig("lhpc_gen_uniform_row_ptr", _i, _i64, _i, _p)
_sig("lhpc_gen_powerlaw_row_ptr", _i, _i64, _i64, _d, _i64, _i64, _u64, _p, _p)
_sig("lhpc_gen_fill_cols", _i, _i64, _i64, _p, _u64, _p)
_sig("lhpc_gen_fill_values", _i, _i, _i, _i64, _u64, _p)
_sig("lhpc_row_ptr_narrow", _i, _p, _i64, _p)
_sig("lhpc_radix_sort_u32", _i, _p, _i64, _i, _i, _i, _p)
_sig("lhpc_radix_sort_pairs_u32", _i, _p, _p, _i64, _i, _i, _i, _p)
_sig("lhpc_radix_sort_pairs_u64", _i, _p, _p, _i64, _i, _i, _i, _p)
_sig("lhpc_scratch_trim", _i, _i)
_sig("lhpc_scratch_poison", _i, _i64, _i, _p)
_sig("lhpc_coo_to_csr", _i, _i, _i64, _i64, _i64, _p, _p, _p, _p, _i, _p, _p, C.POINTER(_i64), _i, _p)
_sig("lhpc_cg_solve", _i, _p, _p, _p, _d, _i, _i, C.POINTER(_i), C.POINTER(_d), _p)
_sig("lhpc_vec_dot", _i, _i, _i64, _p, _p, _p, _p)
_sig("lhpc_spmv_dot", _i, _p, _p, _p, _p, _p, _p)
_sig("lhpc_cg_step_xr", _i, _i, _i64, _p, _p, _p, _p, _p, _p, _p, _p)
_sig("lhpc_cg_step_p", _i, _i, _i64, _p, _p, _p, _p, _p)
_sig("lhpc_cg_step_r", _i, _i, _i64, _p, _p, _p, _p, _p, _p)
_sig("lhpc_cg_step_xp", _i, _i, _i64, _p, _p, _p, _p, _p, _p, _p, _p)
_sig("lhpc_csr_save", _i, C.c_char_p, _i, _i64, _i64, _i64, _p, _i, _p, _p)
_sig("lhpc_csr_load_header", _i, C.c_char_p, C.POINTER(_i), C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64),
     C.POINTER(_i))
_sig("lhpc_csr_load", _i, C.c_char_p, _p, _p, _p)
_sig("lhpc_mm_read_header", _i, C.c_char_p, C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i64), C.POINTER(_i),
     C.POINTER(_i))
_sig("lhpc_mm_read_coo", _i, C.c_char_p, _p, _p, _p, C.POINTER(_i64))
if hasattr(lib, "lhpc_probe_xtile_stamps"):  # diagnostic build only (tools/xt_stamps.py)
    _sig("lhpc_probe_xtile_stamps", _i, _p, _i64)
    _sig("lhpc_probe_xtile_stamps_clear", _i)
_sig("lhpc_dist_get_unique_id", _i, _p)
_sig("lhpc_dist_comm_create", _i, C.POINTER(_p), _p, _i, _i, _i)
_sig("lhpc_dist_comm_info", _i, _p, C.POINTER(_i), C.POINTER(_i), C.POINTER(_i))
_sig("lhpc_dist_comm_destroy", _i, _p)
_sig("lhpc_dist_allreduce_sum_f64", _i, _p, _p, _i64, _p)
_sig("lhpc_dist_allgather_f64", _i, _p, _p, _i64, _p, _p)
_sig("lhpc_dist_cg_solve", _i, _p, _p, _p, _p, _d, _i, _i, C.POINTER(_i), C.POINTER(_d), _p)
_sig("lhpc_dist_spmv_plan_create", _i, C.POINTER(_p), _p, _i, _i64, _i64, _i, _p, _p, _i, _p, _p, _u)
_sig("lhpc_dist_spmv_plan_create_opts", _i, C.POINTER(_p), _p, _i, _i64, _i64, _i, _p, _p, _i, _p, _p, _u, _p)
_sig("lhpc_dist_spmv", _i, _p, _p, _p, _p)
_sig("lhpc_dist_spmv_begin", _i, _p, _p, _p, _p)
_sig("lhpc_dist_spmv_end", _i, _p, _p)
_sig("lhpc_dist_spmv_plan_info", _i, _p, C.POINTER(PlanInfo), C.POINTER(_i))
_sig("lhpc_dist_chain_parts", _i, _p, _i, _i, _i64, _i64, _p, _i64)
_sig("lhpc_dist_exchange", _i, _p, _p, _p)
_sig("lhpc_dist_exchange_schedule", _i, _p, _i, _i, _i, _i, _i, _p, _i64, C.POINTER(_i64))
_sig("lhpc_dist_rccl_calls", _i, _p, _i, _i, _i, _i, _i, _p, _i64, C.POINTER(_i64))
_sig("lhpc_dist_p2p_reset", _i, _p)
_sig("lhpc_dist_p2p_unmap", _i, _p, _p)
_sig("lhpc_dist_spmv_plan_destroy", _i, _p)
_sig("lhpc_dist_stencil7_f32", _i, _p, _p, _p, _i64, _i64, _i64, _i64, _f, _f, _p)
_sig("lhpc_dist_stencil7_f32_x", _i, _p, _p, _p, _i64, _i64, _i64, _i64, _f, _f, _i, _p)
_sig("lhpc_dist_comm_create_local", _i, C.POINTER(_p), _i, _i, _i)
_sig("lhpc_dist_p2p_export", _i, _p, _p, _i64, _p)
_sig("lhpc_dist_p2p_import", _i, _p, _p)
_sig("lhpc_dist_p2p_status", _i, _p)


class LhpcError(RuntimeError):
    """Non-zero status from the C ABI (negative: lhpc, positive: hipError_t)."""

    def __init__(self, status: int, where: str = ""):
        self.status = status
        msg = lib.lhpc_strerror(status).decode()
        super().__init__(f"{where}: {msg} (status {status})" if where else msg)


def _check(st: int, where: str):
    if st != 0:
        raise LhpcError(st, where)


def device_count() -> int:
    return lib.lhpc_device_count()


# ------------------------------------------------------------ buffers
def _is_torch(t) -> bool:
    return type(t).__module__.startswith("torch") and hasattr(t, "data_ptr")


def _buf(a, dtype=None, writable=False):
    """(pointer, on_device) for a numpy array or a torch tensor."""
    if _is_torch(a):
        if not a.is_contiguous():
            raise ValueError("tensor must be contiguous")
        return a.data_ptr(), bool(a.is_cuda)
    if not isinstance(a, np.ndarray):
        raise TypeError(f"expected numpy array or torch tensor, got {type(a)}")
    if dtype is not None and a.dtype != dtype:
        raise TypeError(f"expected dtype {dtype}, got {a.dtype}")
    if not a.flags.c_contiguous or (writable and not a.flags.writeable):
        raise ValueError("array must be C-contiguous (and writable for outputs)")
    return a.ctypes.data, False


def _stream_ptr(stream) -> Optional[int]:
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)  # torch.cuda.Stream


# ------------------------------------------------------------ SpMV
class SpMVPlan:
    """RAII plan for y = A·x (mirrors sparse::SpMVPlan<T> in include/sparse/SpMV.hpp).

    ``row_ptr`` int32/int64 (n_rows+1), ``col_idx`` int32 (nnz), ``val``
    float32/float64 (nnz), all host numpy arrays; A is copied to HBM once.
    """

    def __init__(self, row_ptr, col_idx, val, n_cols: int, flags: int = 0,
                 device: Optional[int] = None, splits=None, options=None, devices=None):
        """``splits``: ascending rows in (0, n_rows); the plan is then a
        row-range plan (lhpc_spmv_plan_create_split: stage(x) once, then
        range(k, y_k) per range) and raises LhpcError (LHPC_ERR_UNSUPPORTED)
        when the matrix does not select the XTILE layout.  ``options``: an
        Options (or dict of its fields) pinning kernel variants
        (lhpc_spmv_plan_create_opts).  ``devices``: a list of HIP device
        ordinals for a single-process multi-device plan (a
        device may repeat: several shares of one GPU); ``plan(x, y)`` then
        takes x, y on devices[0] and ``plan.multi(xs, ys)`` full replicas."""
        if _is_torch(row_ptr) and row_ptr.is_cuda:
            # device-resident CSR (LHPC_PLAN_DEVICE_INPUT): validated and, for
            # XTILE, laid out on the GPU; the tensors must live on the plan's device
            import torch
            if row_ptr.dtype not in (torch.int32, torch.int64) or col_idx.dtype != torch.int32:
                raise TypeError("device row_ptr int32/int64 and col_idx int32")
            if val.dtype not in (torch.float32, torch.float64):
                raise TypeError("val must be float32 or float64")
            for t in (row_ptr, col_idx, val):
                if not (t.is_cuda and t.is_contiguous()):
                    raise ValueError("device CSR arrays must be contiguous CUDA tensors")
            flags |= PLAN_DEVICE_INPUT
            self.dtype = F32 if val.dtype == torch.float32 else F64
            self.np_dtype = np.dtype(np.float32 if self.dtype == F32 else np.float64)
            if device is None and devices is None:
                device = row_ptr.device.index
            self._dev_arrays = (row_ptr, col_idx, val)
            rp_ptr, rp_bits = row_ptr.data_ptr(), 64 if row_ptr.dtype == torch.int64 else 32
            col_ptr, val_ptr = col_idx.data_ptr(), val.data_ptr()
        else:
            row_ptr = np.ascontiguousarray(row_ptr)
            col_idx = np.ascontiguousarray(col_idx, dtype=np.int32)
            val = np.ascontiguousarray(val)
            if row_ptr.dtype not in (np.int32, np.int64):
                raise TypeError("row_ptr must be int32 or int64")
            if val.dtype == np.float32:
                self.dtype = F32
            elif val.dtype == np.float64:
                self.dtype = F64
            else:
                raise TypeError("val must be float32 or float64")
            self.np_dtype = val.dtype
            rp_ptr, rp_bits = row_ptr.ctypes.data, 64 if row_ptr.dtype == np.int64 else 32
            col_ptr, val_ptr = col_idx.ctypes.data, val.ctypes.data
        self.n_rows = int(row_ptr.shape[0] - 1)
        self.n_cols = int(n_cols)
        self.nnz = int(col_idx.shape[0])
        self._h = _p()
        if devices is not None:
            devices = [int(d) for d in devices]
            dev = (_i * len(devices))(*devices)
            ndev = len(devices)
        else:
            dev = (_i * 1)(device) if device is not None else None
            ndev = 1 if device is not None else 0
        self.devices = devices
        self._opts = options if not isinstance(options, dict) else Options(**options)
        if splits is None and options is None:
            self.splits = None
            _check(lib.lhpc_spmv_plan_create(
                C.byref(self._h), self.dtype, self.n_rows, self.n_cols, self.nnz,
                rp_ptr, rp_bits, col_ptr, val_ptr, dev, ndev, flags), "lhpc_spmv_plan_create")
        else:
            sp = np.ascontiguousarray(splits if splits is not None else [], dtype=np.int64)
            self.splits = None if splits is None else [0] + [int(v) for v in sp] + [self.n_rows]
            _check(lib.lhpc_spmv_plan_create_opts(
                C.byref(self._h), self.dtype, self.n_rows, self.n_cols, self.nnz,
                rp_ptr, rp_bits, col_ptr, val_ptr, dev, ndev,
                flags, int(sp.shape[0]), sp.ctypes.data if sp.shape[0] else None, _opts(self._opts)),
                "lhpc_spmv_plan_create_opts")

    def info(self) -> dict:
        inf = PlanInfo()
        _check(lib.lhpc_spmv_plan_info_get(self._h, C.byref(inf)), "lhpc_spmv_plan_info_get")
        return inf.as_dict()

    def layout_digest(self):
        """lhpc_spmv_plan_layout_digest: FNV-1a digests of an XTILE plan's
        device layout arrays (test support)."""
        out = (C.c_uint64 * 10)()
        n = _i()
        _check(lib.lhpc_spmv_plan_layout_digest(self._h, out, 10, C.byref(n)), "lhpc_spmv_plan_layout_digest")
        return [int(v) for v in out[:n.value]]

    def multi_info(self) -> dict:
        """lhpc_spmv_plan_multi_info: devices, chunks K, exchange, row cuts."""
        nd, k, ex = _i(), _i(), _i()
        _check(lib.lhpc_spmv_plan_multi_info(self._h, C.byref(nd), C.byref(k), C.byref(ex), None, None),
               "lhpc_spmv_plan_multi_info")
        ids = (_i * nd.value)()
        cuts = np.zeros(nd.value * k.value + 1, dtype=np.int64)
        _check(lib.lhpc_spmv_plan_multi_info(self._h, None, None, None, ids, cuts.ctypes.data),
               "lhpc_spmv_plan_multi_info")
        return {"n_devices": nd.value, "chunks": k.value, "exchange": ex.value, "devices": list(ids), "cuts": cuts}

    def multi(self, xs, ys, streams=None):
        """lhpc_spmv_multi: full replicas, xs[d]/ys[d] device tensors on
        device d; every ys[d] holds the whole y afterwards (asynchronous on
        ``streams[d]``, default torch's current stream of each device)."""
        import torch
        n = len(xs)
        if len(ys) != n:
            raise ValueError("one x and one y per device")
        for x, y in zip(xs, ys):
            if x.shape[0] < self.n_cols or y.shape[0] < self.n_rows:
                raise ValueError("x/y too short for the plan")
        if streams is None:
            streams = [torch.cuda.current_stream(x.device) for x in xs]
        xa = (_p * n)(*[x.data_ptr() for x in xs])
        ya = (_p * n)(*[y.data_ptr() for y in ys])
        sa = (_p * n)(*[_stream_ptr(s) for s in streams])
        _check(lib.lhpc_spmv_multi(self._h, xa, ya, sa), "lhpc_spmv_multi")
        return ys

    def __call__(self, x, y=None, stream=None):
        """y = A·x.  numpy in → numpy out (synchronous); torch CUDA tensors →
        asynchronous on ``stream`` (default: torch's current stream)."""
        if y is None:
            if _is_torch(x):
                import torch
                y = torch.empty(self.n_rows, dtype=x.dtype, device=x.device)
            else:
                y = np.empty(self.n_rows, dtype=self.np_dtype)
        if x.shape[0] < self.n_cols or y.shape[0] < self.n_rows:
            raise ValueError("x/y too short for the plan")
        xp, xd = _buf(x, None if _is_torch(x) else self.np_dtype)
        yp, yd = _buf(y, None if _is_torch(y) else self.np_dtype, writable=True)
        if xd != yd:
            raise ValueError("x and y must both be host or both be device buffers")
        if xd and stream is None:
            import torch
            stream = torch.cuda.current_stream(y.device)
        _check(lib.lhpc_spmv(self._h, xp, yp, int(xd), _stream_ptr(stream)), "lhpc_spmv")
        return y

    def stage(self, x, stream=None):
        """Row-range plans: stage x (device tensor) for the ranges that follow."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(x.device)
        _check(lib.lhpc_spmv_stage(self._h, x.data_ptr(), _stream_ptr(stream)), "lhpc_spmv_stage")

    def range(self, k: int, y_k, stream=None):
        """Row-range plans: rows [splits[k], splits[k+1]) of A·x into y_k (device)."""
        if y_k.shape[0] < self.splits[k + 1] - self.splits[k]:
            raise ValueError("y_k too short for the range")
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(y_k.device)
        _check(lib.lhpc_spmv_range(self._h, int(k), y_k.data_ptr(), _stream_ptr(stream)), "lhpc_spmv_range")
        return y_k

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib.lhpc_spmv_plan_destroy(self._h)
            self._h = _p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def csr_partition_rows(row_ptr: np.ndarray, parts: int) -> np.ndarray:
    row_ptr = np.ascontiguousarray(row_ptr)
    cuts = np.empty(parts + 1, dtype=np.int64)
    _check(lib.lhpc_csr_partition_rows(row_ptr.ctypes.data,
                                       64 if row_ptr.dtype == np.int64 else 32,
                                       row_ptr.shape[0] - 1, parts, cuts.ctypes.data),
           "lhpc_csr_partition_rows")
    return cuts


# ------------------------------------------------------------ stencils
def padded_shape(dims, ghost):
    """Physical shape of HPCHighDimensionFlatArray<D,T,ghost> with logical dims."""
    return tuple(int(d) + 2 * int(ghost) for d in dims)


def _blur(fn, fn_opts, name, a, b, ny, nx, ghost, nblur, stream, options):
    ap, ad = _buf(a, None if _is_torch(a) else np.float32)
    bp, bd = _buf(b, None if _is_torch(b) else np.float32, writable=True)
    if ad != bd:
        raise ValueError("a and b must both be host or both be device buffers")
    if ad and stream is None:
        import torch
        stream = torch.cuda.current_stream(b.device)
    if options is None:
        _check(fn(ap, bp, ny, nx, ghost, nblur, int(ad), _stream_ptr(stream)), name)
    else:
        _check(fn_opts(ap, bp, ny, nx, ghost, nblur, int(ad), _stream_ptr(stream), _opts(options)), name + "_opts")
    return b


def blur_x(a, b, ny: int, nx: int, ghost: int, nblur: int = 8, stream=None, options=None):
    """b(y,x) = Σ_{k=-nblur..nblur} a(y,x+k) (test_hpc_benchmark.cpp:354-368)."""
    return _blur(lib.lhpc_blur_x_f32, lib.lhpc_blur_x_f32_opts, "lhpc_blur_x_f32", a, b, ny, nx, ghost, nblur,
                 stream, options)


def blur_y(a, b, ny: int, nx: int, ghost: int, nblur: int = 8, stream=None, options=None):
    """b(y,x) = Σ_{k=-nblur..nblur} a(y+k,x) (test_hpc_benchmark.cpp:444-457)."""
    return _blur(lib.lhpc_blur_y_f32, lib.lhpc_blur_y_f32_opts, "lhpc_blur_y_f32", a, b, ny, nx, ghost, nblur,
                 stream, options)


def stencil7(u, out, nz: int, ny: int, nx: int, ghost: int = 1, c0: float = -6.0,
             c1: float = 1.0, stream=None, options=None):
    """options (device tensors only): lhpc_stencil7_f32_planes_opts over every plane."""
    if options is not None:
        return stencil7_planes(u, out, nz, ny, nx, ghost, c0, c1, 0, nz, stream=stream, options=options)
    up, ud = _buf(u, None if _is_torch(u) else np.float32)
    op, od = _buf(out, None if _is_torch(out) else np.float32, writable=True)
    if ud != od:
        raise ValueError("u and out must both be host or both be device buffers")
    if ud and stream is None:
        import torch
        stream = torch.cuda.current_stream(out.device)
    _check(lib.lhpc_stencil7_f32(up, op, nz, ny, nx, ghost, c0, c1, int(ud),
                                 _stream_ptr(stream)), "lhpc_stencil7_f32")
    return out


def stencil7_planes(u, out, nz, ny, nx, ghost, c0, c1, z_begin, z_end, stream=None, options=None):
    up, ud = _buf(u)
    op, od = _buf(out, writable=True)
    if not (ud and od):
        raise ValueError("stencil7_planes takes device tensors")
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(out.device)
    if options is None:
        _check(lib.lhpc_stencil7_f32_planes(up, op, nz, ny, nx, ghost, c0, c1, z_begin, z_end,
                                            _stream_ptr(stream)), "lhpc_stencil7_f32_planes")
    else:
        _check(lib.lhpc_stencil7_f32_planes_opts(up, op, nz, ny, nx, ghost, c0, c1, z_begin, z_end,
                                                 _stream_ptr(stream), _opts(options)),
               "lhpc_stencil7_f32_planes_opts")
    return out


# ------------------------------------------------------------ workloads
SEED_A = 0x5EED0001   # matrix columns / values
SEED_X = 0x5EED0002   # x vector


def gen_values(dtype, dist: int, count: int, seed: int) -> np.ndarray:
    npd = np.float32 if dtype in (F32, np.float32) else np.float64
    out = np.empty(count, dtype=npd)
    _check(lib.lhpc_gen_fill_values(F32 if npd == np.float32 else F64, dist, count, seed,
                                    out.ctypes.data), "lhpc_gen_fill_values")
    return out


def _finish_csr(row_ptr64, n_rows, n_cols, seed, dtype, dist, narrow):
    nnz = int(row_ptr64[-1])
    col = np.empty(nnz, dtype=np.int32)
    _check(lib.lhpc_gen_fill_cols(n_rows, n_cols, row_ptr64.ctypes.data, seed,
                                  col.ctypes.data), "lhpc_gen_fill_cols")
    val = gen_values(dtype, dist, nnz, seed ^ 0xA5A5)
    rp = row_ptr64
    if narrow and nnz <= np.iinfo(np.int32).max:
        rp = np.empty(n_rows + 1, dtype=np.int32)
        _check(lib.lhpc_row_ptr_narrow(row_ptr64.ctypes.data, n_rows + 1, rp.ctypes.data),
               "lhpc_row_ptr_narrow")
    return rp, col, val


def gen_uniform_csr(n_rows: int, n_cols: int, per_row: int, dtype=F32, dist: int = 0,
                    seed: int = SEED_A, narrow: bool = True):
    """Every row: exactly ``per_row`` distinct uniform sorted columns."""
    rp = np.empty(n_rows + 1, dtype=np.int64)
    _check(lib.lhpc_gen_uniform_row_ptr(n_rows, per_row, rp.ctypes.data),
           "lhpc_gen_uniform_row_ptr")
    return _finish_csr(rp, n_rows, n_cols, seed, dtype, dist, narrow)


def gen_powerlaw_csr(n_rows: int, n_cols: int, alpha: float = 1.792, lmin: int = 1,
                     lmax: int = 10_000, dtype=F32, dist: int = 0, seed: int = SEED_A,
                     narrow: bool = True):
    """Row lengths ~ l^-alpha on [lmin,lmax]; rows 0, n/2, n-1 forced to lmax."""
    rp = np.empty(n_rows + 1, dtype=np.int64)
    nnz = C.c_int64()
    _check(lib.lhpc_gen_powerlaw_row_ptr(n_rows, n_cols, alpha, lmin, lmax, seed ^ 0x1111,
                                         rp.ctypes.data, C.byref(nnz)),
           "lhpc_gen_powerlaw_row_ptr")
    return _finish_csr(rp, n_rows, n_cols, seed, dtype, dist, narrow)


# ------------------------------------------------------------ radix sort / COO→CSR
def _elem_bytes(a) -> int:
    return a.element_size() if _is_torch(a) else a.dtype.itemsize


def _numel(a) -> int:
    return a.numel() if _is_torch(a) else a.size


def _dev_stream(a, stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream(a.device)
    return stream


def radix_sort(keys, begin_bit: int = 0, end_bit: Optional[int] = None, stream=None):
    """Sort 32-bit unsigned keys in place, ascending (LSD, 8-bit digits over
    bits [begin_bit, end_bit)).  Mirrors sort::gpu::radix::radix_sort
    (reference lib/gpu/radix_gpu/src/radix_sort_gpu.cpp:24-29), which sorts a
    uint32 vector in place.  ``keys``: numpy uint32 array or a contiguous
    4-byte torch tensor on the GPU (int32 tensors are sorted as their uint32
    bit patterns).  Returns ``keys``."""
    if _elem_bytes(keys) != 4 or (not _is_torch(keys) and keys.dtype != np.uint32):
        raise TypeError("radix_sort: keys must be uint32 (numpy) or a 4-byte tensor")
    kp, kd = _buf(keys, writable=True)
    eb = 32 if end_bit is None else end_bit
    st = _dev_stream(keys, stream) if kd else None
    _check(lib.lhpc_radix_sort_u32(kp, _numel(keys), begin_bit, eb, int(kd), _stream_ptr(st)),
           "lhpc_radix_sort_u32")
    return keys


def radix_sort_pairs(keys, vals, begin_bit: int = 0, end_bit: Optional[int] = None, stream=None):
    """Stable in-place sort of (key, value) pairs: keys uint32 or uint64
    (numpy) / 4- or 8-byte tensors, values 4-byte.  Equal keys keep their
    input order."""
    kb = _elem_bytes(keys)
    if kb not in (4, 8) or _elem_bytes(vals) != 4 or _numel(keys) != _numel(vals):
        raise TypeError("radix_sort_pairs: keys 4/8-byte, values 4-byte, same length")
    if not _is_torch(keys) and keys.dtype not in (np.uint32, np.uint64):
        raise TypeError("radix_sort_pairs: numpy keys must be uint32 or uint64")
    kp, kd = _buf(keys, writable=True)
    vp, vd = _buf(vals, writable=True)
    if kd != vd:
        raise ValueError("keys and vals must both be host or both be device buffers")
    eb = kb * 8 if end_bit is None else end_bit
    st = _dev_stream(keys, stream) if kd else None
    fn = lib.lhpc_radix_sort_pairs_u64 if kb == 8 else lib.lhpc_radix_sort_pairs_u32
    _check(fn(kp, vp, _numel(keys), begin_bit, eb, int(kd), _stream_ptr(st)), fn.__name__)
    return keys, vals


def coo_to_csr(n_rows: int, n_cols: int, rows, cols, vals, row_ptr_bits: int = 64, stream=None):
    """CSR from coordinate triples on the GPU (sort by (row, col), duplicates
    summed in input order).  Host numpy inputs → numpy (row_ptr, col_idx, val);
    device tensors → device tensors.  See include/lhpc.h lhpc_coo_to_csr."""
    nnz = _numel(rows)
    if _numel(cols) != nnz or _numel(vals) != nnz:
        raise ValueError("rows, cols and vals must have the same length")
    vb = _elem_bytes(vals)
    dtype = F32 if vb == 4 else F64
    rp_, rd = _buf(rows, None if _is_torch(rows) else np.int32)
    cp_, cd = _buf(cols, None if _is_torch(cols) else np.int32)
    vp_, vd = _buf(vals, None if _is_torch(vals) else (np.float32 if vb == 4 else np.float64))
    if not (rd == cd == vd):
        raise ValueError("inputs must all be host or all be device buffers")
    out_n = C.c_int64(0)
    if rd:
        import torch
        dev = rows.device
        row_ptr = torch.empty(n_rows + 1, dtype=torch.int64 if row_ptr_bits == 64 else torch.int32, device=dev)
        col = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
        val = torch.empty(max(nnz, 1), dtype=vals.dtype, device=dev)
        st = _dev_stream(rows, stream)
        _check(lib.lhpc_coo_to_csr(dtype, n_rows, n_cols, nnz, rp_, cp_, vp_, row_ptr.data_ptr(), row_ptr_bits,
                                   col.data_ptr(), val.data_ptr(), C.byref(out_n), 1, _stream_ptr(st)),
               "lhpc_coo_to_csr")
        return row_ptr, col[:out_n.value], val[:out_n.value]
    row_ptr = np.empty(n_rows + 1, dtype=np.int64 if row_ptr_bits == 64 else np.int32)
    col = np.empty(max(nnz, 1), dtype=np.int32)
    val = np.empty(max(nnz, 1), dtype=np.float32 if vb == 4 else np.float64)
    _check(lib.lhpc_coo_to_csr(dtype, n_rows, n_cols, nnz, rp_, cp_, vp_, row_ptr.ctypes.data, row_ptr_bits,
                               col.ctypes.data, val.ctypes.data, C.byref(out_n), 0, None), "lhpc_coo_to_csr")
    return row_ptr, col[:out_n.value].copy(), val[:out_n.value].copy()


# ------------------------------------------------------------ files (.lcsr, Matrix Market)
def save_csr(path: str, row_ptr, col_idx, val, n_cols: int):
    """Write a host CSR (row_ptr int32/int64, col_idx int32, val f32/f64) as .lcsr."""
    rp = np.ascontiguousarray(row_ptr)
    col = np.ascontiguousarray(col_idx, dtype=np.int32)
    v = np.ascontiguousarray(val)
    dt = F32 if v.dtype == np.float32 else F64
    if v.dtype not in (np.float32, np.float64) or rp.dtype not in (np.int32, np.int64):
        raise TypeError("save_csr: row_ptr int32/int64, val float32/float64")
    _check(lib.lhpc_csr_save(os.fsencode(path), dt, rp.size - 1, n_cols, col.size, rp.ctypes.data,
                             64 if rp.dtype == np.int64 else 32, col.ctypes.data, v.ctypes.data), "lhpc_csr_save")


def load_csr(path: str):
    """(row_ptr, col_idx, val, n_cols) from an .lcsr file."""
    dt, rpb = C.c_int(0), C.c_int(0)
    nr, nc, nz = C.c_int64(0), C.c_int64(0), C.c_int64(0)
    _check(lib.lhpc_csr_load_header(os.fsencode(path), C.byref(dt), C.byref(nr), C.byref(nc), C.byref(nz),
                                    C.byref(rpb)), "lhpc_csr_load_header")
    rp = np.empty(nr.value + 1, dtype=np.int64 if rpb.value == 64 else np.int32)
    col = np.empty(nz.value, dtype=np.int32)
    val = np.empty(nz.value, dtype=np.float32 if dt.value == F32 else np.float64)
    _check(lib.lhpc_csr_load(os.fsencode(path), rp.ctypes.data, col.ctypes.data, val.ctypes.data), "lhpc_csr_load")
    return rp, col, val, nc.value


def read_matrix_market_coo(path: str):
    """(rows int32, cols int32, vals float64, n_rows, n_cols): 0-based triples,
    symmetric / skew-symmetric files expanded to both triangles."""
    nr, nc, zmax = C.c_int64(0), C.c_int64(0), C.c_int64(0)
    sym, fld = C.c_int(0), C.c_int(0)
    p = os.fsencode(path)
    _check(lib.lhpc_mm_read_header(p, C.byref(nr), C.byref(nc), C.byref(zmax), C.byref(sym), C.byref(fld)),
           "lhpc_mm_read_header")
    rows = np.empty(max(zmax.value, 1), dtype=np.int32)
    cols = np.empty(max(zmax.value, 1), dtype=np.int32)
    vals = np.empty(max(zmax.value, 1), dtype=np.float64)
    cnt = C.c_int64(0)
    _check(lib.lhpc_mm_read_coo(p, rows.ctypes.data, cols.ctypes.data, vals.ctypes.data, C.byref(cnt)),
           "lhpc_mm_read_coo")
    k = cnt.value
    return rows[:k].copy(), cols[:k].copy(), vals[:k].copy(), nr.value, nc.value


def read_matrix_market(path: str, dtype=F64, row_ptr_bits: int = 64):
    """CSR (row_ptr, col_idx, val, n_cols) from a Matrix Market file: parsed on
    the host, assembled on the GPU (lhpc_coo_to_csr; duplicates summed)."""
    rows, cols, vals, n_rows, n_cols = read_matrix_market_coo(path)
    v = vals.astype(np.float32) if dtype == F32 else vals
    rp, col, val = coo_to_csr(n_rows, n_cols, rows, cols, v, row_ptr_bits=row_ptr_bits)
    return rp, col, val, n_cols


# ------------------------------------------------------------ CG
def _dtype_code(t) -> int:
    return F32 if _elem_bytes(t) == 4 else F64


def cg(plan: "SpMVPlan", b, x=None, tol: float = 1e-8, max_iter: int = 1000, check_every: int = 1,
       stream=None):
    """Solve A·x = b (A SPD, the plan's matrix) by conjugate gradient on the
    GPU.  ``b`` (and ``x``, the initial guess, default 0) are device tensors
    of the plan's dtype; x is updated in place.  Returns (x, iterations,
    ‖r‖/‖b‖).  See include/lhpc.h lhpc_cg_solve."""
    import torch
    if x is None:
        x = torch.zeros_like(b)
    bp, bd = _buf(b)
    xp, xd = _buf(x, writable=True)
    if not (bd and xd):
        raise ValueError("cg: b and x must be device tensors")
    st = _dev_stream(b, stream)
    it, res = C.c_int(0), C.c_double(0.0)
    _check(lib.lhpc_cg_solve(plan._h, bp, xp, tol, max_iter, check_every, C.byref(it), C.byref(res),
                             _stream_ptr(st)), "lhpc_cg_solve")
    return x, it.value, res.value


def spmv_dot(plan: "SpMVPlan", x, y, w, out, stream=None):
    """y = A·x and out (1-element float64 device tensor) = w·y, asynchronously
    (one pass for ADAPTIVE plans)."""
    st = _dev_stream(x, stream)
    _check(lib.lhpc_spmv_dot(plan._h, x.data_ptr(), y.data_ptr(), w.data_ptr(), out.data_ptr(), _stream_ptr(st)),
           "lhpc_spmv_dot")
    return y, out


def vec_dot(a, b, out, stream=None):
    """out (1-element float64 device tensor) = a·b, asynchronously."""
    st = _dev_stream(a, stream)
    _check(lib.lhpc_vec_dot(_dtype_code(a), _numel(a), _buf(a)[0], _buf(b)[0], out.data_ptr(), _stream_ptr(st)),
           "lhpc_vec_dot")
    return out


def cg_step_xr(alpha_num, alpha_den, x, p, r, q, rr_out, stream=None):
    st = _dev_stream(x, stream)
    _check(lib.lhpc_cg_step_xr(_dtype_code(x), _numel(x), alpha_num.data_ptr(), alpha_den.data_ptr(), x.data_ptr(),
                               p.data_ptr(), r.data_ptr(), q.data_ptr(), rr_out.data_ptr(), _stream_ptr(st)),
           "lhpc_cg_step_xr")


def cg_step_p(beta_num, beta_den, r, p, stream=None):
    st = _dev_stream(r, stream)
    _check(lib.lhpc_cg_step_p(_dtype_code(r), _numel(r), beta_num.data_ptr(), beta_den.data_ptr(), r.data_ptr(),
                              p.data_ptr(), _stream_ptr(st)), "lhpc_cg_step_p")


def cg_step_r(alpha_num, alpha_den, r, q, rr_out, stream=None):
    """r -= α·q, rr_out = r·r (α = alpha_num/alpha_den, fp64 device scalars)."""
    st = _dev_stream(r, stream)
    _check(lib.lhpc_cg_step_r(_dtype_code(r), _numel(r), alpha_num.data_ptr(), alpha_den.data_ptr(), r.data_ptr(),
                              q.data_ptr(), rr_out.data_ptr(), _stream_ptr(st)), "lhpc_cg_step_r")


def cg_step_xp(alpha_num, alpha_den, beta_num, beta_den, x, p, r, stream=None):
    """x += α·p, then p = r + β·p in the same pass; beta_num None: x only."""
    st = _dev_stream(x, stream)
    bn = beta_num.data_ptr() if beta_num is not None else None
    bd = beta_den.data_ptr() if beta_den is not None else None
    rp = r.data_ptr() if r is not None else None
    _check(lib.lhpc_cg_step_xp(_dtype_code(x), _numel(x), alpha_num.data_ptr(), alpha_den.data_ptr(), bn, bd,
                               x.data_ptr(), p.data_ptr(), rp, _stream_ptr(st)), "lhpc_cg_step_xp")


def gen_laplacian_2d(nx: int, ny: int, dtype=F64, shift: float = 0.0):
    """5-point Dirichlet Laplacian on an nx×ny grid (row i = y·nx + x;
    diagonal 4 + shift, −1 to each existing neighbour): symmetric positive
    definite, columns sorted.  Returns (row_ptr int64, col_idx int32, val).
    Host-side workload generator for the CG solver."""
    n = nx * ny
    i = np.arange(n, dtype=np.int64)
    y, x = np.divmod(i, nx)
    off = np.array([-nx, -1, 0, 1, nx], dtype=np.int64)  # ascending column order
    mask = np.stack([y > 0, x > 0, np.ones(n, bool), x < nx - 1, y < ny - 1], axis=1)
    cols = (i[:, None] + off[None, :])[mask].astype(np.int32)
    w = np.where(off == 0, 4.0 + shift, -1.0)
    vals = np.broadcast_to(w, (n, 5))[mask].astype(np.float32 if dtype == F32 else np.float64)
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(mask.sum(axis=1), out=rp[1:])
    return rp, cols, vals


# ------------------------------------------------------------ multi-GPU (RCCL)
DIST_UNIQUE_ID_BYTES = 128
DIST_P2P_BLOB_BYTES = 192


def dist_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0 makes it, every rank receives it)."""
    buf = (C.c_ubyte * DIST_UNIQUE_ID_BYTES)()
    _check(lib.lhpc_dist_get_unique_id(buf), "lhpc_dist_get_unique_id")
    return bytes(buf)


class DistComm:
    """One RCCL communicator + communication stream per process and GPU
    (include/lhpc.h lhpc_dist_comm_*; C++: sparse::DistComm)."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int):
        if len(unique_id) != DIST_UNIQUE_ID_BYTES:
            raise ValueError("unique id must be 128 bytes")
        uid = (C.c_ubyte * DIST_UNIQUE_ID_BYTES).from_buffer_copy(unique_id)
        self._h = _p()
        _check(lib.lhpc_dist_comm_create(C.byref(self._h), uid, int(nranks), int(rank), int(device)),
               "lhpc_dist_comm_create")
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)

    @classmethod
    def local(cls, nranks: int, rank: int, device: int):
        """A communicator without RCCL (lhpc_dist_comm_create_local): only the
        direct peer exchange of a registered y window (p2p_setup)."""
        self = cls.__new__(cls)
        self._h = _p()
        _check(lib.lhpc_dist_comm_create_local(C.byref(self._h), int(nranks), int(rank), int(device)),
               "lhpc_dist_comm_create_local")
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)
        return self

    def p2p_export(self, y) -> bytes:
        """This rank's blob (IPC handles) for a new y window (a device tensor;
        up to DIST_P2P_MAX_WINDOWS, exported in the same order on every rank)."""
        blob = (C.c_ubyte * DIST_P2P_BLOB_BYTES)()
        _check(lib.lhpc_dist_p2p_export(self._h, y.data_ptr(), y.numel() * y.element_size(), blob),
               "lhpc_dist_p2p_export")
        self.__dict__.setdefault("_p2p_ys", []).append(y)  # a window must outlive its mapping
        return bytes(blob)

    def p2p_reset(self):
        """Unmap every window (lhpc_dist_p2p_reset).  Collective: every rank
        resets, with a barrier before any rank exports again."""
        _check(lib.lhpc_dist_p2p_reset(self._h), "lhpc_dist_p2p_reset")
        self._p2p_ys = []

    def p2p_unmap(self, y):
        """Undo the last window (lhpc_dist_p2p_unmap), exported or imported."""
        _check(lib.lhpc_dist_p2p_unmap(self._h, y.data_ptr()), "lhpc_dist_p2p_unmap")
        ys = self.__dict__.get("_p2p_ys", [])
        if ys and ys[-1] is y:
            ys.pop()

    def p2p_import(self, blobs):
        """Every rank's blob, in rank order."""
        if len(blobs) != self.nranks:
            raise ValueError("one blob per rank")
        buf = (C.c_ubyte * (DIST_P2P_BLOB_BYTES * self.nranks)).from_buffer_copy(b"".join(blobs))
        _check(lib.lhpc_dist_p2p_import(self._h, buf), "lhpc_dist_p2p_import")

    def p2p_setup_torch(self, y, group=None, _fail_import=False):
        """Export y, all-gather the blobs over an initialised torch.distributed
        group (any backend), import them: lhpc_dist_spmv(…, y) then exchanges
        by direct peer stores.

        Collective-safe: every rank takes part in the same collectives
        whatever fails locally (a rank whose export fails sends a marked empty
        blob).  If any rank's export or import failed, every rank that
        exported undoes this window (lhpc_dist_p2p_unmap) before raising
        LhpcError, so the ranks' window lists stay aligned and no rank keeps a
        window its peers never mapped: a caller that catches the error and
        keeps going gets the RCCL exchange on every rank.  ``_fail_import``
        (tests) makes this rank's import fail after the export."""
        import torch
        import torch.distributed as dist
        err = None
        try:
            blob, ok = self.p2p_export(y), 1
        except LhpcError as e:
            blob, ok, err = bytes(DIST_P2P_BLOB_BYTES), 0, e
        mine = np.frombuffer(blob + bytes([ok]), dtype=np.uint8).copy()
        dev = torch.device("cuda", self.device) if dist.get_backend(group) == "nccl" else torch.device("cpu")
        t = torch.from_numpy(mine).to(dev)
        parts = [torch.empty_like(t) for _ in range(self.nranks)]
        dist.all_gather(parts, t, group=group)
        parts = [p.cpu().numpy() for p in parts]
        exported = ok == 1
        if not all(int(p[-1]) == 1 for p in parts):
            if exported:
                self.p2p_unmap(y)
            raise LhpcError(-6, f"p2p export failed on a rank ({err})")  # LHPC_ERR_INTERNAL
        try:
            if _fail_import:
                raise LhpcError(-6, "injected import failure")
            self.p2p_import([p[:-1].tobytes() for p in parts])
            ok = 1
        except LhpcError as e:
            ok, err = 0, e
        flag = torch.tensor([ok], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if int(flag.item()) != 1:
            self.p2p_unmap(y)  # imported here or not: this rank exported it
            raise LhpcError(-6, f"p2p import failed on a rank ({err})")  # LHPC_ERR_INTERNAL

    def p2p_status(self) -> int:
        return int(lib.lhpc_dist_p2p_status(self._h))

    @classmethod
    def from_torch(cls, device: int, group=None):
        """Rank 0's unique id handed to every rank over an initialised
        torch.distributed group (any backend)."""
        import torch
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = np.frombuffer(dist_unique_id(), dtype=np.uint8).copy() if rank == 0 else \
            np.zeros(DIST_UNIQUE_ID_BYTES, dtype=np.uint8)
        backend = dist.get_backend(group)
        t = torch.from_numpy(uid)
        if backend == "nccl":
            t = t.to(torch.device("cuda", device))
        dist.broadcast(t, 0, group=group)
        return cls(t.cpu().numpy().tobytes(), world, rank, device)

    def allgather_f64(self, t, out, stream=None):
        _check(lib.lhpc_dist_allgather_f64(self._h, t.data_ptr(), t.numel(), out.data_ptr(), _stream_ptr(stream)),
               "lhpc_dist_allgather_f64")
        return out

    def allreduce_sum_f64(self, t, stream=None):
        _check(lib.lhpc_dist_allreduce_sum_f64(self._h, t.data_ptr(), t.numel(), _stream_ptr(stream)),
               "lhpc_dist_allreduce_sum_f64")
        return t

    def stencil7(self, u, out, nzl, ny, nx, ghost=1, c0=-6.0, c1=1.0, stream=None, exchange=DIST_EXCHANGE_AUTO):
        """One 7-point step on this rank's z-slab, halo planes exchanged over
        RCCL, or stored straight into the neighbours' ghost planes when u is a
        registered P2P window (lhpc_dist_stencil7_f32_x; exchange AUTO / RCCL /
        P2P)."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream(u.device)
        _check(lib.lhpc_dist_stencil7_f32_x(self._h, u.data_ptr(), out.data_ptr(), nzl, ny, nx, ghost,
                                            float(c0), float(c1), int(exchange), _stream_ptr(stream)),
               "lhpc_dist_stencil7_f32_x")
        return out

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib.lhpc_dist_comm_destroy(self._h)
            self._h = _p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dist_chain_parts(cuts, world: int, K: int, n_cols: int, tile_width: int) -> np.ndarray:
    """lhpc_dist_chain_parts: for each x tile of ``tile_width`` columns, the
    exchange chunk j after which all its columns have landed (a chained
    call's gather of the tile waits for exactly that exchange)."""
    cuts = np.ascontiguousarray(cuts, dtype=np.int64)
    n_tiles = max(1, -(-int(n_cols) // int(tile_width)))
    out = np.zeros(n_tiles, dtype=np.int32)
    _check(lib.lhpc_dist_chain_parts(cuts.ctypes.data, world, K, n_cols, tile_width, out.ctypes.data, n_tiles),
           "lhpc_dist_chain_parts")
    return out


def interleaved_cuts(row_ptr, world: int, K: int) -> np.ndarray:
    """nnz-balanced row cuts into world·K blocks (block k·world + r = rank r's
    chunk k): lhpc_csr_partition_rows with world·K parts."""
    return csr_partition_rows(row_ptr, world * K)


def interleaved_local_csr(row_ptr, col_idx, val, cuts, world: int, K: int, rank: int):
    """The rank's K blocks stacked in chunk order (row_ptr rebased, global
    columns): the local input of DistSpMVPlan / lhpc_dist_spmv_plan_create."""
    blocks = [(int(cuts[k * world + rank]), int(cuts[k * world + rank + 1])) for k in range(K)]
    n_local = sum(r1 - r0 for r0, r1 in blocks)
    lrp = np.zeros(n_local + 1, dtype=np.int64)
    cols, vals, at, off = [], [], 0, 0
    for r0, r1 in blocks:
        k0, k1 = int(row_ptr[r0]), int(row_ptr[r1])
        lrp[at:at + r1 - r0 + 1] = row_ptr[r0:r1 + 1].astype(np.int64) - k0 + off
        cols.append(col_idx[k0:k1])
        vals.append(val[k0:k1])
        at += r1 - r0
        off += k1 - k0
    if off < 2 ** 31:
        lrp = lrp.astype(np.int32)
    col = np.concatenate(cols) if cols else col_idx[:0]
    v = np.concatenate(vals) if vals else val[:0]
    return lrp, col, v


DIST_P2P_MAX_WINDOWS = 4


def dist_exchange_schedule(cuts, nranks: int, K: int, rank: int, exchange: int = DIST_EXCHANGE_RCCL,
                           broadcast: bool = False):
    """The transfers lhpc_dist_spmv issues on `rank` (include/lhpc.h
    lhpc_dist_exchange_schedule): a list of dicts {chunk, kind, root, group,
    offset, count, send_offset} in issue order."""
    cuts = np.ascontiguousarray(cuts, dtype=np.int64)
    if cuts.shape[0] != nranks * K + 1:
        raise ValueError("cuts must hold nranks*K + 1 rows")
    cap = nranks * K
    buf = (DistXfer * max(cap, 1))()
    n = _i64(0)
    _check(lib.lhpc_dist_exchange_schedule(cuts.ctypes.data, nranks, K, rank, exchange, int(broadcast), buf, cap,
                                           C.byref(n)), "lhpc_dist_exchange_schedule")
    return [{f: getattr(buf[i], f) for f, _ in DistXfer._fields_} for i in range(n.value)]


RCCL_ALLGATHER, RCCL_BROADCAST = 1, 2


def dist_rccl_calls(cuts, nranks: int, K: int, rank: int, dtype: int = F32, broadcast: bool = False):
    """The RCCL calls, argument by argument, that the device paths issue for
    `rank` (include/lhpc.h lhpc_dist_rccl_calls): a list of dicts {chunk, op,
    root, datatype, group_begin, group_end, send_byte_offset,
    recv_byte_offset, count} in issue order."""
    cuts = np.ascontiguousarray(cuts, dtype=np.int64)
    if cuts.shape[0] != nranks * K + 1:
        raise ValueError("cuts must hold nranks*K + 1 rows")
    cap = nranks * K
    buf = (RcclCall * max(cap, 1))()
    n = _i64(0)
    _check(lib.lhpc_dist_rccl_calls(cuts.ctypes.data, nranks, K, rank, int(broadcast), dtype, buf, cap, C.byref(n)),
           "lhpc_dist_rccl_calls")
    return [{f: getattr(buf[i], f) for f, _ in RcclCall._fields_} for i in range(n.value)]


class DistSpMVPlan:
    """y = A·x over ranks with RCCL behind the C ABI (lhpc_dist_spmv_*):
    the rank's K interleaved nnz-balanced blocks, x staged once, chunk k
    reduced then broadcast (in place, exact slices) while chunk k+1 runs.
    ``row_ptr/col_idx/val`` are the rank's LOCAL stacked CSR
    (interleaved_local_csr); ``cuts`` the global world·K+1 cuts."""

    def __init__(self, comm: DistComm, n_rows: int, n_cols: int, K: int, cuts, row_ptr, col_idx, val,
                 flags: int = 0, options=None):
        row_ptr = np.ascontiguousarray(row_ptr)
        col_idx = np.ascontiguousarray(col_idx, dtype=np.int32)
        val = np.ascontiguousarray(val)
        self.cuts = np.ascontiguousarray(cuts, dtype=np.int64)
        if self.cuts.shape[0] != comm.nranks * K + 1:
            raise ValueError("cuts must hold nranks*K + 1 rows")
        self.dtype = F32 if val.dtype == np.float32 else F64
        self.n_rows, self.n_cols, self.K, self.comm = int(n_rows), int(n_cols), int(K), comm
        self._h = _p()
        self._opts = options if not isinstance(options, dict) else Options(**options)
        _check(lib.lhpc_dist_spmv_plan_create_opts(
            C.byref(self._h), comm._h, self.dtype, self.n_rows, self.n_cols, self.K, self.cuts.ctypes.data,
            row_ptr.ctypes.data, 64 if row_ptr.dtype == np.int64 else 32, col_idx.ctypes.data, val.ctypes.data,
            flags, _opts(self._opts)), "lhpc_dist_spmv_plan_create_opts")

    def __call__(self, x, y=None, stream=None):
        """Full y (n_rows) on every rank from the full x (device tensors)."""
        import torch
        if y is None:
            y = torch.empty(self.n_rows, dtype=x.dtype, device=x.device)
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        _check(lib.lhpc_dist_spmv(self._h, x.data_ptr(), y.data_ptr(), _stream_ptr(stream)), "lhpc_dist_spmv")
        return y

    def begin(self, x, y, stream=None):
        """lhpc_dist_spmv_begin: y = A·x with the exchange of y left in
        flight; when x is the y of the previous begin, its gather runs by
        column parts, each waiting only for the exchange that delivers it
        (cross-step overlap).  ``end`` makes ``stream`` wait for the last
        begun exchange."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(x.device)
        _check(lib.lhpc_dist_spmv_begin(self._h, x.data_ptr(), y.data_ptr(), _stream_ptr(stream)),
               "lhpc_dist_spmv_begin")
        return y

    def end(self, stream=None):
        import torch
        if stream is None:
            stream = torch.cuda.current_stream()
        _check(lib.lhpc_dist_spmv_end(self._h, _stream_ptr(stream)), "lhpc_dist_spmv_end")

    def local_info(self) -> dict:
        """lhpc_dist_spmv_plan_info: the rank's local plan (kernel family,
        tiles, chained column parts …)."""
        inf = PlanInfo()
        chain = _i()
        _check(lib.lhpc_dist_spmv_plan_info(self._h, C.byref(inf), C.byref(chain)), "lhpc_dist_spmv_plan_info")
        d = inf.as_dict()
        d["chained_stage"] = bool(chain.value)
        return d

    def cg(self, b, x, p_work, tol: float = 1e-8, max_iter: int = 1000, check_every: int = 1, stream=None):
        """lhpc_dist_cg_solve: b, x (initial guess in, whole solution out on
        every rank) and p_work full-length device tensors; p_work registered
        as a P2P window gives peer-store exchanges.  Returns (x, iterations,
        ‖r‖/‖b‖)."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(b.device)
        it, res = _i(), _d()
        _check(lib.lhpc_dist_cg_solve(self._h, b.data_ptr(), x.data_ptr(), p_work.data_ptr(), float(tol),
                                      int(max_iter), int(check_every), C.byref(it), C.byref(res),
                                      _stream_ptr(stream)), "lhpc_dist_cg_solve")
        return x, it.value, res.value

    def exchange(self, y, stream=None):
        """The call's y exchange alone (every chunk; lhpc_dist_exchange)."""
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(y.device)
        _check(lib.lhpc_dist_exchange(self._h, y.data_ptr(), _stream_ptr(stream)), "lhpc_dist_exchange")
        return y

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib.lhpc_dist_spmv_plan_destroy(self._h)
            self._h = _p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
