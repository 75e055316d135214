// lhpc_runtime.hip — status strings, build tag and device discovery for the C ABI.

// Build tag (lhpc_build_flags), read before any header sets a default, so
// only command-line -D flags count: timing-only probes that skip work and
// compute wrong results, and A/B variants of the product kernels.
#if defined(LHPC_XT_PROBE_GVAL) || defined(LHPC_XT_PROBE_NOVAL) || defined(LHPC_XT_PROBE_VI) || \
    defined(LHPC_XT_PROBE_XG) || defined(LHPC_XT_PROBE_GROUPED) || defined(LHPC_SORT_PROBE)
#define LHPC_TAG_PROBE 1
#endif
#if defined(LHPC_XT_RBLK32) || defined(LHPC_XT_RBLK64) || defined(LHPC_XT_IP_WAVES) || defined(LHPC_XT_LDS_TOTAL) || \
    defined(LHPC_XT_XG_CPOL) || defined(LHPC_XT_SEGHI) || defined(LHPC_XT_STAMPS) ||   \
    defined(LHPC_SELL_NO_SHFL) || defined(LHPC_SCRATCH_DEFAULT_POOL) || defined(LHPC_SORT_KEYS_VARIANT) || \
    defined(LHPC_SORT_P32_VARIANT) || defined(LHPC_SORT_P64_VARIANT) || defined(LHPC_SORT_WPE) || \
    defined(LHPC_SORT_UP_Q) || defined(LHPC_SORT_SCAN_TRAIL) || defined(LHPC_AB_BUILD)
#define LHPC_TAG_AB 1
#endif
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "lhpc_common.hpp"

extern "C" const char *lhpc_strerror(int status) {
  switch (status) {
    case LHPC_OK: return "success";
    case LHPC_ERR_INVALID_ARG: return "lhpc: invalid argument";
    case LHPC_ERR_BAD_CSR: return "lhpc: malformed CSR (row_ptr/col_idx)";
    case LHPC_ERR_ALLOC: return "lhpc: allocation failed";
    case LHPC_ERR_NO_DEVICE: return "lhpc: no gfx950 (MI355X) device";
    case LHPC_ERR_UNSUPPORTED: return "lhpc: unsupported configuration";
    case LHPC_ERR_INTERNAL: return "lhpc: internal error";
    case LHPC_ERR_BUSY: return "lhpc: plan work in use by another call (one CG solve per plan at a time)";
    default:
      if (status >= LHPC_RCCL_STATUS_BASE)
        return ncclGetErrorString(static_cast<ncclResult_t>(status - LHPC_RCCL_STATUS_BASE));
      if (status > 0) return hipGetErrorString(static_cast<hipError_t>(status));
      return "lhpc: unknown status";
  }
}

extern "C" int lhpc_abi_version(void) {
  try { return LHPC_ABI_VERSION;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_build_flags(void) {
  int f = 0;
#ifdef LHPC_TUNING_ENV
  f |= LHPC_BUILD_TUNING;
#endif
#if defined(LHPC_DEBUG_BOUNDS) || defined(LHPC_DEBUG_SYNC)
  f |= LHPC_BUILD_DEBUG;
#endif
#ifdef LHPC_TAG_PROBE
  f |= LHPC_BUILD_PROBE;
#endif
#ifdef LHPC_TAG_AB
  f |= LHPC_BUILD_AB;
#endif
  return f;
}

extern "C" int lhpc_device_count(void) {
  try {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int good = 0;
    for (int d = 0; d < n; ++d) {
      hipDeviceProp_t p;
      if (hipGetDeviceProperties(&p, d) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0)
        ++good;
    }
    return good;
  } LHPC_ABI_CATCH
}

extern "C" void lhpc_options_init(lhpc_options *o) {
  if (!o) return;
  std::memset(o, 0, sizeof(*o));
  o->struct_size = sizeof(*o);
}

namespace lhpc {
namespace {
#ifdef LHPC_TUNING_ENV
// tuning build only: LHPC_* variables over the caller's options (the names
// the A/B scripts of tools/ and DESIGN.md §4 use)
void env_overlay(lhpc_options &o) {
  auto i32 = [](const char *n, int32_t &f) {
    if (const char *e = tuning_env(n)) f = std::atoi(e);
  };
  auto i64 = [](const char *n, int64_t &f) {
    if (const char *e = tuning_env(n)) f = std::atoll(e);
  };
  if (const char *e = tuning_env("LHPC_SPMV_XTILE")) o.spmv_no_xtile = std::atoi(e) == 0;
  if (const char *e = tuning_env("LHPC_SPMV_LOCALITY")) o.spmv_locality = std::atof(e);
  if (const char *e = tuning_env("LHPC_SPMV_ROWGROUP")) std::sscanf(e, "%d,%d", &o.rowgroup_lanes, &o.rowgroup_rows);
  if (const char *e = tuning_env("LHPC_XTILE_IPERM"))
    o.xtile_reduce = std::atoi(e) ? LHPC_XTILE_REDUCE_IPERM : LHPC_XTILE_REDUCE_PERM;
  if (const char *e = tuning_env("LHPC_XTILE_MALL")) o.xtile_ranges = std::max(1, std::atoi(e));
  i32("LHPC_XTILE_RING", o.xtile_ring);
  i32("LHPC_XTILE_PRETABLE", o.xtile_pretable);
  i32("LHPC_XTILE_U", o.xtile_steps);
  if (const char *e = tuning_env("LHPC_XTILE_NTSTORE")) o.xtile_store = std::atoi(e) ? LHPC_STORE_NT : LHPC_STORE_PLAIN;
  i32("LHPC_XTILE_CUT", o.xtile_cut);
  i32("LHPC_XTILE_ALIGN", o.xtile_align);
  i64("LHPC_XTILE_PIECE", o.xtile_piece);
  i64("LHPC_XTILE_MALL_PIECE", o.xtile_range_piece);
  i32("LHPC_XSLICE_S", o.xslice_slices);
  if (const char *e = tuning_env("LHPC_XSLICE_PARTIAL")) o.xslice_partial = std::strcmp(e, "f64") ? 1 : 2;
  i32("LHPC_XSLICE_NB", o.xslice_window);
  if (const char *e = tuning_env("LHPC_XSLICE_MB")) o.xslice_mb = std::atof(e);
  if (const char *e = tuning_env("LHPC_STENCIL7_IMPL"))
    o.stencil7_impl = !std::strcmp(e, "buf4lds") ? LHPC_S7_RING_X4_LDS : !std::strcmp(e, "buf4") ? LHPC_S7_RING_X4
                      : !std::strcmp(e, "buf") ? LHPC_S7_RING : LHPC_S7_SIMPLE;
  if (const char *e = tuning_env("LHPC_STENCIL7_STORE"))
    o.stencil7_store = !std::strcmp(e, "plain") ? LHPC_STORE_PLAIN : !std::strcmp(e, "staged") ? LHPC_STORE_STAGED : LHPC_STORE_NT;
  if (const char *e = tuning_env("LHPC_STENCIL7_BUF"))
    std::sscanf(e, "%d,%d,%d,%d", &o.stencil7_ry, &o.stencil7_nj, &o.stencil7_zc, &o.stencil7_pf);
  i32("LHPC_STENCIL7_BLOCKS", o.stencil7_blocks);
  i32("LHPC_BLUR_X_RW", o.blur_x_rows);
  if (const char *e = tuning_env("LHPC_BLUR_Y_CFG")) std::sscanf(e, "%d,%d", &o.blur_y_vec, &o.blur_y_rows);
  if (const char *e = tuning_env("LHPC_DIST_P2P")) o.dist_exchange = std::atoi(e) ? LHPC_DIST_EXCHANGE_P2P : LHPC_DIST_EXCHANGE_RCCL;
  i32("LHPC_DIST_BCAST", o.dist_broadcast);
  i32("LHPC_DIST_EXCHANGE", o.dist_world1);
}
#endif

// library-owned stream-ordered scratch pools, one per device (see
// lhpc_common.hpp scratch_alloc); created once under a per-device once_flag
constexpr int kMaxDevices = 64;
std::once_flag g_pool_once[kMaxDevices];
hipMemPool_t g_pool[kMaxDevices] = {};
hipError_t g_pool_err[kMaxDevices] = {};

hipError_t scratch_pool(int dev, hipMemPool_t *out) {
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::call_once(g_pool_once[dev], [dev] {
#ifdef LHPC_SCRATCH_DEFAULT_POOL  // A/B build: the device's default pool
    hipError_t e = hipDeviceGetDefaultMemPool(&g_pool[dev], dev);
    if (e == hipSuccess) {
      uint64_t thr = UINT64_MAX;
      e = hipMemPoolSetAttribute(g_pool[dev], hipMemPoolAttrReleaseThreshold, &thr);
    }
    g_pool_err[dev] = e;
    return;
#endif
    hipMemPoolProps props{};
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = dev;
    hipError_t e = hipMemPoolCreate(&g_pool[dev], &props);
    if (e == hipSuccess) {
      uint64_t thr = UINT64_MAX;  // keep freed scratch for the next call
      e = hipMemPoolSetAttribute(g_pool[dev], hipMemPoolAttrReleaseThreshold, &thr);
    }
    g_pool_err[dev] = e;
  });
  *out = g_pool[dev];
  return g_pool_err[dev];
}
}  // namespace

// The pool of the stream's device (a caller whose current device differs
// from its stream's still gets scratch where the stream runs); the current
// device only for the null stream.
hipError_t scratch_alloc(void **p, size_t bytes, hipStream_t s) {
  int dev = 0;
  hipError_t e;
  if (s) {
    hipDevice_t sd = 0;
    e = hipStreamGetDevice(s, &sd);
    dev = static_cast<int>(sd);
  } else {
    e = hipGetDevice(&dev);
  }
  if (e != hipSuccess) return e;
  hipMemPool_t pool;
  if ((e = scratch_pool(dev, &pool)) != hipSuccess) return e;
  return hipMallocFromPoolAsync(p, bytes ? bytes : 16, pool, s);
}

lhpc_options resolve_options(const lhpc_options *in) {
  lhpc_options o;
  lhpc_options_init(&o);
  if (in && in->struct_size >= sizeof(uint32_t)) {
    const size_t n = in->struct_size < sizeof(o) ? in->struct_size : sizeof(o);
    std::memcpy(&o, in, n);
    o.struct_size = sizeof(o);
  }
#ifdef LHPC_TUNING_ENV
  env_overlay(o);
#endif
  return o;
}

}  // namespace lhpc

// Hands the current device's cached scratch back to the driver (the pool
// keeps freed scratch between calls: GBs after a 500M-key sort).
extern "C" int lhpc_scratch_trim(int device) {
  try {
    hipMemPool_t pool;
    LHPC_HIP_TRY(lhpc::scratch_pool(device, &pool));
    LHPC_HIP_TRY(hipDeviceSynchronize());
    LHPC_HIP_TRY(hipMemPoolTrimTo(pool, 0));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

// Test support: leave `bytes` of the current device's scratch pool filled
// with `value`, so the next scratch allocations on `stream` come back dirty
// (tests/test_gpu_sort.py::test_coo_to_csr_poisoned_pool).
extern "C" int lhpc_scratch_poison(int64_t bytes, int value, void *stream) {
  try {
    if (bytes < 0) return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    void *p = nullptr;
    LHPC_HIP_TRY(lhpc::scratch_alloc(&p, static_cast<size_t>(bytes), s));
    LHPC_HIP_TRY(hipMemsetAsync(p, value, static_cast<size_t>(bytes), s));
    LHPC_HIP_TRY(hipFreeAsync(p, s));
    LHPC_HIP_TRY(hipStreamSynchronize(s));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
