// lhpc_runtime.hip — status strings and device discovery for the C ABI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>

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
    default:
      if (status >= LHPC_RCCL_STATUS_BASE)
        return ncclGetErrorString(static_cast<ncclResult_t>(status - LHPC_RCCL_STATUS_BASE));
      if (status > 0) return hipGetErrorString(static_cast<hipError_t>(status));
      return "lhpc: unknown status";
  }
}

extern "C" int lhpc_abi_version(void) { return LHPC_ABI_VERSION; }

extern "C" int lhpc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int good = 0;
  for (int d = 0; d < n; ++d) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess && std::strncmp(p.gcnArchName, "gfx950", 6) == 0)
      ++good;
  }
  return good;
}
