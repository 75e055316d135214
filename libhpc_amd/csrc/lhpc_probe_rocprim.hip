// lhpc_probe_rocprim.hip — MEASUREMENT PROBE ONLY (not part of the ABI or the
// product): rocPRIM's device radix sort, timed beside lhpc_radix_sort_* so
// DESIGN.md can place the hand-written sort against a tuned library sort.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdint>

extern "C" int lhpc_probe_rocprim_sort_u32(const uint32_t *in, uint32_t *out, int64_t n, void *tmp,
                                           size_t *tmp_bytes, void *stream) {
  return static_cast<int>(rocprim::radix_sort_keys(tmp, *tmp_bytes, in, out, static_cast<size_t>(n), 0, 32,
                                                   static_cast<hipStream_t>(stream)));
}

extern "C" int lhpc_probe_rocprim_sort_pairs_u64(const uint64_t *kin, uint64_t *kout, const uint32_t *vin,
                                                 uint32_t *vout, int64_t n, int end_bit, void *tmp,
                                                 size_t *tmp_bytes, void *stream) {
  return static_cast<int>(rocprim::radix_sort_pairs(tmp, *tmp_bytes, kin, kout, vin, vout, static_cast<size_t>(n), 0,
                                                    end_bit, static_cast<hipStream_t>(stream)));
}
