// ref_sort.cpp — TEST INFRASTRUCTURE ONLY.  C entry points over the
// REFERENCE's own CPU radix sort, compiled from its sources where they lie
// (lib/sort/radix_cpu/include/radix_sort_cpu.hpp + src/helper.cpp) by
// oracle/Makefile into oracle/_ref/libref_sort.so.  Used by tests/ to pin the
// GPU sort and the C restatement, and by bench.py's cpu_baseline leg
// (kind "reference") for the sort workload.  Never linked into the product.
#include <radix_sort_cpu.hpp>

#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

extern "C" {
// sort::radix::radix_sort(std::vector<uint32_t>&) → radix_sort_cache_thread_v2<256>
// (radix_sort_cpu.hpp:326-331, :268-323), called on the caller's buffer.
void ref_radix_sort_u32(uint32_t *a, size_t n) { sort::radix::details::radix_sort_cache_thread_v2<256>(a, n); }

// single-threaded LSD (radix_sort_cpu.hpp:125-166)
void ref_radix_sort_v4_u32(uint32_t *a, size_t n) { sort::radix::details::radix_sort_v4<256>(a, n); }

// the CPU tests' input generator (lib/sort/radix_cpu/src/helper.cpp:21-28)
void ref_generate_random(uint32_t *out, size_t n) {
  std::vector<uint32_t> v;
  sort::radix::details::helper::generate_random(v, n);
  std::memcpy(out, v.data(), n * sizeof(uint32_t));
}

// the GPU test's input generator, restated (lib/gpu/radix_gpu/src/radix_sort_gpu.cpp:11-20 is a
// CUDA translation unit): default-seeded std::mt19937, uniform_int_distribution<uint32_t>(100, max-100)
void ref_gpu_test_keys(uint32_t *out, size_t n) {
  std::mt19937 rng{};
  std::uniform_int_distribution<uint32_t> uni(100, UINT32_MAX - 100);
  for (size_t i = 0; i < n; ++i) out[i] = uni(rng);
}
}
