// race_diag.hip — one-shot diagnostic for the round-2 host-path race (commit
// 67202ac: the 4-entry Matrix Market COO->CSR read its rows as 0 in 4 of 25
// runs).  It replays the old host-buffer path's sequence of operations, in one
// process, many times, under variants that each change one ingredient:
//
//   pool_pageable_null   the old path: hipMallocAsync staging on the NULL
//                        stream, pageable hipMemcpyAsync H2D, two 8-B pool
//                        scratch words zeroed by hipMemsetAsync (the old
//                        `flag` / `grand`), a kernel reading the staged rows,
//                        pageable D2H, sync, then hipFreeAsync of everything
//                        (the old DevBuf destructors ran after the sync)
//   pool_pinned_null     the same with pinned host buffers
//   malloc_pageable_null hipMalloc / hipFree staging (what the fix uses),
//                        asynchronous pageable copies kept
//   pool_pageable_stream the old path on a created (blocking) stream
//   *_pending            each iteration first zero-fills a 1 MB pool block
//                        with a kernel and frees it (stream-ordered, no
//                        sync), so the staging allocations may reuse memory
//                        an unfinished kernel still writes — what a copy that
//                        is not ordered behind that kernel would expose
//
// Per iteration the kernel writes out[i] = 2·in[i] + 1 for a fresh pattern;
// a mismatch is counted with its kind (input read as 0 / stale value /
// other), and every allocation is checked against the live ones for overlap.
// Prints one JSON line per variant.  Not part of the ABI; run once
// (tools/gpu_race_diag.sh), never in a loop of processes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("{\"error\": \"%s at line %d\"}\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ void k_zero(int32_t *p, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    p[i] = 0;
}

__global__ void k_consume(const int32_t *rows, const int32_t *cols, const uint32_t *flag, int32_t *out, int n) {
  const int i = threadIdx.x;
  if (i < n) out[i] = 2 * rows[i] + 1 + (cols[i] - cols[i]) + static_cast<int32_t>(flag[0] & 0u);
}

struct Alloc {
  void *p;
  size_t n;
};

static bool overlaps(const std::vector<Alloc> &live, void *p, size_t n) {
  const auto a = reinterpret_cast<uintptr_t>(p);
  for (const Alloc &q : live) {
    const auto b = reinterpret_cast<uintptr_t>(q.p);
    if (a < b + q.n && b < a + n) return true;
  }
  return false;
}

static int run(const char *name, bool pool, bool pinned, bool null_stream, int iters, bool pending = false) {
  hipStream_t s = nullptr;
  if (!null_stream) CK(hipStreamCreate(&s));
  const int n = 4;
  int32_t *h_rows, *h_cols, *h_out;
  std::vector<int32_t> pr(n), pc(n), po(n);
  if (pinned) {
    CK(hipHostMalloc(reinterpret_cast<void **>(&h_rows), n * 4));
    CK(hipHostMalloc(reinterpret_cast<void **>(&h_cols), n * 4));
    CK(hipHostMalloc(reinterpret_cast<void **>(&h_out), n * 4));
  } else {
    h_rows = pr.data();
    h_cols = pc.data();
    h_out = po.data();
  }
  long zero_reads = 0, stale = 0, other = 0, aliased = 0;
  int32_t prev_first = -1;
  for (int it = 0; it < iters; ++it) {
    for (int i = 0; i < n; ++i) {
      h_rows[i] = 1000 + (it * 7 + i) % 997;  // never 0
      h_cols[i] = i;
      h_out[i] = -1;
    }
    if (pending) {  // a pool block still being zero-filled when it is freed
      void *big = nullptr;
      const int64_t nb = 1 << 18;
      if (pool) CK(hipMallocAsync(&big, nb * 4, s));
      else CK(hipMalloc(&big, nb * 4));
      hipLaunchKernelGGL(k_zero, dim3(64), dim3(256), 0, s, static_cast<int32_t *>(big), nb);
      CK(hipGetLastError());
      if (pool) CK(hipFreeAsync(big, s));
      else CK(hipFree(big));
    }
    std::vector<Alloc> live;
    void *d[6] = {};
    const size_t sz[6] = {16, 16, 32, 32, 16, 32};  // rows, cols, vals, row_ptr, col_out, val_out (nnz = 4)
    for (int k = 0; k < 6; ++k) {
      if (pool) CK(hipMallocAsync(&d[k], sz[k], s));
      else CK(hipMalloc(&d[k], sz[k]));
      if (overlaps(live, d[k], sz[k])) ++aliased;
      live.push_back({d[k], sz[k]});
    }
    CK(hipMemcpyAsync(d[0], h_rows, n * 4, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(d[1], h_cols, n * 4, hipMemcpyHostToDevice, s));
    void *flag = nullptr, *grand = nullptr;  // the old coo_to_csr_dev scratch words
    if (pool) {
      CK(hipMallocAsync(&flag, 8, s));
      CK(hipMallocAsync(&grand, 8, s));
    } else {
      CK(hipMalloc(&flag, 8));
      CK(hipMalloc(&grand, 8));
    }
    if (overlaps(live, flag, 8)) ++aliased;
    live.push_back({flag, 8});
    if (overlaps(live, grand, 8)) ++aliased;
    live.push_back({grand, 8});
    CK(hipMemsetAsync(flag, 0, 8, s));
    CK(hipMemsetAsync(grand, 0, 8, s));
    hipLaunchKernelGGL(k_consume, dim3(1), dim3(64), 0, s, static_cast<int32_t *>(d[0]),
                       static_cast<int32_t *>(d[1]), static_cast<uint32_t *>(flag), static_cast<int32_t *>(d[4]), n);
    CK(hipGetLastError());
    CK(hipMemcpyAsync(h_out, d[4], n * 4, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < n; ++i) {
      const int32_t want = 2 * h_rows[i] + 1;
      if (h_out[i] == want) continue;
      if (h_out[i] == 1) ++zero_reads;  // rows[i] read as 0
      else if (i == 0 && h_out[i] == 2 * prev_first + 1) ++stale;
      else ++other;
    }
    prev_first = h_rows[0];
    // the old DevBuf destructors: stream-ordered frees after the sync
    for (int k = 0; k < 6; ++k) {
      if (pool) CK(hipFreeAsync(d[k], s));
      else CK(hipFree(d[k]));
    }
    if (pool) {
      CK(hipFreeAsync(flag, s));
      CK(hipFreeAsync(grand, s));
    } else {
      CK(hipFree(flag));
      CK(hipFree(grand));
    }
  }
  CK(hipStreamSynchronize(s));
  std::printf("{\"variant\": \"%s\", \"iters\": %d, \"zero_reads\": %ld, \"stale\": %ld, \"other\": %ld, "
              "\"aliased_allocs\": %ld}\n",
              name, iters, zero_reads, stale, other, aliased);
  std::fflush(stdout);
  if (pinned) {
    (void)hipHostFree(h_rows);
    (void)hipHostFree(h_cols);
    (void)hipHostFree(h_out);
  }
  if (s) (void)hipStreamDestroy(s);
  return 0;
}

int main(int argc, char **argv) {
  const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
  int rc = 0;
  rc |= run("pool_pageable_null", true, false, true, iters);
  rc |= run("pool_pinned_null", true, true, true, iters);
  rc |= run("malloc_pageable_null", false, false, true, iters);
  rc |= run("pool_pageable_stream", true, false, false, iters);
  rc |= run("pool_pageable_null_pending", true, false, true, iters, true);
  rc |= run("pool_pinned_null_pending", true, true, true, iters, true);
  rc |= run("malloc_pageable_null_pending", false, false, true, iters, true);
  return rc;
}
