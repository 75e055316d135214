// mall_probe.hip — does a scratch buffer written by one kernel and read back
// by the next stay in the 256 MiB Infinity Cache (MALL)?  Measures, for
// scratch sizes B, the write kernel and the read-back kernel separately, with
// the scratch reused in place (ring of one) against a scratch that walks a
// 4 GiB buffer (every write lands on cold lines), plain vs non-temporal
// stores/loads, and with an HBM side stream read beside both kernels (the
// SpMV's col16/val streams).  Standalone: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

// write n16 16-B vectors; optionally read a side stream of s16 vectors too
template <bool NT>
__global__ __launch_bounds__(256) void k_write(f32x4 *__restrict__ d, int64_t n16, const f32x4 *__restrict__ side,
                                               int64_t s16, float *__restrict__ sink, float v) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  float acc = 0.f;
  for (int64_t i = t; i < s16; i += stride) {
    const f32x4 a = __builtin_nontemporal_load(side + i);
    acc += a[0] + a[1] + a[2] + a[3];
  }
  for (int64_t i = t; i < n16; i += stride) {
    const f32x4 a = f32x4{v, v + 1.f, v + 2.f, static_cast<float>(i)};
    if constexpr (NT) __builtin_nontemporal_store(a, d + i);
    else d[i] = a;
  }
  if (acc == 12345.678f) sink[0] = acc;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_read(const f32x4 *__restrict__ s, int64_t n16, const f32x4 *__restrict__ side,
                                              int64_t s16, float *__restrict__ sink) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  float acc = 0.f;
  for (int64_t i = t; i < s16; i += stride) {
    const f32x4 a = __builtin_nontemporal_load(side + i);
    acc += a[0] + a[1] + a[2] + a[3];
  }
  for (int64_t i = t; i < n16; i += stride) {
    const f32x4 a = NT ? __builtin_nontemporal_load(s + i) : s[i];
    acc += a[0] + a[1] + a[2] + a[3];
  }
  if (acc == 12345.678f) sink[0] = acc;
}

int main(int argc, char **argv) {
  const int64_t big = 4LL << 30;  // bytes: the walking scratch
  const int64_t side_big = 4LL << 30;
  f32x4 *buf, *side;
  float *sink;
  CK(hipMalloc(&buf, big));
  CK(hipMalloc(&side, side_big));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 0, big));
  CK(hipMemset(side, 0, side_big));
  hipEvent_t ev[4];
  for (auto &e : ev) CK(hipEventCreate(&e));
  const int grid = 256 * 8;
  const int reps = 12;
  std::vector<int> mbs = {16, 32, 64, 96, 128, 160, 192, 256, 384, 1024};
  for (int side_ratio : {0, 1}) {       // side stream bytes = side_ratio * B (both kernels)
    for (int nt : {0, 1}) {             // store/load policy of the scratch
      for (int ring : {1, 0}) {         // 1: scratch reused in place; 0: walks the 4 GiB buffer
        for (int mb : mbs) {
          const int64_t B = static_cast<int64_t>(mb) << 20, n16 = B / 16;
          const int64_t s16 = side_ratio * n16;
          std::vector<float> tw, tr;
          int64_t off = 0, soff = 0;
          for (int r = 0; r < reps; ++r) {
            f32x4 *d = buf + off / 16;
            const f32x4 *sd0 = side + soff / 16;
            soff = (soff + s16 * 16) % (side_big - 2 * s16 * 16 - 16);
            const f32x4 *sd1 = side + soff / 16;
            soff = (soff + s16 * 16) % (side_big - 2 * s16 * 16 - 16);
            CK(hipEventRecord(ev[0], 0));
            if (nt) hipLaunchKernelGGL(k_write<true>, dim3(grid), dim3(256), 0, 0, d, n16, sd0, s16, sink, 1.f * r);
            else hipLaunchKernelGGL(k_write<false>, dim3(grid), dim3(256), 0, 0, d, n16, sd0, s16, sink, 1.f * r);
            CK(hipEventRecord(ev[1], 0));
            if (nt) hipLaunchKernelGGL(k_read<true>, dim3(grid), dim3(256), 0, 0, d, n16, sd1, s16, sink);
            else hipLaunchKernelGGL(k_read<false>, dim3(grid), dim3(256), 0, 0, d, n16, sd1, s16, sink);
            CK(hipEventRecord(ev[2], 0));
            CK(hipEventSynchronize(ev[2]));
            float a, b;
            CK(hipEventElapsedTime(&a, ev[0], ev[1]));
            CK(hipEventElapsedTime(&b, ev[1], ev[2]));
            if (r >= 2) {
              tw.push_back(a);
              tr.push_back(b);
            }
            if (!ring) off = (off + B) % (big - B);
          }
          std::sort(tw.begin(), tw.end());
          std::sort(tr.begin(), tr.end());
          const double w = tw[tw.size() / 2] * 1e-3, rd = tr[tr.size() / 2] * 1e-3;
          const double bytes_w = static_cast<double>(B + s16 * 16), bytes_r = static_cast<double>(B + s16 * 16);
          std::printf(
              "{\"side_ratio\": %d, \"nt\": %d, \"ring\": %d, \"MB\": %d, \"write_us\": %.1f, \"read_us\": %.1f, "
              "\"write_TBs\": %.2f, \"read_TBs\": %.2f, \"pair_TBs\": %.2f}\n",
              side_ratio, nt, ring, mb, w * 1e6, rd * 1e6, bytes_w / w / 1e12, bytes_r / rd / 1e12,
              (bytes_w + bytes_r) / (w + rd) / 1e12);
          std::fflush(stdout);
        }
      }
    }
  }
  return 0;
}
