// lhpc_stencil.hip — ghost-cell stencils for gfx950 on the reference's
// HPCHighDimensionFlatArray layout (lib/hpc/include/HPCHighDimensionFlatArray.hpp:161-187:
// row-major, stride[D-1] = 1, stride[d] = Π_{e>d}(dim[e] + Low + High),
// offset = Σ stride[d]·(i[d] + Low)).
//
//  blur_x  b(y,x) = Σ_{k=-nb..nb} a(y, x+k)   test_hpc_benchmark.cpp:354-368
//  blur_y  b(y,x) = Σ_{k=-nb..nb} a(y+k, x)   test_hpc_benchmark.cpp:444-457
//  Both sum in ascending k starting from 0.0f, exactly like the reference's
//  scalar loops and its SSE twins (:425-441, :575-601, which add lane-wise in
//  the same order), so the results are bit-identical to them.
//
//  stencil7 out = c0·u + c1·(((((u_{z-1}+u_{z+1})+u_{y-1})+u_{y+1})+u_{x-1})+u_{x+1})
//  (BASELINE config C5; build-defined, same ghost-layout contract) — the two
//  products are rounded separately (__fmul_rn/__fadd_rn: no contraction).
//
// All three are HBM-bound (8 B/cell algorithmic: read once, write once).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "lhpc_common.hpp"

namespace lhpc {
namespace {

constexpr int kBlurThreads = 256;

// ---------------------------------------------------------------- blur x
// One workgroup = one 1024-wide output segment of one row.  The segment plus
// its 2·NB ghost columns is staged in LDS with coalesced loads; each thread
// then forms 4 consecutive outputs from 4+2·NB staged values.
template <int NB, bool VEC>
__global__ __launch_bounds__(kBlurThreads) void k_blur_x(const float *__restrict__ a,
                                                         float *__restrict__ b, int64_t ny,
                                                         int64_t nx, int64_t ghost) {
  constexpr int SEG = 4 * kBlurThreads;
  constexpr int W = SEG + 2 * NB;
  __shared__ __attribute__((aligned(16))) float tile[W + 4];
  const int64_t P = nx + 2 * ghost;  // physical row length of a
  const int64_t nseg = (nx + SEG - 1) / SEG;
  const int64_t y = blockIdx.x / nseg;
  const int64_t x0 = (blockIdx.x % nseg) * SEG;
  // physical column of logical x0 - NB
  const float *src = a + (y + ghost) * P + (x0 + ghost - NB);
  const int64_t avail = nx + 2 * NB - x0;  // staged values that exist in the row window
  const int t = threadIdx.x;
  if constexpr (VEC) {
    for (int i = t; i < W / 4; i += kBlurThreads) {
      if (4 * i + 3 < avail) {
        *reinterpret_cast<f32x4 *>(tile + 4 * i) =
            __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src) + i);
      } else {
        for (int j = 0; j < 4; ++j) tile[4 * i + j] = (4 * i + j < avail) ? src[4 * i + j] : 0.f;
      }
    }
  } else {
    for (int i = t; i < W; i += kBlurThreads) tile[i] = (i < avail) ? src[i] : 0.f;
  }
  __syncthreads();
  float w[4 + 2 * NB];
#pragma unroll
  for (int j = 0; j < (4 + 2 * NB) / 4; ++j) {
    const f32x4 q = *reinterpret_cast<const f32x4 *>(tile + 4 * t + 4 * j);
    w[4 * j] = q[0];
    w[4 * j + 1] = q[1];
    w[4 * j + 2] = q[2];
    w[4 * j + 3] = q[3];
  }
  float o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float res = 0.f;
#pragma unroll
    for (int k = 0; k <= 2 * NB; ++k) res += w[j + k];
    o[j] = res;
  }
  const int64_t x = x0 + 4 * t;
  float *dst = b + y * nx + x;
  if (VEC && x + 3 < nx) {
    const f32x4 q = {o[0], o[1], o[2], o[3]};
    __builtin_nontemporal_store(q, reinterpret_cast<f32x4 *>(dst));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (x + j < nx) dst[j] = o[j];
  }
}

// Generic x blur for any nblur (one thread per output).
__global__ __launch_bounds__(kBlurThreads) void k_blur_x_generic(const float *__restrict__ a,
                                                                 float *__restrict__ b, int64_t ny,
                                                                 int64_t nx, int64_t ghost, int nb) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlurThreads + threadIdx.x;
  if (i >= ny * nx) return;
  const int64_t y = i / nx, x = i % nx;
  const float *row = a + (y + ghost) * (nx + 2 * ghost) + ghost + x;
  float res = 0.f;
  for (int k = -nb; k <= nb; ++k) res += row[k];
  b[i] = res;
}

// ---------------------------------------------------------------- blur y
// Thread = VEC adjacent columns × TY consecutive output rows; the TY + 2·NB
// input rows it needs are loaded once into registers (deep memory-level
// parallelism, no LDS).  Tiles are remapped so that the tiles sharing an XCD
// (blockIdx % 8) walk consecutive y-tiles of one column strip: their 2·NB
// overlapping rows then hit that XCD's L2 instead of HBM.
template <int NB, int VEC, int TY>
__global__ __launch_bounds__(kBlurThreads) void k_blur_y(const float *__restrict__ a,
                                                         float *__restrict__ b, int64_t ny,
                                                         int64_t nx, int64_t ghost,
                                                         int64_t n_strips, int64_t n_ytiles) {
  using V = typename std::conditional<VEC == 4, f32x4, typename std::conditional<VEC == 2, f32x2, float>::type>::type;
  const int64_t nwg = n_strips * n_ytiles;
  // bijective XCD remap (cdna_hip_programming.md §5, "XCD swizzle must be bijective")
  const int64_t orig = blockIdx.x;
  const int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int64_t tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int64_t strip = tile / n_ytiles;
  const int64_t y0 = (tile % n_ytiles) * TY;
  const int64_t x = (strip * kBlurThreads + threadIdx.x) * VEC;
  if (x >= nx) return;
  const int64_t P = nx + 2 * ghost;
  const float *src = a + (y0 + ghost - NB) * P + ghost + x;
  const int64_t rows_in = ny + 2 * NB - y0;  // input rows available from y0-NB
  constexpr int WIN = TY + 2 * NB;
  float w[WIN][VEC];
  const bool full = (x + VEC <= nx);
  if (full && rows_in >= WIN) {
    // interior tile: unconditional loads, so every load stays in flight
#pragma unroll
    for (int i = 0; i < WIN; ++i) {
      const V q = __builtin_nontemporal_load(reinterpret_cast<const V *>(src + i * P));
      if constexpr (VEC == 1) {
        w[i][0] = q;
      } else if constexpr (VEC == 2) {
        w[i][0] = q[0]; w[i][1] = q[1];
      } else {
        w[i][0] = q[0]; w[i][1] = q[1]; w[i][2] = q[2]; w[i][3] = q[3];
      }
    }
  } else {
#pragma unroll
  for (int i = 0; i < WIN; ++i) {
    if (i < rows_in) {
      if (full) {
        const V q = __builtin_nontemporal_load(reinterpret_cast<const V *>(src + i * P));
        if constexpr (VEC == 1) {
          w[i][0] = q;
        } else if constexpr (VEC == 2) {
          w[i][0] = q[0]; w[i][1] = q[1];
        } else {
          w[i][0] = q[0]; w[i][1] = q[1]; w[i][2] = q[2]; w[i][3] = q[3];
        }
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) w[i][j] = (x + j < nx) ? src[i * P + j] : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) w[i][j] = 0.f;
    }
  }
  }
#pragma unroll
  for (int o = 0; o < TY; ++o) {
    if (y0 + o >= ny) break;
    float res[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      res[j] = 0.f;
#pragma unroll
      for (int k = 0; k <= 2 * NB; ++k) res[j] += w[o + k][j];
    }
    float *dst = b + (y0 + o) * nx + x;
    if (full) {
      V q;
      if constexpr (VEC == 1) {
        q = res[0];
      } else if constexpr (VEC == 2) {
        q[0] = res[0]; q[1] = res[1];
      } else {
        q[0] = res[0]; q[1] = res[1]; q[2] = res[2]; q[3] = res[3];
      }
      __builtin_nontemporal_store(q, reinterpret_cast<V *>(dst));
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (x + j < nx) dst[j] = res[j];
    }
  }
}

__global__ __launch_bounds__(kBlurThreads) void k_blur_y_generic(const float *__restrict__ a,
                                                                 float *__restrict__ b, int64_t ny,
                                                                 int64_t nx, int64_t ghost, int nb) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kBlurThreads + threadIdx.x;
  if (i >= ny * nx) return;
  const int64_t y = i / nx, x = i % nx;
  const int64_t P = nx + 2 * ghost;
  const float *col = a + (y + ghost) * P + ghost + x;
  float res = 0.f;
  for (int k = -nb; k <= nb; ++k) res += col[k * P];
  b[i] = res;
}

// ------------------------------------------------------------- stencil7
// Thread = one (y, x) column of a 64×4 tile; it streams ZC consecutive z
// planes keeping u(z-1), u(z), u(z+1) in registers; x±1 / y±1 neighbours are
// read from the L1/L2 lines the neighbouring lanes just fetched.
constexpr int kS7X = 64, kS7Y = 4, kS7Z = 16;

__global__ __launch_bounds__(kS7X *kS7Y) void k_stencil7(const float *__restrict__ u,
                                                         float *__restrict__ out, int64_t nz,
                                                         int64_t ny, int64_t nx, int64_t g,
                                                         float c0, float c1, int64_t z_begin,
                                                         int64_t z_end) {
  const int64_t x = static_cast<int64_t>(blockIdx.x) * kS7X + threadIdx.x;
  const int64_t y = static_cast<int64_t>(blockIdx.y) * kS7Y + threadIdx.y;
  const int64_t zs = z_begin + static_cast<int64_t>(blockIdx.z) * kS7Z;
  if (x >= nx || y >= ny || zs >= z_end) return;
  const int64_t ze = zs + kS7Z < z_end ? zs + kS7Z : z_end;
  const int64_t Px = nx + 2 * g;
  const int64_t Pyx = (ny + 2 * g) * Px;
  const int64_t base = (zs + g) * Pyx + (y + g) * Px + (x + g);
  const float *p = u + base;
  float zm = p[-Pyx];
  float zc = p[0];
  for (int64_t z = zs; z < ze; ++z) {
    const float zp = p[Pyx];
    float s = __fadd_rn(zm, zp);
    s = __fadd_rn(s, p[-Px]);
    s = __fadd_rn(s, p[Px]);
    s = __fadd_rn(s, p[-1]);
    s = __fadd_rn(s, p[1]);
    const float r = __fadd_rn(__fmul_rn(c0, zc), __fmul_rn(c1, s));
    __builtin_nontemporal_store(r, out + (p - u));
    zm = zc;
    zc = zp;
    p += Pyx;
  }
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

struct HostStage {
  // device staging for host-pointer calls; freed on scope exit
  void *d = nullptr;
  ~HostStage() {
    if (d) (void)hipFree(d);
  }
};

int blur_launch(bool ydir, const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                int nb, hipStream_t s) {
  const int64_t cells = ny * nx;
  if (cells == 0) return LHPC_OK;
  const int64_t P = nx + 2 * ghost;
  if (!ydir) {
    if (nb == 8) {
      constexpr int SEG = 4 * kBlurThreads;
      const int64_t grid = ny * ((nx + SEG - 1) / SEG);
      const bool vec = aligned16(a) && aligned16(b) && P % 4 == 0 && nx % 4 == 0 &&
                       (ghost - 8) % 4 == 0;
      if (vec)
        hipLaunchKernelGGL((k_blur_x<8, true>), dim3(static_cast<unsigned>(grid)), dim3(kBlurThreads),
                           0, s, a, b, ny, nx, ghost);
      else
        hipLaunchKernelGGL((k_blur_x<8, false>), dim3(static_cast<unsigned>(grid)), dim3(kBlurThreads),
                           0, s, a, b, ny, nx, ghost);
    } else {
      hipLaunchKernelGGL(k_blur_x_generic, dim3(static_cast<unsigned>((cells + kBlurThreads - 1) / kBlurThreads)),
                         dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, nb);
    }
  } else {
    if (nb == 8) {
      const bool vec4 = aligned16(a) && aligned16(b) && P % 4 == 0 && nx % 4 == 0 && ghost % 4 == 0;
      constexpr int TY = 16;
      const int64_t n_ytiles = (ny + TY - 1) / TY;
      if (vec4) {
        const int64_t n_strips = (nx + 4 * kBlurThreads - 1) / (4 * kBlurThreads);
        hipLaunchKernelGGL((k_blur_y<8, 4, TY>), dim3(static_cast<unsigned>(n_strips * n_ytiles)),
                           dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, n_strips, n_ytiles);
      } else {
        const int64_t n_strips = (nx + kBlurThreads - 1) / kBlurThreads;
        hipLaunchKernelGGL((k_blur_y<8, 1, TY>), dim3(static_cast<unsigned>(n_strips * n_ytiles)),
                           dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, n_strips, n_ytiles);
      }
    } else {
      hipLaunchKernelGGL(k_blur_y_generic, dim3(static_cast<unsigned>((cells + kBlurThreads - 1) / kBlurThreads)),
                         dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, nb);
    }
  }
  return check_launch(s);
}

int blur_entry(bool ydir, const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
               int nblur, int on_device, void *stream) {
  if (!a || !b || ny < 0 || nx < 0 || nblur < 0 || ghost < nblur) return LHPC_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (on_device) return blur_launch(ydir, a, b, ny, nx, ghost, nblur, s);
  const size_t in_bytes = static_cast<size_t>((ny + 2 * ghost) * (nx + 2 * ghost)) * 4;
  const size_t out_bytes = static_cast<size_t>(ny * nx) * 4;
  HostStage da, db;
  LHPC_HIP_TRY(hipMalloc(&da.d, in_bytes ? in_bytes : 16));
  LHPC_HIP_TRY(hipMalloc(&db.d, out_bytes ? out_bytes : 16));
  LHPC_HIP_TRY(hipMemcpyAsync(da.d, a, in_bytes, hipMemcpyHostToDevice, s));
  LHPC_TRY(blur_launch(ydir, static_cast<float *>(da.d), static_cast<float *>(db.d), ny, nx, ghost,
                       nblur, s));
  LHPC_HIP_TRY(hipMemcpyAsync(b, db.d, out_bytes, hipMemcpyDeviceToHost, s));
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  return LHPC_OK;
}

int s7_launch(const float *u, float *out, int64_t nz, int64_t ny, int64_t nx, int64_t g, float c0,
              float c1, int64_t zb, int64_t ze, hipStream_t s) {
  if (zb >= ze || ny == 0 || nx == 0) return LHPC_OK;
  dim3 grid(static_cast<unsigned>((nx + kS7X - 1) / kS7X), static_cast<unsigned>((ny + kS7Y - 1) / kS7Y),
            static_cast<unsigned>((ze - zb + kS7Z - 1) / kS7Z));
  hipLaunchKernelGGL(k_stencil7, grid, dim3(kS7X, kS7Y), 0, s, u, out, nz, ny, nx, g, c0, c1, zb, ze);
  return check_launch(s);
}

}  // namespace
}  // namespace lhpc

using namespace lhpc;

extern "C" int lhpc_blur_x_f32(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                               int nblur, int on_device, void *stream) {
  return blur_entry(false, a, b, ny, nx, ghost, nblur, on_device, stream);
}

extern "C" int lhpc_blur_y_f32(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                               int nblur, int on_device, void *stream) {
  return blur_entry(true, a, b, ny, nx, ghost, nblur, on_device, stream);
}

extern "C" int lhpc_stencil7_f32_planes(const float *u, float *out, int64_t nz, int64_t ny,
                                        int64_t nx, int64_t ghost, float c0, float c1,
                                        int64_t z_begin, int64_t z_end, void *stream) {
  if (!u || !out || nz < 0 || ny < 0 || nx < 0 || ghost < 1 || z_begin < 0 || z_end > nz)
    return LHPC_ERR_INVALID_ARG;
  return s7_launch(u, out, nz, ny, nx, ghost, c0, c1, z_begin, z_end, static_cast<hipStream_t>(stream));
}

extern "C" int lhpc_stencil7_f32(const float *u, float *out, int64_t nz, int64_t ny, int64_t nx,
                                 int64_t ghost, float c0, float c1, int on_device, void *stream) {
  if (!u || !out || nz < 0 || ny < 0 || nx < 0 || ghost < 1) return LHPC_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (on_device) return s7_launch(u, out, nz, ny, nx, ghost, c0, c1, 0, nz, s);
  const size_t bytes =
      static_cast<size_t>((nz + 2 * ghost) * (ny + 2 * ghost) * (nx + 2 * ghost)) * 4;
  HostStage du, dout;
  LHPC_HIP_TRY(hipMalloc(&du.d, bytes));
  LHPC_HIP_TRY(hipMalloc(&dout.d, bytes));
  LHPC_HIP_TRY(hipMemcpyAsync(du.d, u, bytes, hipMemcpyHostToDevice, s));
  // ghost cells of `out` keep the caller's values
  LHPC_HIP_TRY(hipMemcpyAsync(dout.d, out, bytes, hipMemcpyHostToDevice, s));
  LHPC_TRY(s7_launch(static_cast<float *>(du.d), static_cast<float *>(dout.d), nz, ny, nx, ghost, c0,
                     c1, 0, nz, s));
  LHPC_HIP_TRY(hipMemcpyAsync(out, dout.d, bytes, hipMemcpyDeviceToHost, s));
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  return LHPC_OK;
}
