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

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "lhpc_common.hpp"

namespace lhpc {
namespace {

constexpr int kBlurThreads = 256;

// Bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): the blocks the dispatcher deals to one XCD (orig % 8) get a
// contiguous range of logical tiles, in dispatch order — neighbouring tiles
// then share that XCD's L2 (halo rows, 128-B lines straddling a tile edge).
__device__ __forceinline__ int64_t xcd_tile(int64_t orig, int64_t nwg) {
  const int64_t q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// ---------------------------------------------------------------- blur x
// One workgroup = ROWS rows × one 1024-wide output segment.  Each row's
// segment plus its 2·NB ghost columns is staged in LDS with coalesced loads
// (ROWS loads in flight per thread); each thread then forms 4 consecutive
// outputs per row from 4+2·NB staged values.
template <int NB, bool VEC, int ROWS>
__global__ __launch_bounds__(kBlurThreads) void k_blur_x(const float *__restrict__ a,
                                                         float *__restrict__ b, int64_t ny,
                                                         int64_t nx, int64_t ghost) {
  constexpr int SEG = 4 * kBlurThreads;
  constexpr int W = SEG + 2 * NB;
  constexpr int WP = W + 4;
  __shared__ __attribute__((aligned(16))) float tile[ROWS][WP];
  const int64_t P = nx + 2 * ghost;  // physical row length of a
  const int64_t nseg = (nx + SEG - 1) / SEG;
  const int64_t y0 = (blockIdx.x / nseg) * ROWS;
  const int64_t x0 = (blockIdx.x % nseg) * SEG;
  const int64_t avail = nx + 2 * NB - x0;  // staged values that exist in the row window
  const int t = threadIdx.x;
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    const int64_t yy = y0 + r < ny ? y0 + r : ny - 1;  // clamp (rows past ny are not stored)
    const float *src = a + (yy + ghost) * P + (x0 + ghost - NB);
    if constexpr (VEC) {
      for (int i = t; i < W / 4; i += kBlurThreads) {
        if (4 * i + 3 < avail) {
          *reinterpret_cast<f32x4 *>(&tile[r][4 * i]) =
              __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src) + i);
        } else {
          for (int j = 0; j < 4; ++j) tile[r][4 * i + j] = (4 * i + j < avail) ? src[4 * i + j] : 0.f;
        }
      }
    } else {
      for (int i = t; i < W; i += kBlurThreads) tile[r][i] = (i < avail) ? src[i] : 0.f;
    }
  }
  __syncthreads();
  const int64_t x = x0 + 4 * t;
#pragma unroll
  for (int r = 0; r < ROWS; ++r) {
    if (y0 + r >= ny) break;
    float w[4 + 2 * NB];
#pragma unroll
    for (int j = 0; j < (4 + 2 * NB) / 4; ++j) {
      const f32x4 q = *reinterpret_cast<const f32x4 *>(&tile[r][4 * t + 4 * j]);
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
    float *dst = b + (y0 + r) * nx + x;
    if (VEC && x + 3 < nx) {
      const f32x4 q = {o[0], o[1], o[2], o[3]};
      __builtin_nontemporal_store(q, reinterpret_cast<f32x4 *>(dst));
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (x + j < nx) dst[j] = o[j];
    }
  }
}

// Wave-private x blur (nblur = 8, 16-B aligned rows): a wave owns one
// 256-wide x segment × RW consecutive rows.  Each row's window
// [x0-8, x0+264) is loaded with float4 non-temporal loads (64 lanes: 256
// floats; lanes 0-3: the last 16) into the wave's own LDS slot — no block
// barrier — and the next row's loads are issued before this row's LDS work,
// so every wave keeps a row in flight.  Each lane then forms 4 outputs from
// 20 window values in the same ascending-tap order as k_blur_x (bit-exact).
template <int RW>
__global__ __launch_bounds__(kBlurThreads) void k_blur_x_wave(const float *__restrict__ a, float *__restrict__ b,
                                                              int64_t ny, int64_t nx, int64_t ghost, int64_t nseg,
                                                              int64_t nwaves) {
  constexpr int NB = 8, W = 256 + 2 * NB;
  __shared__ __attribute__((aligned(16))) float buf[kBlurThreads / kWave][2][W];
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  const int64_t gw = static_cast<int64_t>(blockIdx.x) * (kBlurThreads / kWave) + w;
  if (gw >= nwaves) return;  // wave-uniform
  const int64_t seg = gw % nseg, rg = gw / nseg;
  const int64_t x0 = seg * 256, y0 = rg * RW;
  const int64_t P = nx + 2 * ghost;
  const int64_t avail = nx + 2 * NB - x0;  // window floats that exist in the row
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  auto load = [&](int64_t y, f32x4 &m, f32x4 &t) {
    const float *src = a + (y + ghost) * P + (ghost - NB) + x0;
    m = zero;
    t = zero;
    if (4 * lane + 3 < avail) {
      m = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src) + lane);
    } else {
      for (int j = 0; j < 4; ++j)
        if (4 * lane + j < avail) m[j] = src[4 * lane + j];
    }
    if (lane < 4) {
      const int64_t o = 256 + 4 * lane;
      if (o + 3 < avail) {
        t = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(src + o));
      } else {
        for (int j = 0; j < 4; ++j)
          if (o + j < avail) t[j] = src[o + j];
      }
    }
  };
  f32x4 m, t;
  load(y0, m, t);
  for (int r = 0; r < RW; ++r) {
    const int64_t y = y0 + r;
    if (y >= ny) break;  // wave-uniform
    float *wb = buf[w][r & 1];
    *reinterpret_cast<f32x4 *>(wb + 4 * lane) = m;
    if (lane < 4) *reinterpret_cast<f32x4 *>(wb + 256 + 4 * lane) = t;
    if (r + 1 < RW && y + 1 < ny) load(y + 1, m, t);  // next row in flight
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float v[4 + 2 * NB];
#pragma unroll
    for (int j = 0; j < (4 + 2 * NB) / 4; ++j) {
      const f32x4 q = *reinterpret_cast<const f32x4 *>(wb + 4 * lane + 4 * j);
      v[4 * j] = q[0];
      v[4 * j + 1] = q[1];
      v[4 * j + 2] = q[2];
      v[4 * j + 3] = q[3];
    }
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float res = 0.f;
#pragma unroll
      for (int k = 0; k <= 2 * NB; ++k) res += v[j + k];
      o[j] = res;
    }
    const int64_t x = x0 + 4 * lane;
    float *dst = b + y * nx + x;
    if (x + 3 < nx) {
      __builtin_nontemporal_store(o, reinterpret_cast<f32x4 *>(dst));
    } else {
      for (int j = 0; j < 4; ++j)
        if (x + j < nx) dst[j] = o[j];
    }
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
      // plain (cached) loads: the next y-tile re-reads the last 2·NB rows from this XCD's L2
      const V q = *reinterpret_cast<const V *>(src + i * P);
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
                                                         int64_t z_end, int64_t ntx, int64_t nty,
                                                         int64_t ntz) {
  // logical tile (x fastest, then y, then z) after the XCD remap
  const int64_t t = xcd_tile(blockIdx.x, ntx * nty * ntz);
  const int64_t tx = t % ntx, ty = (t / ntx) % nty, tz = t / (ntx * nty);
  const int64_t x = tx * kS7X + threadIdx.x;
  const int64_t y = ty * kS7Y + threadIdx.y;
  const int64_t zs = z_begin + tz * kS7Z;
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
    out[p - u] = r;  // plain: L2 merges partial lines with the x-neighbour tile (same XCD)
    zm = zc;
    zc = zp;
    p += Pyx;
  }
}

// Buffer-addressed ring: a wave owns RY rows × 64·NJ consecutive x and streams
// a z chunk through a register ring of planes (z-1, z, z+1 in use, PF
// loading), addressed so the ring costs registers only for data:
//  * loads/stores are raw buffer ops on per-row descriptors (scalar base =
//    plane + row), voffset = one per-lane VGPR (x), the 64-float block step an
//    immediate — no 64-bit VGPR address per load (the flat version spent ~200
//    VGPRs on them: 340 → 1 wave/SIMD);
//  * x±1 are DPP wave_shr:1 / wave_shl:1 moves whose lane-0 / lane-63 inputs
//    (the neighbouring block's edge value) are readlane broadcasts, instead of
//    ds_bpermute shuffles;
//  * the z chunk is a runtime argument so the grid can be sized to occupancy.
// Lanes of the last x tile may read past their row (x ≥ nx + g): those values
// feed only lanes that are never stored; past the array end the descriptor's
// range check returns 0.
__device__ __forceinline__ int fbits(float v) { return __builtin_bit_cast(int, v); }
__device__ __forceinline__ float bitsf(int v) { return __builtin_bit_cast(float, v); }
constexpr int kDppWaveShl1 = 0x130;  // lane i ← lane i+1 (lane 63 keeps `old`)
constexpr int kDppWaveShr1 = 0x138;  // lane i ← lane i-1 (lane 0 keeps `old`)

// PF = prefetch distance in planes: the ring holds PF + 3 slots (planes z-1, z, z+1 being used,
// PF planes in flight); its rotation is unrolled so every slot index is a compile-time constant.
// STORE: 0 plain dword stores, 1 non-temporal dword stores, 4 staged: each row's
// results go to the wave's LDS row (shifted so the body is 16-B aligned) and
// leave as float4 stores plus ≤ 3-float head/tail pieces (needs a 16-B aligned
// `out`).
template <int RY, int NJ, int STORE, int PF = 1>
__global__ __launch_bounds__(256) void k_stencil7_buf(const float *__restrict__ u, float *__restrict__ out,
                                                      int64_t nz, int64_t ny, int64_t nx, int64_t g,
                                                      float c0, float c1, int64_t z_begin, int64_t z_end,
                                                      int64_t ntx, int64_t nty, int64_t ntz, int64_t zc) {
  constexpr int TW = NJ * kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int64_t t = xcd_tile(blockIdx.x, ntx * nty * ntz);
  const int64_t x0 = (t % ntx) * TW;
  const int64_t y0 = (((t / ntx) % nty) * 4 + w) * RY;
  const int64_t zs = z_begin + (t / (ntx * nty)) * zc;
  if (zs >= z_end || y0 >= ny) return;  // wave-uniform
  const int64_t ze = zs + zc < z_end ? zs + zc : z_end;
  const int64_t Px = nx + 2 * g;
  const int64_t Pyx = (ny + 2 * g) * Px;
  const int vx = static_cast<int>((x0 + lane + g) * 4);
  const int ve = static_cast<int>((lane == 0 ? x0 - 1 + g : x0 + TW + g) * 4);
  // Element offsets of rows y0-1 .. y0+RY (wave-uniform).  Every row gets its own
  // descriptor (scalar base = plane + row, num_records = bytes left to the end
  // of the padded array), so voffset is only x and the range check still stops
  // the x-tile lanes past the last ghost row of the last plane.
  int64_t rowo[RY + 2];
#pragma unroll
  for (int r = 0; r < RY + 2; ++r) {
    int64_t yy = y0 - 1 + r;
    yy = yy < ny ? yy : ny;
    rowo[r] = (yy + g) * Px;
  }
  const int64_t total = (nz + 2 * g) * Pyx;  // padded array elements (u and out alike)
  auto rsrc = [&](const float *base, int64_t z, int r) {
    const int64_t off = ((z < nz ? z : nz) + g) * Pyx + rowo[r];
    const int64_t left = (total - off) * 4;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base + off), 0,
                                             static_cast<int>(left < 0x7fffffff ? left : 0x7fffffff), 0x00020000);
  };
  struct Slot {
    float v[RY + 2][NJ];
    float e[RY];
  };
  constexpr int NS = PF + 3;
  Slot R[NS];
  auto load = [&](Slot &S, int64_t z) {
#pragma unroll
    for (int r = 0; r < RY + 2; ++r) {
      const auto rs = rsrc(u, z, r);
#pragma unroll
      for (int j = 0; j < NJ; ++j) S.v[r][j] = bitsf(__builtin_amdgcn_raw_buffer_load_b32(rs, vx + 256 * j, 0, 0));
      if (r >= 1 && r <= RY) S.e[r - 1] = bitsf(__builtin_amdgcn_raw_buffer_load_b32(rs, ve, 0, 0));
    }
  };
  constexpr int SROW = STORE == 4 ? TW + 4 : 1;
  __shared__ __attribute__((aligned(16))) float stage[STORE == 4 ? 4 : 1][STORE == 4 ? RY : 1][SROW];
  const int64_t len = nx - x0 < TW ? nx - x0 : TW;  // outputs of this tile per row
  auto step = [&](const Slot &M, const Slot &Cc, const Slot &Pp, int64_t z) {
    if (z >= ze) return;
    // staged store: element offset of (z, y0+r, x0) and its 16-B head length, per row
    int hd[RY];
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      const int64_t e0 = (z + g) * Pyx + rowo[r + 1] + g + x0;
      hd[r] = static_cast<int>((4 - (e0 & 3)) & 3);
    }
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      if (y0 + r >= ny) break;
      const auto ws = rsrc(out, z, r + 1);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float cz = Cc.v[r + 1][j];
        // bit patterns throughout: readlane/update_dpp and the b32 buffer builtins take/return
        // integers (a float would convert by value)
        const int lft = j > 0 ? __builtin_amdgcn_readlane(fbits(Cc.v[r + 1][j > 0 ? j - 1 : 0]), kWave - 1)
                              : __builtin_amdgcn_readlane(fbits(Cc.e[r]), 0);
        const int rgt = j < NJ - 1 ? __builtin_amdgcn_readlane(fbits(Cc.v[r + 1][j < NJ - 1 ? j + 1 : 0]), 0)
                                   : __builtin_amdgcn_readlane(fbits(Cc.e[r]), kWave - 1);
        const float xm = bitsf(__builtin_amdgcn_update_dpp(lft, fbits(cz), kDppWaveShr1, 0xF, 0xF, false));
        const float xp = bitsf(__builtin_amdgcn_update_dpp(rgt, fbits(cz), kDppWaveShl1, 0xF, 0xF, false));
        float sum = __fadd_rn(M.v[r + 1][j], Pp.v[r + 1][j]);
        sum = __fadd_rn(sum, Cc.v[r][j]);
        sum = __fadd_rn(sum, Cc.v[r + 2][j]);
        sum = __fadd_rn(sum, xm);
        sum = __fadd_rn(sum, xp);
        const float res = __fadd_rn(__fmul_rn(c0, cz), __fmul_rn(c1, sum));
        if constexpr (STORE == 4) {
          stage[w][r][kWave * j + lane + ((4 - hd[r]) & 3)] = res;  // x_local + shift: body 16-B aligned
        } else if (x0 + kWave * j + lane < nx) {
          __builtin_amdgcn_raw_buffer_store_b32(fbits(res), ws, vx + 256 * j, 0, STORE == 1 ? 2 : 0);
        }
      }
    }
    if constexpr (STORE == 4) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int r = 0; r < RY; ++r) {
        if (y0 + r >= ny) break;
        const int h = hd[r] < len ? hd[r] : static_cast<int>(len);
        const int sh = (4 - hd[r]) & 3;
        float *orow = out + (z + g) * Pyx + rowo[r + 1] + g + x0;
        const float *st = stage[w][r];
        if (lane < h) __builtin_nontemporal_store(st[lane + sh], orow + lane);
        const int nb4 = static_cast<int>((len - h) / 4);
#pragma unroll
        for (int k = 0; k < (TW + kWave * 4 - 1) / (kWave * 4); ++k) {
          const int q = lane + kWave * k;
          if (q < nb4)
            __builtin_nontemporal_store(*reinterpret_cast<const f32x4 *>(st + h + 4 * q + sh),
                                        reinterpret_cast<f32x4 *>(orow + h + 4 * q));
        }
        const int t0 = h + 4 * nb4;
        if (lane < len - t0) __builtin_nontemporal_store(st[t0 + lane + sh], orow + t0 + lane);
      }
    }
  };
  // plane p lives in slot (p - zs + 1) mod NS
#pragma unroll
  for (int k = 0; k < PF + 2; ++k) load(R[k], zs - 1 + k);
  for (int64_t z = zs; z < ze; z += NS) {
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      load(R[(k + PF + 2) % NS], z + k + PF + 1);
      step(R[k % NS], R[(k + 1) % NS], R[(k + 2) % NS], z + k);
    }
  }
}

// x4 ring (`LHPC_STENCIL7_IMPL=buf4`): the buffer ring with 4 consecutive x per
// lane — lane l of x-block j (256 floats) holds x0 + 256j + 4l .. +3, loaded by
// one dwordx4 per row and block at 4-B alignment (the 514-float pitch never
// makes rows 8-B aligned; unaligned 16-B buffer loads run at the full rate).
// x±1 inside a lane are register moves; across lanes one DPP move per side,
// whose lane-0 / lane-63 inputs are readlane broadcasts as in k_stencil7_buf.
// Same operation order per cell, so results are bit-identical.  With
// nx % (64·NJ) == 0 (PART false) every x4 of a tile ends at or before column
// nx-1+g.  PART: the last x tile is partial; its 256-column blocks that reach
// past nx (a wave-uniform test) load their x4s as four dword buffer loads
// (the row's ghost column and whatever follows it, 0 past the array end —
// never a partially out-of-range x4) and store only the lane's columns below
// nx: a whole x4 as one dwordx4, a 1–3-column remainder as dwords.  STORE: 5
// the 4 results leave as one unaligned dwordx4 store, 6 the same non-temporal.
// SHARE: the four waves of a block hold consecutive row groups, so a wave's
// y±1 halo rows of the centre plane are its neighbours' edge rows: those go
// through LDS (double-buffered by plane parity, one block barrier per plane)
// and only the block's outer two halo rows are loaded, 10 rows per plane and
// block instead of 16.  Waves past ny then stay to the end (barriers) and
// store nothing.  Same values in the same registers: bit-identical.
template <int RY, int NJ, int STORE, int PF = 1, bool PART = false, bool SHARE = false>
__global__ __launch_bounds__(256) void k_stencil7_buf4(const float *__restrict__ u, float *__restrict__ out,
                                                       int64_t nz, int64_t ny, int64_t nx, int64_t g,
                                                       float c0, float c1, int64_t z_begin, int64_t z_end,
                                                       int64_t ntx, int64_t nty, int64_t ntz, int64_t zc) {
  static_assert(NJ % 4 == 0, "x4 blocks");
  constexpr int NB = NJ / 4;
  constexpr int TW = NJ * kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x) / kWave);
  const int64_t t = xcd_tile(blockIdx.x, ntx * nty * ntz);
  const int64_t x0 = (t % ntx) * TW;
  const int64_t y0 = (((t / ntx) % nty) * 4 + w) * RY;
  const int64_t zs = z_begin + (t / (ntx * nty)) * zc;
  if (zs >= z_end) return;                // block-uniform
  if (!SHARE && y0 >= ny) return;         // wave-uniform
  __shared__ u32x4 hx[SHARE ? 2 : 1][SHARE ? 4 : 1][2][NB][kWave];
  const int64_t ze = zs + zc < z_end ? zs + zc : z_end;
  const int64_t Px = nx + 2 * g;
  const int64_t Pyx = (ny + 2 * g) * Px;
  const int vx = static_cast<int>((x0 + 4 * lane + g) * 4);
  const int ve = static_cast<int>((lane == 0 ? x0 - 1 + g : x0 + TW + g) * 4);
  int64_t rowo[RY + 2];
#pragma unroll
  for (int r = 0; r < RY + 2; ++r) {
    int64_t yy = y0 - 1 + r;
    yy = yy < ny ? yy : ny;
    rowo[r] = (yy + g) * Px;
  }
  const int64_t total = (nz + 2 * g) * Pyx;
  auto rsrc = [&](const float *base, int64_t z, int r) {
    const int64_t off = ((z < nz ? z : nz) + g) * Pyx + rowo[r];
    const int64_t left = (total - off) * 4;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base + off), 0,
                                             static_cast<int>(left < 0x7fffffff ? left : 0x7fffffff), 0x00020000);
  };
  struct Slot {
    u32x4 v[RY + 2][NB];
    float e[RY];
  };
  constexpr int NS = PF + 3;
  Slot R[NS];
  auto load = [&](Slot &S, int64_t z) {
#pragma unroll
    for (int r = 0; r < RY + 2; ++r) {
      // SHARE: inner halo rows come from the neighbouring wave through LDS
      if (SHARE && ((r == 0 && w > 0) || (r == RY + 1 && w < 3))) continue;
      const auto rs = rsrc(u, z, r);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (PART && x0 + 256 * (j + 1) > nx) {  // block reaches past nx: dword loads
#pragma unroll
          for (int k = 0; k < 4; ++k)
            S.v[r][j][k] = static_cast<uint32_t>(__builtin_amdgcn_raw_buffer_load_b32(rs, vx + 1024 * j + 4 * k, 0, 0));
        } else {
          S.v[r][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, vx + 1024 * j, 0, 0);
        }
      }
      if (r >= 1 && r <= RY) S.e[r - 1] = bitsf(__builtin_amdgcn_raw_buffer_load_b32(rs, ve, 0, 0));
    }
  };
  auto step = [&](const Slot &M, Slot &Cc, const Slot &Pp, int64_t z) {
    if (z >= ze) return;  // block-uniform
    if constexpr (SHARE) {
      const int par = static_cast<int>(z & 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        hx[par][w][0][j][lane] = Cc.v[1][j];
        hx[par][w][1][j][lane] = Cc.v[RY][j];
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if (w > 0) Cc.v[0][j] = hx[par][w - 1][1][j][lane];
        if (w < 3) Cc.v[RY + 1][j] = hx[par][w + 1][0][j][lane];
      }
    }
#pragma unroll
    for (int r = 0; r < RY; ++r) {
      if (y0 + r >= ny) break;
      const auto ws = rsrc(out, z, r + 1);
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const u32x4 c = Cc.v[r + 1][j];
        const int lft = j > 0 ? __builtin_amdgcn_readlane(static_cast<int>(Cc.v[r + 1][j > 0 ? j - 1 : 0][3]), kWave - 1)
                              : __builtin_amdgcn_readlane(fbits(Cc.e[r]), 0);
        const int rgt = j < NB - 1
                            ? __builtin_amdgcn_readlane(static_cast<int>(Cc.v[r + 1][j < NB - 1 ? j + 1 : 0][0]), 0)
                            : __builtin_amdgcn_readlane(fbits(Cc.e[r]), kWave - 1);
        const float xm0 = bitsf(__builtin_amdgcn_update_dpp(lft, static_cast<int>(c[3]), kDppWaveShr1, 0xF, 0xF, false));
        const float xp3 = bitsf(__builtin_amdgcn_update_dpp(rgt, static_cast<int>(c[0]), kDppWaveShl1, 0xF, 0xF, false));
        u32x4 res;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float cz = bitsf(static_cast<int>(c[k]));
          const float xm = k > 0 ? bitsf(static_cast<int>(c[k > 0 ? k - 1 : 0])) : xm0;
          const float xp = k < 3 ? bitsf(static_cast<int>(c[k < 3 ? k + 1 : 3])) : xp3;
          float sum = __fadd_rn(bitsf(static_cast<int>(M.v[r + 1][j][k])), bitsf(static_cast<int>(Pp.v[r + 1][j][k])));
          sum = __fadd_rn(sum, bitsf(static_cast<int>(Cc.v[r][j][k])));
          sum = __fadd_rn(sum, bitsf(static_cast<int>(Cc.v[r + 2][j][k])));
          sum = __fadd_rn(sum, xm);
          sum = __fadd_rn(sum, xp);
          const float o = __fadd_rn(__fmul_rn(c0, cz), __fmul_rn(c1, sum));
          res[k] = static_cast<uint32_t>(fbits(o));
        }
        if (PART && x0 + 256 * (j + 1) > nx) {
          const int64_t vc = nx - (x0 + 256 * j + 4 * lane);  // this lane's columns below nx
          if (vc >= 4) {
            __builtin_amdgcn_raw_buffer_store_b128(res, ws, vx + 1024 * j, 0, STORE == 6 ? 2 : 0);
          } else {
#pragma unroll
            for (int k = 0; k < 3; ++k)
              if (k < vc)
                __builtin_amdgcn_raw_buffer_store_b32(static_cast<int>(res[k]), ws, vx + 1024 * j + 4 * k, 0,
                                                      STORE == 6 ? 2 : 0);
          }
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(res, ws, vx + 1024 * j, 0, STORE == 6 ? 2 : 0);
        }
      }
    }
  };
#pragma unroll
  for (int k = 0; k < PF + 2; ++k) load(R[k], zs - 1 + k);
  for (int64_t z = zs; z < ze; z += NS) {
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      load(R[(k + PF + 2) % NS], z + k + PF + 1);
      step(R[k % NS], R[(k + 1) % NS], R[(k + 2) % NS], z + k);
    }
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
                int nb, hipStream_t s, const lhpc_options &o) {
  const int64_t cells = ny * nx;
  if (cells == 0) return LHPC_OK;
  const int64_t P = nx + 2 * ghost;
  if (!ydir) {
    if (nb == 8) {
      constexpr int SEG = 4 * kBlurThreads;
      const int64_t nseg = (nx + SEG - 1) / SEG;
      const bool vec = aligned16(a) && aligned16(b) && P % 4 == 0 && nx % 4 == 0 &&
                       (ghost - 8) % 4 == 0;
      const dim3 bd(kBlurThreads);
#define LHPC_BX(V, R)                                                                                  \
  hipLaunchKernelGGL((k_blur_x<8, V, R>), dim3(static_cast<unsigned>(((ny + R - 1) / R) * nseg)), bd, 0, s, \
                     a, b, ny, nx, ghost)
      // the wave-private kernel, 2 rows per wave (measured 85 us against 99-103 us for the
      // block-LDS kernel on 8192^2); the block-LDS kernel only for rows that
      // are not 16-B aligned
      if (vec) {
        const int rw = o.blur_x_rows > 0 ? o.blur_x_rows : 2;
        const int64_t nseg256 = (nx + 255) / 256;
#define LHPC_BXW(RWV)                                                                                        \
  do {                                                                                                       \
    const int64_t nw = nseg256 * ((ny + RWV - 1) / RWV);                                                      \
    hipLaunchKernelGGL((k_blur_x_wave<RWV>), dim3(static_cast<unsigned>((nw + 3) / 4)), bd, 0, s, a, b, ny, nx, \
                       ghost, nseg256, nw);                                                                  \
  } while (0)
        switch (rw) {
          case 1: LHPC_BXW(1); break;
          case 2: LHPC_BXW(2); break;
          case 4: LHPC_BXW(4); break;
          case 16: LHPC_BXW(16); break;
          case 32: LHPC_BXW(32); break;
          default: LHPC_BXW(8); break;
        }
#undef LHPC_BXW
      } else {
        LHPC_BX(false, 2);
      }
#undef LHPC_BX
    } else {
      hipLaunchKernelGGL(k_blur_x_generic, dim3(static_cast<unsigned>((cells + kBlurThreads - 1) / kBlurThreads)),
                         dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, nb);
    }
  } else {
    if (nb == 8) {
      const bool vec4 = aligned16(a) && aligned16(b) && P % 4 == 0 && nx % 4 == 0 && ghost % 4 == 0;
      const bool vec2 = aligned16(a) && aligned16(b) && P % 2 == 0 && nx % 2 == 0 && ghost % 2 == 0;
      // register-window shape: VEC columns × TY rows per thread (window TY+16 rows)
      // register-window shape (vec, ty); plain loads: 4x16 measured best (84 us, 8192^2)
      const int cfg = (o.blur_y_vec > 0 ? o.blur_y_vec : 4) * 1000 + (o.blur_y_rows > 0 ? o.blur_y_rows : 16);
#define LHPC_BY(V, TY)                                                                              \
  do {                                                                                              \
    const int64_t n_ytiles = (ny + TY - 1) / TY;                                                    \
    const int64_t n_strips = (nx + V * kBlurThreads - 1) / (V * kBlurThreads);                       \
    hipLaunchKernelGGL((k_blur_y<8, V, TY>), dim3(static_cast<unsigned>(n_strips * n_ytiles)),       \
                       dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, n_strips, n_ytiles);           \
  } while (0)
      if (vec4 && cfg == 4016) LHPC_BY(4, 16);
      else if (vec4 && cfg == 4032) LHPC_BY(4, 32);
      else if (vec2 && cfg == 2032) LHPC_BY(2, 32);
      else if (vec2 && cfg == 2048) LHPC_BY(2, 48);
      else if (cfg == 1064) LHPC_BY(1, 64);
      else if (cfg == 1048) LHPC_BY(1, 48);
      else if (vec4) LHPC_BY(4, 16);
      else LHPC_BY(1, 16);
#undef LHPC_BY
    } else {
      hipLaunchKernelGGL(k_blur_y_generic, dim3(static_cast<unsigned>((cells + kBlurThreads - 1) / kBlurThreads)),
                         dim3(kBlurThreads), 0, s, a, b, ny, nx, ghost, nb);
    }
  }
  return check_launch(s);
}

int blur_entry(bool ydir, const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
               int nblur, int on_device, void *stream, const lhpc_options *opts) {
  if (!a || !b || ny < 0 || nx < 0 || nblur < 0 || ghost < nblur) return LHPC_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const lhpc_options o = resolve_options(opts);
  if (on_device) return blur_launch(ydir, a, b, ny, nx, ghost, nblur, s, o);
  const size_t in_bytes = static_cast<size_t>((ny + 2 * ghost) * (nx + 2 * ghost)) * 4;
  const size_t out_bytes = static_cast<size_t>(ny * nx) * 4;
  HostStage da, db;
  LHPC_HIP_TRY(hipMalloc(&da.d, in_bytes ? in_bytes : 16));
  LHPC_HIP_TRY(hipMalloc(&db.d, out_bytes ? out_bytes : 16));
  LHPC_HIP_TRY(hipMemcpy(da.d, a, in_bytes, hipMemcpyHostToDevice));  // host buffers: synchronous copies
  LHPC_TRY(blur_launch(ydir, static_cast<float *>(da.d), static_cast<float *>(db.d), ny, nx, ghost,
                       nblur, s, o));
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  LHPC_HIP_TRY(hipMemcpy(b, db.d, out_bytes, hipMemcpyDeviceToHost));
  return LHPC_OK;
}

#ifdef LHPC_TUNING_ENV
constexpr bool kS7AllTiles = true;
#else
constexpr bool kS7AllTiles = false;
#endif
struct S7Args {
  const float *u;
  float *out;
  int64_t nz, ny, nx, g;
  float c0, c1;
  int64_t zb, ze, zc;
  hipStream_t s;
};
// x4 ring, one tile shape: LDS-shared halos (prefetch 2) or the private ring
// at prefetch depth 1–3.  Product build: the 2-row tile only with shared halos
template <int RY, int NJ, int M, bool P>
int s74_launch(const S7Args &a, bool share, int pf) {
  const int64_t ntx = (a.nx + NJ * kWave - 1) / (NJ * kWave), nty = (a.ny + 4 * RY - 1) / (4 * RY),
                ntz = (a.ze - a.zb + a.zc - 1) / a.zc;
  const dim3 grid(static_cast<unsigned>(ntx * nty * ntz)), blk(256);
#define LHPC_S74_GO(PFV, SH)                                                                               \
  hipLaunchKernelGGL((k_stencil7_buf4<RY, NJ, M, PFV, P, SH>), grid, blk, 0, a.s, a.u, a.out, a.nz, a.ny, a.nx, \
                     a.g, a.c0, a.c1, a.zb, a.ze, ntx, nty, ntz, a.zc)
  if (share) {
    LHPC_S74_GO(2, true);
  } else if constexpr (kS7AllTiles || RY == 1) {
    if (pf == 2) LHPC_S74_GO(2, false);
    else if (pf == 3) LHPC_S74_GO(3, false);
    else LHPC_S74_GO(1, false);
  } else {
    return LHPC_ERR_UNSUPPORTED;
  }
#undef LHPC_S74_GO
  return LHPC_OK;
}
template <int RY, int NJ>
int s74_store(const S7Args &a, bool m5, bool part, bool share, int pf) {
  if (m5) return part ? s74_launch<RY, NJ, 5, true>(a, share, pf) : s74_launch<RY, NJ, 5, false>(a, share, pf);
  return part ? s74_launch<RY, NJ, 6, true>(a, share, pf) : s74_launch<RY, NJ, 6, false>(a, share, pf);
}
// dword ring, one tile shape and store mode, prefetch depth 1–3
template <int RY, int NJ, int M>
int s7b_launch(const S7Args &a, int pf) {
  const int64_t ntx = (a.nx + NJ * kWave - 1) / (NJ * kWave), nty = (a.ny + 4 * RY - 1) / (4 * RY),
                ntz = (a.ze - a.zb + a.zc - 1) / a.zc;
  const dim3 grid(static_cast<unsigned>(ntx * nty * ntz)), blk(256);
#define LHPC_S7B_GO(PFV)                                                                                   \
  hipLaunchKernelGGL((k_stencil7_buf<RY, NJ, M, PFV>), grid, blk, 0, a.s, a.u, a.out, a.nz, a.ny, a.nx, a.g,  \
                     a.c0, a.c1, a.zb, a.ze, ntx, nty, ntz, a.zc)
  if (pf == 2) LHPC_S7B_GO(2);
  else if (pf == 3) LHPC_S7B_GO(3);
  else LHPC_S7B_GO(1);
#undef LHPC_S7B_GO
  return LHPC_OK;
}
template <int RY, int NJ>
int s7b_store(const S7Args &a, int store_mode, int pf) {
  if (store_mode == 1) return s7b_launch<RY, NJ, 1>(a, pf);
  if (store_mode == 4) return s7b_launch<RY, NJ, 4>(a, pf);
  return s7b_launch<RY, NJ, 0>(a, pf);
}

int s7_launch(const float *u, float *out, int64_t nz, int64_t ny, int64_t nx, int64_t g, float c0,
              float c1, int64_t zb, int64_t ze, hipStream_t s, const lhpc_options &o) {
  if (zb >= ze || ny == 0 || nx == 0) return LHPC_OK;
  // implementation: the buffer ring ("buf"), in its x4 form ("buf4") when the x
  // tiles are full; the thread-per-column kernel only when a row's byte
  // offset does not fit a buffer voffset.  The measured alternatives (LDS
  // 2.5-D tile, register ring, deep prefetch, flat wide ring) are in DESIGN.md §4.
  const int impl = o.stencil7_impl;
  // Store policy of the dword ring: staged (default: float4 stores via the
  // wave's LDS row, 219-220 us vs 225-226 plain on 512^3; plain when `out` is
  // not 16-B aligned) | plain | nt.
  const int stm = o.stencil7_store;
  const bool buf4_req = impl == LHPC_S7_RING_X4 || impl == LHPC_S7_RING_X4_LDS;
  const bool buf_impl = impl == LHPC_S7_AUTO || impl == LHPC_S7_RING || buf4_req;
  int store_mode = stm == LHPC_STORE_PLAIN ? 0 : stm == LHPC_STORE_NT ? 1 : 4;
  if (store_mode == 4 && !aligned16(out)) store_mode = 0;  // staged float4 stores need a 16-B base
  // buffer-addressed ring: the in-row byte offset (voffset) must fit 31 bits
  const bool row_b31 = (nx + 2 * g + 1024) * 4 < (int64_t{1} << 31);
  if (buf_impl && row_b31) {
    // Tiling RY×(64·NJ) per wave, 4 waves per block.  The z chunk is sized so the grid is about
    // one block per CU (256): measured on 512^3, fewer concurrent z fronts beat
    // more waves — 2,8 at zc 128 (256 blocks) 209-220 us vs 250 us at zc 32 (1024 blocks);
    // prefetch depth (PF) and store policy (plain vs nt) are secondary.
    // default tile: 2 rows × 8 blocks for the dword ring; 2 rows × 4 blocks (256 x) for the
    // x4 ring with LDS-shared halos (512^3, same box, three runs each: 2,8 200.9 µs, 2,4 195.6,
    // 1,8 196.0, 4,8 214.7; 384 / 512 blocks instead of 256: 232-234 µs)
    // Round 5 (512^3, same box, five interleaved runs each, profiles/r05/stencil_ab.jsonl):
    // 1 row × 8 blocks (a wave owns 512 consecutive x of one row) 188.4–190.2 µs against
    // 192.2–195.0 for 2 × 4, so rows of ≥ 512 columns take 1 × 8.  More waves per block
    // (one z front over 8 or 16 waves' rows) were slower: 196–236 µs.
    const bool x4_default = impl == LHPC_S7_AUTO || impl == LHPC_S7_RING_X4_LDS;
    const bool wide = x4_default && nx >= 512;
    // (the dword ring — opt-in, S7_RING — takes 1 row × 8 blocks: its 2-row
    // tiles spill SGPRs and are tuning-build only since round 6)
    int ry = o.stencil7_ry > 0 ? o.stencil7_ry : (x4_default && !wide ? 2 : 1),
        nj = o.stencil7_nj > 0 ? o.stencil7_nj : (x4_default && !wide ? 4 : 8);
    int zc = o.stencil7_zc, pf = o.stencil7_pf;
    // x4 ring by default when every x tile is full (nx % (64·NJ) == 0): 198-211 us against
    // 209-225 us for the dword ring on 512^3, same boxes; "buf" forces the dword ring
    // (partial last x tiles included: k_stencil7_buf4<…, PART>)
    const bool buf4 = (buf4_req || impl == LHPC_S7_AUTO) && (nj == 4 || nj == 8);
    const bool part = nx % (int64_t{nj} * kWave) != 0;
    // LDS-shared halo rows (x4 ring, prefetch depth 2): the default (512^3,
    // same box, two runs each: 206.8 / 198.4 µs → 201.3 / 193.2 µs)
    const bool share = impl == LHPC_S7_RING_X4_LDS || impl == LHPC_S7_AUTO;
    if (pf < 1) pf = buf4 ? 2 : 1;  // prefetch planes: x4 PF 2 198 us vs PF 1 210-217 / PF 3 203
    if (zc < 1) {
      const int64_t target = o.stencil7_blocks > 0 ? o.stencil7_blocks : 256;
      const int64_t tw = int64_t{nj} * kWave, th = 4 * int64_t{ry};
      const int64_t xy = ((nx + tw - 1) / tw) * ((ny + th - 1) / th);
      const int64_t nchunks = std::max<int64_t>(1, (target + xy - 1) / xy);
      zc = static_cast<int>(std::max<int64_t>(4, (ze - zb + nchunks - 1) / nchunks));
    }
    // product build: only the tiles whose kernels keep every register in
    // registers (1 row per wave, or the x4 ring's LDS-shared 2 × 4 default;
    // tests/test_kernel_resources.py) — any other tile is LHPC_ERR_UNSUPPORTED.
    // The tuning build (-DLHPC_TUNING_ENV) compiles every measured tile.
    const S7Args a{u, out, nz, ny, nx, g, c0, c1, zb, ze, zc, s};
    int st = LHPC_ERR_UNSUPPORTED;
    if (buf4) {  // x4 ring: non-temporal dwordx4 stores ("plain": plain)
      const bool m5 = stm == LHPC_STORE_PLAIN;
      if (ry == 1 && nj == 8) st = s74_store<1, 8>(a, m5, part, share, pf);
      else if (ry == 1 && nj == 4) st = s74_store<1, 4>(a, m5, part, share, pf);
      else if (ry == 2 && nj == 4) st = s74_store<2, 4>(a, m5, part, share, pf);
#ifdef LHPC_TUNING_ENV
      else if (ry == 4 && nj == 8) st = s74_store<4, 8>(a, m5, part, share, pf);
      else if (ry == 4 && nj == 4) st = s74_store<4, 4>(a, m5, part, share, pf);
      else st = s74_store<2, 8>(a, m5, part, share, pf);
#endif
    } else {
      if (ry == 1 && nj == 8) st = s7b_store<1, 8>(a, store_mode, pf);
      else if (ry == 1 && nj == 4) st = s7b_store<1, 4>(a, store_mode, pf);
#ifdef LHPC_TUNING_ENV
      else if (ry == 4 && nj == 8) st = s7b_store<4, 8>(a, store_mode, pf);
      else if (ry == 2 && nj == 4) st = s7b_store<2, 4>(a, store_mode, pf);
      else if (ry == 4 && nj == 4) st = s7b_store<4, 4>(a, store_mode, pf);
      else st = s7b_store<2, 8>(a, store_mode, pf);
#endif
    }
    if (st != LHPC_OK) return st;
    return check_launch(s);
  }
  const int64_t ntx = (nx + kS7X - 1) / kS7X, nty = (ny + kS7Y - 1) / kS7Y, ntz = (ze - zb + kS7Z - 1) / kS7Z;
  hipLaunchKernelGGL(k_stencil7, dim3(static_cast<unsigned>(ntx * nty * ntz)), dim3(kS7X, kS7Y), 0, s, u, out, nz,
                     ny, nx, g, c0, c1, zb, ze, ntx, nty, ntz);
  return check_launch(s);
}

}  // namespace
}  // namespace lhpc

using namespace lhpc;

extern "C" int lhpc_blur_x_f32(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                               int nblur, int on_device, void *stream) {
  try {
    return blur_entry(false, a, b, ny, nx, ghost, nblur, on_device, stream, nullptr);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_blur_y_f32(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                               int nblur, int on_device, void *stream) {
  try {
    return blur_entry(true, a, b, ny, nx, ghost, nblur, on_device, stream, nullptr);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_blur_x_f32_opts(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost, int nblur,
                                    int on_device, void *stream, const lhpc_options *opts) {
  try {
    return blur_entry(false, a, b, ny, nx, ghost, nblur, on_device, stream, opts);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_blur_y_f32_opts(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost, int nblur,
                                    int on_device, void *stream, const lhpc_options *opts) {
  try {
    return blur_entry(true, a, b, ny, nx, ghost, nblur, on_device, stream, opts);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_stencil7_f32_planes_opts(const float *u, float *out, int64_t nz, int64_t ny, int64_t nx,
                                             int64_t ghost, float c0, float c1, int64_t z_begin, int64_t z_end,
                                             void *stream, const lhpc_options *opts) {
  try {
    if (!u || !out || nz < 0 || ny < 0 || nx < 0 || ghost < 1 || z_begin < 0 || z_end > nz)
      return LHPC_ERR_INVALID_ARG;
    return s7_launch(u, out, nz, ny, nx, ghost, c0, c1, z_begin, z_end, static_cast<hipStream_t>(stream),
                     resolve_options(opts));
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_stencil7_f32_planes(const float *u, float *out, int64_t nz, int64_t ny,
                                        int64_t nx, int64_t ghost, float c0, float c1,
                                        int64_t z_begin, int64_t z_end, void *stream) {
  try {
    return lhpc_stencil7_f32_planes_opts(u, out, nz, ny, nx, ghost, c0, c1, z_begin, z_end, stream, nullptr);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_stencil7_f32(const float *u, float *out, int64_t nz, int64_t ny, int64_t nx,
                                 int64_t ghost, float c0, float c1, int on_device, void *stream) {
  try {
    if (!u || !out || nz < 0 || ny < 0 || nx < 0 || ghost < 1) return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const lhpc_options o = resolve_options(nullptr);
    if (on_device) return s7_launch(u, out, nz, ny, nx, ghost, c0, c1, 0, nz, s, o);
    const size_t bytes =
        static_cast<size_t>((nz + 2 * ghost) * (ny + 2 * ghost) * (nx + 2 * ghost)) * 4;
    HostStage du, dout;
    LHPC_HIP_TRY(hipMalloc(&du.d, bytes));
    LHPC_HIP_TRY(hipMalloc(&dout.d, bytes));
    LHPC_HIP_TRY(hipMemcpy(du.d, u, bytes, hipMemcpyHostToDevice));  // host buffers: synchronous copies
    // ghost cells of `out` keep the caller's values
    LHPC_HIP_TRY(hipMemcpy(dout.d, out, bytes, hipMemcpyHostToDevice));
    LHPC_TRY(s7_launch(static_cast<float *>(du.d), static_cast<float *>(dout.d), nz, ny, nx, ghost, c0,
                       c1, 0, nz, s, o));
    LHPC_HIP_TRY(hipStreamSynchronize(s));
    LHPC_HIP_TRY(hipMemcpy(out, dout.d, bytes, hipMemcpyDeviceToHost));
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
