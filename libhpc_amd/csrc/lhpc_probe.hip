// lhpc_probe.hip — attainable-rate probes used by bench.py / DESIGN.md to
// place the SpMV and stencil kernels against measured ceilings (not part of
// the include/lhpc.h ABI).  The reference's own probe of this kind is the
// coalescing micro-benchmark lib/gpu/stall_lg_testsuite/src/cuda_tut_stall_lg.cu:63-71
// (int4-wide copy); these are written for wave64 / gfx950.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "lhpc_common.hpp"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace {

__global__ __launch_bounds__(256) void k_copy16(const f32x4 *__restrict__ s, f32x4 *__restrict__ d,
                                               int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}

// width / cache-policy / access-order copy probes (stencil write-path study):
// CHUNKED = false: grid-stride (the whole grid sweeps one front through memory);
// CHUNKED = true: block b copies its own contiguous 1/grid of the buffer (grid fronts).
template <typename T, bool NT, bool CHUNKED>
__global__ __launch_bounds__(256) void k_copyw(const T *__restrict__ s, T *__restrict__ d, int64_t n) {
  if constexpr (CHUNKED) {
    const int64_t per = (n + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = static_cast<int64_t>(blockIdx.x) * per;
    const int64_t b1 = b0 + per < n ? b0 + per : n;
    for (int64_t i = b0 + threadIdx.x; i < b1; i += 256) {
      if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
      else d[i] = s[i];
    }
  } else {
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
      if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
      else d[i] = s[i];
    }
  }
}

// Read:write mix probe (round 5): block t reads one 16-KB tile (16 B per lane,
// non-temporal) and writes W 16-KB tiles (W stores per lane, plain or
// non-temporal), so the stream moves W bytes written per byte read — the mix
// of the XTILE gather (fp32: col16 2 B read per 4 B of xg written; fp64 per
// 8 B) against the 1:1 copy.
template <int W, bool NTS>
__global__ __launch_bounds__(1024) void k_fan(const f32x4 *__restrict__ s, f32x4 *__restrict__ d, int64_t tiles) {
  extern __shared__ float fan_lds[];  // dynamic LDS: only to cap blocks per CU (occupancy study)
  if (threadIdx.x == 0 && tiles < 0) fan_lds[0] = 0.f;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const f32x4 v = __builtin_nontemporal_load(s + t * 1024 + threadIdx.x);
#pragma unroll
    for (int w = 0; w < W; ++w) {
      f32x4 o = v;
      o.x += static_cast<float>(w);
      if constexpr (NTS) __builtin_nontemporal_store(o, d + (t * W + w) * 1024 + threadIdx.x);
      else d[(t * W + w) * 1024 + threadIdx.x] = o;
    }
  }
}

// Unrolled 16-B/lane probes (round 5 calibration against MI355X_MICROARCH.md's
// 6.29 TB/s float4 copy): a block moves a tile of U·BLK float4 per iteration
// (U loads in flight per lane, each wave instruction 1 KB contiguous) and
// strides over tiles by the grid.  MODE bit 0: non-temporal loads, bit 1:
// non-temporal stores, bit 2: read only (sum kept alive), bit 3: write only.
template <int BLK, int U, int MODE>
__global__ __launch_bounds__(BLK) void k_copy_u(const f32x4 *__restrict__ s, f32x4 *__restrict__ d, int64_t n) {
  constexpr bool NTL = MODE & 1, NTS = MODE & 2, RO = MODE & 4, WO = MODE & 8;
  const int64_t tile = static_cast<int64_t>(BLK) * U;
  const int64_t tiles = n / tile;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t b = t * tile + threadIdx.x;
    f32x4 v[U];
    if constexpr (!WO) {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = NTL ? __builtin_nontemporal_load(s + b + u * BLK) : s[b + u * BLK];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = f32x4{static_cast<float>(t), 1.f, 2.f, static_cast<float>(u)};
    }
    if constexpr (RO) {
#pragma unroll
      for (int u = 0; u < U; ++u) acc += v[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if constexpr (NTS) __builtin_nontemporal_store(v[u], d + b + u * BLK);
        else d[b + u * BLK] = v[u];
      }
    }
  }
  // the tail (n not a multiple of the tile): block 0, one float4 per lane
  if (blockIdx.x == 0)
    for (int64_t i = tiles * tile + threadIdx.x; i < n; i += BLK) {
      if constexpr (RO) acc += s[i];
      else d[i] = WO ? f32x4{0.f, 0.f, 0.f, 0.f} : s[i];
    }
  if constexpr (RO)
    if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.678f) d[0] = acc;  // keep the loads alive
}

__global__ __launch_bounds__(256) void k_read16(const f32x4 *__restrict__ s, float *__restrict__ sink,
                                               int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  float acc = 0.f;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
    const f32x4 v = __builtin_nontemporal_load(s + i);
    acc += v[0] + v[1] + v[2] + v[3];
  }
  if (acc == 12345.678f) sink[0] = acc;  // keep the loads alive
}

// dword-per-lane streaming read (FETCH_SIZE calibration for 4-byte loads)
__global__ __launch_bounds__(256) void k_read4(const float *__restrict__ s, float *__restrict__ sink,
                                              int64_t n) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  float acc = 0.f;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride)
    acc += __builtin_nontemporal_load(s + i);
  if (acc == 12345.678f) sink[0] = acc;
}

// out[i] = table[idx[i]]: a 4-byte random gather per lane with the index
// stream read non-temporally (the SpMV x-gather in isolation).
template <int U>
__global__ __launch_bounds__(256) void k_gather(const int32_t *__restrict__ idx,
                                               const float *__restrict__ table,
                                               float *__restrict__ out, int64_t n) {
  const int64_t base = (static_cast<int64_t>(blockIdx.x) * 256 * U) + threadIdx.x;
  int32_t c[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    c[u] = i < n ? __builtin_nontemporal_load(idx + i) : -1;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (c[u] >= 0) __builtin_nontemporal_store(table[c[u]], out + i);
  }
}

// Column-sliced variant: block b gathers only from slice sl(b) of the table,
// idx holds offsets within a slice.  S <= 8: sl = b % S (one slice per XCD
// group).  S = 16: XCD group k = b % 8 does slice k for its first half of
// blocks, then slice k + 8.
template <int U, bool NT>
__global__ __launch_bounds__(256) void k_gather_sliced(const int32_t *__restrict__ idx,
                                                      const float *__restrict__ table,
                                                      float *__restrict__ out, int64_t n,
                                                      int S, int64_t slice_len) {
  const int64_t b = blockIdx.x;
  int sl;
  if (S <= 8) {
    sl = static_cast<int>(b % S);
  } else {
    const int64_t per = (static_cast<int64_t>(gridDim.x) + 7) / 8;
    sl = static_cast<int>(b % 8) + 8 * static_cast<int>((b / 8) * 2 / per);
  }
  const float *tb = table + sl * slice_len;
  const int64_t base = (b * 256 * U) + threadIdx.x;
  int32_t c[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    c[u] = i < n ? __builtin_nontemporal_load(idx + i) : -1;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (c[u] >= 0) {
      const float v = NT ? __builtin_nontemporal_load(tb + c[u]) : tb[c[u]];
      __builtin_nontemporal_store(v, out + i);
    }
  }
}

// Fragment probe (round 6): the XTILE reduce's memory access shape and
// occupancy without its compute (scan, rank, segmented scan).  One block per
// chunk of M = BLK·RUN positions, chunks walked as the reduce walks them
// (c = C − 1 − ((b % 8)·Cx + b / 8)); per chunk:
//   round trip 1  the chunk's row of the segment table: S u32 starts;
//   stream        RUN values of T + RUN u16 per thread, wave-transposed (each
//                 load instruction 1 KB contiguous, non-temporal) — the
//                 reduce's val + iperm;
//   round trip 2  the chunk's S fragments of xg (segment j = flat positions
//                 [⌊j·M/S⌋, ⌊(j+1)·M/S⌋), in the tile-major stream at
//                 C·⌊j·M/S⌋ + c·len_j) into LDS in flat order: fp32 by 4-B
//                 LDS-DMA (as the reduce); fp64 (F64 = 0) as 8-B buffer loads
//                 + ds_write_b64 (as the reduce), (F64 = 1) as two 4-B LDS-DMA
//                 per 64 lanes (32 positions per instruction);
// then one barrier and a trivial read of the run (kept alive through sink).
template <typename T, int BLK, int F64>
__global__ __launch_bounds__(BLK) void k_frag(const uint32_t *__restrict__ seg, const T *__restrict__ xg,
                                             int xg_bytes, const T *__restrict__ val,
                                             const uint16_t *__restrict__ ip, int S, int64_t C, int64_t Cx,
                                             double *__restrict__ sink) {
  constexpr int RUN = 64 / static_cast<int>(sizeof(T)), M = BLK * RUN, NB = M / BLK;
  constexpr int VW = 16 / static_cast<int>(sizeof(T)), NV = RUN / VW, REG = lhpc::kWave * RUN, NIP = RUN * 2 / 16;
  typedef T tvec __attribute__((ext_vector_type(VW)));
  extern __shared__ __align__(16) unsigned char frag_lds[];
  T *xs = reinterpret_cast<T *>(frag_lds);
  int *base = reinterpret_cast<int *>(xs + M + VW);
  const int tid = threadIdx.x, lane = tid & (lhpc::kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid / lhpc::kWave);
  const int64_t c = C - 1 - (static_cast<int64_t>(blockIdx.x % 8) * Cx + blockIdx.x / 8);
  if (c < 0) return;
  for (int j = tid; j < S; j += BLK)
    base[j] = static_cast<int>(seg[c * S + j]) - static_cast<int>(static_cast<int64_t>(j) * M / S);
  tvec vv[NV];
  {
    const tvec *vp = reinterpret_cast<const tvec *>(val + c * M + wv * REG) + lane;
#pragma unroll
    for (int q = 0; q < NV; ++q) vv[q] = __builtin_nontemporal_load(vp + q * lhpc::kWave);
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<T *>(xg), 0, xg_bytes, 0x00020000);
  auto src_of = [&](int f) {  // stream index of flat position f of chunk c
    const int j = static_cast<int>((static_cast<int64_t>(f + 1) * S + M - 1) / M) - 1;
    return base[j] + f;
  };
  if constexpr (sizeof(T) == 4) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int u = 0; u < NB; ++u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void *)(xs + (wv * NB + u) * lhpc::kWave), 4,
          src_of((wv * NB + u) * lhpc::kWave + lane) * 4, 0, 0, 0);
#endif
  } else if constexpr (F64 == 1) {
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
    for (int u = 0; u < 2 * NB; ++u)  // 32 positions (64 dwords) per instruction
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void *)(xs + (wv * NB * 2 + u) * 32), 4,
          src_of((wv * NB * 2 + u) * 32 + lane / 2) * 8 + (lane & 1) * 4, 0, 0, 0);
#endif
  } else {
    T xv[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u)
      xv[u] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(
                                        rs, src_of((wv * NB + u) * lhpc::kWave + lane) * 8, 0, 0));
#pragma unroll
    for (int u = 0; u < NB; ++u) xs[(wv * NB + u) * lhpc::kWave + lane] = xv[u];
  }
  lhpc::u32x4 ipv[NIP];
  {
    const lhpc::u32x4 *p = reinterpret_cast<const lhpc::u32x4 *>(ip + c * M + wv * REG) + lane;
#pragma unroll
    for (int q = 0; q < NIP; ++q) ipv[q] = __builtin_nontemporal_load(p + q * lhpc::kWave);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  double acc = 0.0;
#pragma unroll
  for (int j = 0; j < RUN; ++j)
    acc += static_cast<double>(vv[j / VW][j % VW]) * static_cast<double>(xs[tid * RUN + j]) +
           static_cast<double>(ipv[j / 8][(j % 8) / 2] & 1u);
  if (acc == 1234.5678) sink[0] = acc;  // keep every load alive
}

}  // namespace

// k_frag: t = 4 (fp32, 512 threads) or 8 (fp64, 1024 threads); f64_dma picks
// the fp64 fragment load (0: b64 + ds_write, 1: 4-B LDS-DMA); lds_bytes of
// dynamic LDS (≥ M·t + 16 + 4·S) sets the blocks per CU as the reduce's does.
// seg[c·S + j] = stream start of chunk c's segment j; val: C·M of t, ip: C·M u16.
extern "C" int lhpc_probe_frag(const uint32_t *seg, const void *xg, int64_t xg_bytes, const void *val,
                               const uint16_t *ip, int S, int64_t C, int t, int f64_dma, int lds_bytes,
                               double *sink, void *stream) {
  if (C <= 0 || S <= 0 || xg_bytes <= 0 || xg_bytes >= (int64_t{1} << 31)) return static_cast<int>(hipErrorInvalidValue);
  const int64_t Cx = (C + 7) / 8;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 grid(static_cast<unsigned>(8 * Cx));
  if (t == 4) {
    const int M = 512 * 16;
    if (lds_bytes < M * 4 + 16 + 4 * S) return static_cast<int>(hipErrorInvalidValue);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(k_frag<float, 512, 0>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    hipLaunchKernelGGL((k_frag<float, 512, 0>), grid, dim3(512), lds_bytes, st, seg, static_cast<const float *>(xg),
                       static_cast<int>(xg_bytes), static_cast<const float *>(val), ip, S, C, Cx, sink);
  } else if (t == 8) {
    const int M = 1024 * 8;
    if (lds_bytes < M * 8 + 16 + 4 * S) return static_cast<int>(hipErrorInvalidValue);
    const void *fn = f64_dma ? reinterpret_cast<const void *>(k_frag<double, 1024, 1>)
                             : reinterpret_cast<const void *>(k_frag<double, 1024, 0>);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    if (f64_dma)
      hipLaunchKernelGGL((k_frag<double, 1024, 1>), grid, dim3(1024), lds_bytes, st, seg,
                         static_cast<const double *>(xg), static_cast<int>(xg_bytes),
                         static_cast<const double *>(val), ip, S, C, Cx, sink);
    else
      hipLaunchKernelGGL((k_frag<double, 1024, 0>), grid, dim3(1024), lds_bytes, st, seg,
                         static_cast<const double *>(xg), static_cast<int>(xg_bytes),
                         static_cast<const double *>(val), ip, S, C, Cx, sink);
  } else {
    return static_cast<int>(hipErrorInvalidValue);
  }
  return static_cast<int>(hipGetLastError());
}

// Check of lhpc::wave_incl_scan (DPP) against a shuffle scan, per wave.
__global__ __launch_bounds__(256) void k_wave_scan(const int *__restrict__ in, int *__restrict__ dpp,
                                                   int *__restrict__ ref, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int v = i < n ? in[i] : 0;
  int r = v;
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(r, d, 64);
    if (lane >= d) r += t;
  }
  const int s = lhpc::wave_incl_scan(v);
  if (i < n) {
    dpp[i] = s;
    ref[i] = r;
  }
}

extern "C" int lhpc_probe_wave_scan(const int *in, int *dpp, int *ref, int64_t n, void *stream) {
  hipLaunchKernelGGL(k_wave_scan, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), in, dpp, ref, n);
  return static_cast<int>(hipGetLastError());
}

extern "C" int lhpc_probe_gather_sliced(const int32_t *idx, const float *table, float *out,
                                        int64_t n, int S, int64_t slice_len, int nt, void *stream) {
  constexpr int U = 8;
  const int64_t blocks = (n + 256 * U - 1) / (256 * U);
  if (nt)
    hipLaunchKernelGGL((k_gather_sliced<U, true>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), idx, table, out, n, S, slice_len);
  else
    hipLaunchKernelGGL((k_gather_sliced<U, false>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), idx, table, out, n, S, slice_len);
  return static_cast<int>(hipGetLastError());
}

extern "C" int lhpc_probe_copy(const void *src, void *dst, int64_t bytes, int grid, void *stream) {
  hipLaunchKernelGGL(k_copy16, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const f32x4 *>(src), static_cast<f32x4 *>(dst), bytes / 16);
  return static_cast<int>(hipGetLastError());
}

extern "C" int lhpc_probe_read(const void *src, void *sink, int64_t bytes, int grid, void *stream) {
  hipLaunchKernelGGL(k_read16, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const f32x4 *>(src), static_cast<float *>(sink), bytes / 16);
  return static_cast<int>(hipGetLastError());
}

extern "C" int lhpc_probe_read4(const void *src, void *sink, int64_t bytes, int grid, void *stream) {
  hipLaunchKernelGGL(k_read4, dim3(grid), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const float *>(src), static_cast<float *>(sink), bytes / 4);
  return static_cast<int>(hipGetLastError());
}

extern "C" int lhpc_probe_gather(const int32_t *idx, const float *table, float *out, int64_t n,
                                 void *stream) {
  constexpr int U = 8;
  const int64_t blocks = (n + 256 * U - 1) / (256 * U);
  hipLaunchKernelGGL((k_gather<U>), dim3(static_cast<unsigned>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), idx, table, out, n);
  return static_cast<int>(hipGetLastError());
}

// k_copy_u: block ∈ {256, 512, 1024}, unroll ∈ {1, 2, 4, 8}, mode as k_copy_u's
// MODE (0–15; read-only and write-only exclusive).  Returns hipErrorInvalidValue
// for a combination not instantiated.
template <int BLK, int U>
static hipError_t launch_copy_u(const f32x4 *s, f32x4 *d, int64_t n, int grid, int mode, hipStream_t st) {
  switch (mode) {
#define LHPC_CU(M) \
  case M: hipLaunchKernelGGL((k_copy_u<BLK, U, M>), dim3(grid), dim3(BLK), 0, st, s, d, n); break;
    LHPC_CU(0) LHPC_CU(1) LHPC_CU(2) LHPC_CU(3) LHPC_CU(4) LHPC_CU(5) LHPC_CU(8) LHPC_CU(10)
#undef LHPC_CU
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
template <int BLK>
static hipError_t launch_copy_b(const f32x4 *s, f32x4 *d, int64_t n, int grid, int unroll, int mode, hipStream_t st) {
  switch (unroll) {
    case 1: return launch_copy_u<BLK, 1>(s, d, n, grid, mode, st);
    case 2: return launch_copy_u<BLK, 2>(s, d, n, grid, mode, st);
    case 4: return launch_copy_u<BLK, 4>(s, d, n, grid, mode, st);
    case 8: return launch_copy_u<BLK, 8>(s, d, n, grid, mode, st);
    default: return hipErrorInvalidValue;
  }
}
extern "C" int lhpc_probe_copy_u(const void *src, void *dst, int64_t bytes, int grid, int block, int unroll,
                                 int mode, void *stream) {
  const f32x4 *s = static_cast<const f32x4 *>(src);
  f32x4 *d = static_cast<f32x4 *>(dst);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t n = bytes / 16;
  hipError_t e = block == 256    ? launch_copy_b<256>(s, d, n, grid, unroll, mode, st)
                 : block == 512  ? launch_copy_b<512>(s, d, n, grid, unroll, mode, st)
                 : block == 1024 ? launch_copy_b<1024>(s, d, n, grid, unroll, mode, st)
                                 : hipErrorInvalidValue;
  return static_cast<int>(e);
}

// width ∈ {4, 8, 16} bytes per lane; mode bit 0 = non-temporal, bit 1 = chunked (see k_copyw)
extern "C" int lhpc_probe_copy_w(const void *src, void *dst, int64_t bytes, int grid, int width, int mode,
                                 void *stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
#define LHPC_CW(T, W)                                                                                     \
  do {                                                                                                    \
    const T *sp = static_cast<const T *>(src);                                                           \
    T *dp = static_cast<T *>(dst);                                                                        \
    const int64_t n = bytes / W;                                                                          \
    switch (mode & 3) {                                                                                   \
      case 0: hipLaunchKernelGGL((k_copyw<T, false, false>), dim3(grid), dim3(256), 0, st, sp, dp, n); break; \
      case 1: hipLaunchKernelGGL((k_copyw<T, true, false>), dim3(grid), dim3(256), 0, st, sp, dp, n); break;  \
      case 2: hipLaunchKernelGGL((k_copyw<T, false, true>), dim3(grid), dim3(256), 0, st, sp, dp, n); break;  \
      default: hipLaunchKernelGGL((k_copyw<T, true, true>), dim3(grid), dim3(256), 0, st, sp, dp, n); break;  \
    }                                                                                                     \
  } while (0)
  if (width == 4) LHPC_CW(float, 4);
  else if (width == 8) LHPC_CW(f32x2, 8);
  else LHPC_CW(f32x4, 16);
#undef LHPC_CW
  return static_cast<int>(hipGetLastError());
}

// tiles 16-KB tiles read, tiles·w written (w ∈ {1, 2, 3, 4}); nt_store: non-temporal stores;
// lds_bytes of dynamic LDS per block (0: none) caps the blocks per CU
extern "C" int lhpc_probe_fan(const void *src, void *dst, int64_t tiles, int w, int nt_store, int grid,
                              int lds_bytes, void *stream) {
  const f32x4 *s = static_cast<const f32x4 *>(src);
  f32x4 *d = static_cast<f32x4 *>(dst);
  hipStream_t st = static_cast<hipStream_t>(stream);
#define LHPC_FAN(W)                                                                                     \
  case W:                                                                                               \
    if (nt_store) hipLaunchKernelGGL((k_fan<W, true>), dim3(grid), dim3(1024), lds_bytes, st, s, d, tiles); \
    else hipLaunchKernelGGL((k_fan<W, false>), dim3(grid), dim3(1024), lds_bytes, st, s, d, tiles);         \
    break;
  switch (w) {
    LHPC_FAN(1) LHPC_FAN(2) LHPC_FAN(3) LHPC_FAN(4)
    default: return static_cast<int>(hipErrorInvalidValue);
  }
#undef LHPC_FAN
  return static_cast<int>(hipGetLastError());
}
