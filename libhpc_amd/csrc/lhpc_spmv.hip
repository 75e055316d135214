// lhpc_spmv.hip — CSR SpMV y = A·x for gfx950 (MI355X), behind include/lhpc.h.
//
// The reference has no SpMV; the operator is defined
// here as y[i] = Σ_{k=row_ptr[i]}^{row_ptr[i+1]-1} val[k]·x[col_idx[k]].
// Numerics: every dtype accumulates in fp64 registers and rounds once at the
// store (SURVEY §8c "binding recommendation"), so fp32 results are within
// 2^-24·|y| + ~1e-16·Σ|a·x| of the exact sum for any row length.
//
// Kernel families:
//   ROWGROUP  L lanes per row (L | 64), R rows per lane group per wave, all
//             loads hoisted so a wave keeps R gathers + R val/col loads in
//             flight; the row sum is a DPP butterfly inside one 16-lane DPP
//             row for L <= 16 (no LDS), then one coalesced y store per wave.
//   ADAPTIVE  nnz-balanced row blocks: a 256-thread workgroup streams up to
//             kBlockNnz contiguous nonzeros (coalesced), stages fp64 products
//             in LDS, and reduces each row with L = 256/rows lanes; a row
//             longer than kBlockNnz gets a workgroup to itself.  For skewed
//             (power-law) row lengths.  Deterministic: fixed trees only.
// Both read val/col_idx with non-temporal loads (streamed once) so the
// gathered x keeps its place in L2 / Infinity Cache.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "lhpc_common.hpp"
#include "lhpc_plan.hpp"

namespace lhpc {
namespace {

constexpr int kBlock = 256;
constexpr int kBlockNnz = 2048;  // ADAPTIVE: nonzeros per stream block
constexpr int kLongRow = 48;     // XSLICE: in-slice rows longer than this are wave-reduced

// ------------------------------------------------------------- ROWGROUP
template <typename T, typename I, int L, int R>
__global__ __launch_bounds__(kBlock) void k_spmv_rowgroup(
    const I *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const T *__restrict__ val, const T *__restrict__ x, T *__restrict__ y,
    int64_t n_rows) {
  constexpr int G = kWave / L;     // lane groups (rows) per wave per step
  constexpr int WR = G * R;        // rows per wave
  static_assert(WR <= kWave, "one y store per wave");
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane & (L - 1);  // lane within its group
  const int grp = lane / L;        // group within the wave
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) / kWave;
  const int64_t row0 = wave * WR;
  if (row0 >= n_rows) return;  // wave-uniform

  int64_t s[R], e[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t row = row0 + r * G + grp;
    if (row < n_rows) {
      s[r] = row_ptr[row];
      e[r] = row_ptr[row + 1];
    } else {
      s[r] = e[r] = 0;
    }
  }
  // first L-wide chunk of every row, loads hoisted for memory-level parallelism
  int32_t c[R];
  T v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t k = s[r] + sub;
    c[r] = -1;
    v[r] = T(0);
    if (k < e[r]) {
      c[r] = ld_stream(col + k);
      v[r] = ld_stream(val + k);
    }
  }
  double acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    acc[r] = 0.0;
    if (c[r] >= 0) acc[r] = static_cast<double>(v[r]) * static_cast<double>(x[c[r]]);
  }
  // rows longer than L (rare for the uniform workload)
#pragma unroll
  for (int r = 0; r < R; ++r) {
    for (int64_t k = s[r] + sub + L; k < e[r]; k += L)
      acc[r] += static_cast<double>(ld_stream(val + k)) *
                static_cast<double>(x[ld_stream(col + k)]);
  }
  // all 64 lanes active here: DPP reads never see a disabled source lane
  T out = T(0);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const T tot = static_cast<T>(group_sum<L>(acc[r]));
    // lane l (< WR) stores row row0 + l = row0 + (l/G)*G + l%G: take the
    // sum of step r = l/G from group g = l%G
    const T mine = __shfl(tot, (lane % G) * L, kWave);
    if (lane / G == r) out = mine;
  }
  if (lane < WR && row0 + lane < n_rows) __builtin_nontemporal_store(out, y + row0 + lane);
}

// ------------------------------------------------------------- ADAPTIVE
// blocks[b] = first row of block b; blocks[n_blocks] = n_rows.
template <typename T, typename I>
__global__ __launch_bounds__(kBlock) void k_spmv_adaptive(
    const I *__restrict__ row_ptr, const int32_t *__restrict__ col,
    const T *__restrict__ val, const T *__restrict__ x, T *__restrict__ y,
    const int64_t *__restrict__ blocks, const T *__restrict__ w, double *__restrict__ dpart) {
  // DOT (w != nullptr): also dpart[block] = Σ_rows y[row]·w[row] over the block's rows
  // (the stored, rounded y), reduced in a fixed order — the CG p·q fused into the SpMV.
  __shared__ double prod[kBlockNnz];
  __shared__ double wsum[kBlock / kWave];
  const int tid = threadIdx.x;
  const int64_t r0 = blocks[blockIdx.x];
  const int64_t r1 = blocks[blockIdx.x + 1];
  const int64_t base = row_ptr[r0];
  const int64_t cnt = static_cast<int64_t>(row_ptr[r1]) - base;
  const int64_t nrows = r1 - r0;

  if (cnt > kBlockNnz) {
    // one long row: strided per-thread sums, then a fixed block tree
    double a = 0.0;
    for (int64_t k = tid; k < cnt; k += kBlock)
      a += static_cast<double>(ld_stream(val + base + k)) *
           static_cast<double>(x[ld_stream(col + base + k)]);
    a = group_sum<kWave>(a);
    if ((tid & (kWave - 1)) == 0) wsum[tid / kWave] = a;
    __syncthreads();
    if (tid == 0) {
      double t = wsum[0];
#pragma unroll
      for (int i = 1; i < kBlock / kWave; ++i) t += wsum[i];
      const T yv = static_cast<T>(t);
      y[r0] = yv;
      if (w) dpart[blockIdx.x] = static_cast<double>(yv) * static_cast<double>(w[r0]);
    }
    return;
  }
  // stream phase: every thread products kBlockNnz/kBlock nonzeros
  constexpr int PER = kBlockNnz / kBlock;
  int32_t c[PER];
  T v[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int64_t k = i * kBlock + tid;
    c[i] = -1;
    v[i] = T(0);
    if (k < cnt) {
      c[i] = ld_stream(col + base + k);
      v[i] = ld_stream(val + base + k);
    }
  }
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int k = i * kBlock + tid;
    if (c[i] >= 0) prod[k] = static_cast<double>(v[i]) * static_cast<double>(x[c[i]]);
  }
  __syncthreads();
  // reduce: L lanes per row, L = largest power of two with nrows*L <= 256
  int L = kWave;
  while (L > 1 && nrows * L > kBlock) L >>= 1;
  const int grp = tid / L, sub = tid & (L - 1);
  double a = 0.0;
  int64_t rs = 0, re = 0;
  if (grp < nrows) {
    rs = static_cast<int64_t>(row_ptr[r0 + grp]) - base;
    re = static_cast<int64_t>(row_ptr[r0 + grp + 1]) - base;
    for (int64_t k = rs + sub; k < re; k += L) a += prod[k];
  }
  switch (L) {  // block-uniform
    case 64: a = group_sum<64>(a); break;
    case 32: a = group_sum<32>(a); break;
    case 16: a = group_sum<16>(a); break;
    case 8: a = group_sum<8>(a); break;
    case 4: a = group_sum<4>(a); break;
    case 2: a = group_sum<2>(a); break;
    default: break;
  }
  double d = 0.0;
  if (grp < nrows && sub == 0) {
    const T yv = static_cast<T>(a);
    y[r0 + grp] = yv;
    if (w) d = static_cast<double>(yv) * static_cast<double>(w[r0 + grp]);
  }
  if (w) {  // block-uniform
    d = group_sum<kWave>(d);
    __syncthreads();  // wsum reuse
    if ((tid & (kWave - 1)) == 0) wsum[tid / kWave] = d;
    __syncthreads();
    if (tid == 0) {
      double t = wsum[0];
#pragma unroll
      for (int i = 1; i < kBlock / kWave; ++i) t += wsum[i];
      dpart[blockIdx.x] = t;
    }
  }
}

// --------------------------------------------------------------- XSLICE
// Column-sliced SpMV.  Slice s = g + 8·phase is processed
// by the blocks with blockIdx % 8 == g (the blocks the dispatcher deals to one
// XCD), phase after phase, so each XCD's L2 holds one x slice (≈ 2.5–5 MB)
// and the random x-gathers hit L2 instead of Infinity Cache / HBM (measured:
// 151–168 G gathers/s vs 59 unsliced, tools/probe_slices.py).  Placement is a
// speed heuristic only: any block→XCD mapping gives the same result.
// One lane per row, one wave per 64-row chunk; the chunk's in-slice
// nonzeros are jagged-diagonal, so iteration j reads the active lanes'
// elements contiguously (ballot + mbcnt addressing, no padding).  Each row
// accumulates its in-slice products in fp64 in CSR order and stores one
// partial per (slice, row); k_xslice_reduce adds the S partials in slice
// order.  Loads are unconditional (clamped index) so hipcc keeps U
// iterations of loads in flight instead of branching around each one.
template <typename T, int U>
__global__ __launch_bounds__(kBlock) void k_spmv_xslice(
    const uint8_t *__restrict__ lens, const int64_t *__restrict__ cbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, const T *__restrict__ x,
    T *__restrict__ partial, int64_t n_rows, int64_t n_rows_pad, int64_t n_chunks,
    int64_t blocks_per_slice, int S, int64_t nnz_last) {
  const int64_t b = blockIdx.x;
  int s;
  int64_t wb;
  if (S >= 8) {
    const int64_t g = b % 8, idx = b / 8;
    s = static_cast<int>(g + 8 * (idx / blocks_per_slice));
    wb = idx % blocks_per_slice;
  } else {
    s = static_cast<int>(b % S);
    wb = b / S;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t chunk = wb * (kBlock / kWave) + threadIdx.x / kWave;
  if (s >= S || chunk >= n_chunks) return;  // wave-uniform
  const int64_t row = chunk * kWave + lane;
  const int len = lens[static_cast<int64_t>(s) * n_rows_pad + row];
  int64_t pos = cbase[static_cast<int64_t>(s) * n_chunks + chunk];
  double acc = 0.0;
  for (int j = 0;; j += U) {
    if (__ballot(j < len) == 0) break;  // wave-uniform exit
    int64_t k[U];
    bool act[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      act[u] = (j + u) < len;
      const uint64_t m = __ballot(act[u]);
      const int rank = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0));
      k[u] = act[u] ? pos + rank : (pos < nnz_last ? pos : nnz_last);
      pos += __popcll(m);
    }
    int32_t c[U];
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      c[u] = ld_stream(col + k[u]);
      v[u] = ld_stream(val + k[u]);
    }
    T xv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) xv[u] = x[c[u]];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (act[u]) acc += static_cast<double>(v[u]) * static_cast<double>(xv[u]);
  }
  if (row < n_rows) __builtin_nontemporal_store(static_cast<T>(acc), partial + static_cast<int64_t>(s) * n_rows_pad + row);
}

// XSLICE "stream" form (default): same slicing and XCD grouping, but the
// chunk's in-slice nonzeros are in CSR order and the whole wave streams
// them NB·64 at a time — every lane loads / gathers (full lane utilisation,
// NB gathers in flight per lane) — staging exact fp64 products in a
// wave-private LDS window; lane r then adds its row's products in CSR order.
// Row offsets inside the chunk come from a wave prefix sum of the uint8
// lengths.  A chunk with more than NB·64 nonzeros loops over windows (rows
// spanning windows keep accumulating in order, so the result is unchanged).
template <typename T, typename P, typename LT, int NB>
__global__ __launch_bounds__(kBlock) void k_spmv_xslice_stream(
    const LT *__restrict__ lens, const int64_t *__restrict__ cbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, const T *__restrict__ x,
    P *__restrict__ partial, int64_t n_rows, int64_t n_rows_pad, int64_t n_chunks,
    int64_t blocks_per_slice, int S) {
  constexpr int CAP = NB * kWave;
  __shared__ double prod[kBlock / kWave][CAP];
  const int64_t b = blockIdx.x;
  int s;
  int64_t wb;
  if (S >= 8) {
    const int64_t g = b % 8, idx = b / 8;
    s = static_cast<int>(g + 8 * (idx / blocks_per_slice));
    wb = idx % blocks_per_slice;
  } else {
    s = static_cast<int>(b % S);
    wb = b / S;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const int64_t chunk = wb * (kBlock / kWave) + wv;
  if (s >= S || chunk >= n_chunks) return;  // wave-uniform
  const int64_t row = chunk * kWave + lane;
  const int len = lens[static_cast<int64_t>(s) * n_rows_pad + row];
  const int64_t base = cbase[static_cast<int64_t>(s) * n_chunks + chunk];
  // inclusive wave scan of len → this lane's row offset inside the chunk
  int inc = len;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int t = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += t;
  }
  const int off = inc - len;
  const int cnt = __shfl(inc, kWave - 1, kWave);
  double acc = 0.0;
  double *wp = prod[wv];
  for (int w0 = 0; w0 < cnt; w0 += CAP) {  // wave-uniform
    int32_t c[NB];
    T v[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      int k = w0 + i * kWave + lane;
      k = k < cnt ? k : cnt - 1;  // clamped: loads stay unconditional
      c[i] = ld_stream(col + base + k);
      v[i] = ld_stream(val + base + k);
    }
    T xv[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) xv[i] = x[c[i]];
#pragma unroll
    for (int i = 0; i < NB; ++i)
      wp[i * kWave + lane] = static_cast<double>(v[i]) * static_cast<double>(xv[i]);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int lo = off > w0 ? off : w0;
    const int hi = (off + len) < (w0 + CAP) ? (off + len) : (w0 + CAP);
    // short rows: the owning lane adds its products in CSR order
    if (len <= kLongRow)
      for (int k = lo; k < hi; ++k) acc += wp[k - w0];
    // long rows (skewed matrices): the whole wave sums the row's part of the
    // window — strided lane sums, then a fixed DPP/shuffle tree
    uint64_t m = __ballot(len > kLongRow && lo < hi);
    while (m) {  // wave-uniform
      const int r = __builtin_ctzll(m);
      m &= m - 1;
      const int rlo = __shfl(lo, r, kWave), rhi = __shfl(hi, r, kWave);
      double t = 0.0;
      for (int k = rlo + lane; k < rhi; k += kWave) t += wp[k - w0];
      t = group_sum<kWave>(t);
      if (lane == r) acc += t;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  if (row < n_rows)
    __builtin_nontemporal_store(static_cast<P>(acc), partial + static_cast<int64_t>(s) * n_rows_pad + row);
}

// XSLICE, fused reduction.  Same per-slice work as k_spmv_xslice_stream, but
// instead of a second kernel, the LAST of the S slice-blocks that cover a
// 256-row block adds the S fp64 partial slabs (slice order, identical to
// k_xslice_reduce) and writes y.  Hand-off per cdna_hip_programming.md §6
// Guideline 16 R1: partials stored write-through (8-B agent-scope relaxed
// atomic stores = global_store sc1), every storing wave drains vmcnt, block
// barrier, one lane adds to the block's arrival counter (agent scope); the
// block whose add returns S-1 takes one agent acquire (buffer_inv sc1),
// drains, barriers, and reads the slabs with sc1 loads.  Counters are zeroed
// by a hipMemsetAsync on the same stream before every launch.  Correct for
// any block→XCD placement; placement only changes speed.
template <typename T, typename LT, int NB>
__global__ __launch_bounds__(kBlock) void k_spmv_xslice_fused(
    const LT *__restrict__ lens, const int64_t *__restrict__ cbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, const T *__restrict__ x,
    double *__restrict__ partial, unsigned *__restrict__ arrive, T *__restrict__ y,
    int64_t n_rows, int64_t n_rows_pad, int64_t n_chunks, int64_t blocks_per_slice, int S) {
  constexpr int CAP = NB * kWave;
  __shared__ double prod[kBlock / kWave][CAP];
  __shared__ int last_flag;
  const int64_t b = blockIdx.x;
  int s;
  int64_t wb;
  if (S >= 8) {
    const int64_t g = b % 8, idx = b / 8;
    s = static_cast<int>(g + 8 * (idx / blocks_per_slice));
    wb = idx % blocks_per_slice;
  } else {
    s = static_cast<int>(b % S);
    wb = b / S;
  }
  if (s >= S) return;  // block-uniform (only for grids rounded past S)
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const int64_t chunk = wb * (kBlock / kWave) + wv;
  const bool live = chunk < n_chunks;  // wave-uniform; dead waves still join the barriers
  const int64_t row = chunk * kWave + lane;
  double acc = 0.0;
  if (live) {
    const int len = lens[static_cast<int64_t>(s) * n_rows_pad + row];
    const int64_t base = cbase[static_cast<int64_t>(s) * n_chunks + chunk];
    int inc = len;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int t = __shfl_up(inc, d, kWave);
      if (lane >= d) inc += t;
    }
    const int off = inc - len;
    const int cnt = __shfl(inc, kWave - 1, kWave);
    double *wp = prod[wv];
    for (int w0 = 0; w0 < cnt; w0 += CAP) {
      int32_t c[NB];
      T v[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        int k = w0 + i * kWave + lane;
        k = k < cnt ? k : cnt - 1;
        c[i] = ld_stream(col + base + k);
        v[i] = ld_stream(val + base + k);
      }
      T xv[NB];
#pragma unroll
      for (int i = 0; i < NB; ++i) xv[i] = x[c[i]];
#pragma unroll
      for (int i = 0; i < NB; ++i)
        wp[i * kWave + lane] = static_cast<double>(v[i]) * static_cast<double>(xv[i]);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const int lo = off > w0 ? off : w0;
      const int hi = (off + len) < (w0 + CAP) ? (off + len) : (w0 + CAP);
      if (len <= kLongRow)
        for (int k = lo; k < hi; ++k) acc += wp[k - w0];
      uint64_t m = __ballot(len > kLongRow && lo < hi);
      while (m) {
        const int r = __builtin_ctzll(m);
        m &= m - 1;
        const int rlo = __shfl(lo, r, kWave), rhi = __shfl(hi, r, kWave);
        double t = 0.0;
        for (int k = rlo + lane; k < rhi; k += kWave) t += wp[k - w0];
        t = group_sum<kWave>(t);
        if (lane == r) acc += t;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    // R1 payload: write-through 8-byte store of this row's slice partial
    __hip_atomic_store(reinterpret_cast<unsigned long long *>(partial + static_cast<int64_t>(s) * n_rows_pad + row),
                       __builtin_bit_cast(unsigned long long, acc), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(arrive + wb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_flag = (old == static_cast<unsigned>(S - 1));
    if (last_flag) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last_flag) return;  // block-uniform
  const int64_t r = wb * kBlock + threadIdx.x;
  if (r >= n_rows) return;
  double a = 0.0;
  for (int q = 0; q < S; ++q)
    a += __builtin_bit_cast(double, __hip_atomic_load(
                                        reinterpret_cast<unsigned long long *>(partial + static_cast<int64_t>(q) * n_rows_pad + r),
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  y[r] = static_cast<T>(a);
}

// XSLICE, persistent and partial-free (default for XSLICE plans).  A
// resident grid of waves; in each pass wave w owns G consecutive 64-row
// chunks (one row per lane per chunk, G fp64 accumulators per lane in
// registers) and walks ALL slices in order.  Every wave moves through the
// slices in step, so at any time the chip's L2s hold (about) one x slice —
// no XCD mapping and no per-slice partial sums in HBM.  The G chunks of one
// slice are contiguous (slice-major layout), so a wave streams them as one
// range in windows of NB·64 nonzeros: col/val loads and x gathers at full
// lane utilisation, exact fp64 products staged in a wave-private LDS window,
// then each lane adds its rows' products in CSR order (rows longer than
// kLongRow in one slice are summed by the whole wave).  Row sums therefore
// accumulate slice by slice in fixed order: deterministic.
template <typename T, typename LT, int NB, int G>
__global__ __launch_bounds__(kBlock) void k_spmv_xslice_persist(
    const LT *__restrict__ lens, const int64_t *__restrict__ cbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, const T *__restrict__ x,
    T *__restrict__ y, int64_t n_rows, int64_t n_rows_pad, int64_t n_chunks, int S) {
  constexpr int CAP = NB * kWave;
  __shared__ double prod[kBlock / kWave][CAP];
  const int lane = threadIdx.x & (kWave - 1);
  const int wv = threadIdx.x / kWave;
  const int64_t w = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + wv;
  const int64_t waves = static_cast<int64_t>(gridDim.x) * (kBlock / kWave);
  const int64_t per_pass = waves * G;
  double *wp = prod[wv];
  for (int64_t pass = 0; pass * per_pass < n_chunks; ++pass) {
    const int64_t c0 = pass * per_pass + w * G;
    if (c0 >= n_chunks) break;  // wave-uniform
    const int nc = static_cast<int>((n_chunks - c0) < G ? (n_chunks - c0) : G);
    double acc[G];
#pragma unroll
    for (int c = 0; c < G; ++c) acc[c] = 0.0;
    for (int sl = 0; sl < S; ++sl) {
      int len[G], off[G];
#pragma unroll
      for (int c = 0; c < G; ++c)
        len[c] = c < nc ? static_cast<int>(lens[static_cast<int64_t>(sl) * n_rows_pad + (c0 + c) * kWave + lane]) : 0;
      const int64_t cb = cbase[static_cast<int64_t>(sl) * n_chunks + c0 + (lane <= nc ? lane : nc)];
      const int64_t base = __shfl(cb, 0, kWave);
      const int total = static_cast<int>(__shfl(cb, nc, kWave) - base);
#pragma unroll
      for (int c = 0; c < G; ++c) {
        int inc = len[c];
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
          const int t = __shfl_up(inc, d, kWave);
          if (lane >= d) inc += t;
        }
        off[c] = static_cast<int>(__shfl(cb, c < nc ? c : nc, kWave) - base) + inc - len[c];
      }
      for (int w0 = 0; w0 < total; w0 += CAP) {  // wave-uniform
        int32_t cc[NB];
        T vv[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          int k = w0 + i * kWave + lane;
          k = k < total ? k : total - 1;  // clamped: loads stay unconditional
          cc[i] = ld_stream(col + base + k);
          vv[i] = ld_stream(val + base + k);
        }
        T xv[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) xv[i] = x[cc[i]];
#pragma unroll
        for (int i = 0; i < NB; ++i)
          wp[i * kWave + lane] = static_cast<double>(vv[i]) * static_cast<double>(xv[i]);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int c = 0; c < G; ++c) {
          const int lo = off[c] > w0 ? off[c] : w0;
          const int hi = (off[c] + len[c]) < (w0 + CAP) ? (off[c] + len[c]) : (w0 + CAP);
          if (len[c] <= kLongRow)
            for (int k = lo; k < hi; ++k) acc[c] += wp[k - w0];
          uint64_t m = __ballot(len[c] > kLongRow && lo < hi);
          while (m) {  // wave-uniform
            const int r = __builtin_ctzll(m);
            m &= m - 1;
            const int rlo = __shfl(lo, r, kWave), rhi = __shfl(hi, r, kWave);
            double t = 0.0;
            for (int k = rlo + lane; k < rhi; k += kWave) t += wp[k - w0];
            t = group_sum<kWave>(t);
            if (lane == r) acc[c] += t;
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    }
#pragma unroll
    for (int c = 0; c < G; ++c) {
      const int64_t row = (c0 + c) * kWave + lane;
      if (c < nc && row < n_rows) __builtin_nontemporal_store(static_cast<T>(acc[c]), y + row);
    }
  }
}

// y[i] = Σ_{s=0}^{S-1} partial[s][i], fp64, fixed slice order; 4 rows/thread.
template <typename T, typename P>
__global__ __launch_bounds__(kBlock) void k_xslice_reduce(const P *__restrict__ partial,
                                                          T *__restrict__ y, int64_t n_rows,
                                                          int64_t n_rows_pad, int S) {
  const int64_t i0 = (static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x) * 4;
  if (i0 >= n_rows) return;
  double a[4] = {0.0, 0.0, 0.0, 0.0};
  for (int s = 0; s < S; ++s) {
    const P *p = partial + static_cast<int64_t>(s) * n_rows_pad + i0;
    if constexpr (sizeof(P) == 4) {
      const f32x4 q = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
      a[0] += q[0]; a[1] += q[1]; a[2] += q[2]; a[3] += q[3];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += __builtin_nontemporal_load(p + j);
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (i0 + j < n_rows) y[i0 + j] = static_cast<T>(a[j]);
}

// ---------------------------------------------------------------- XTILE
// (layout: lhpc_plan.hpp XtileHost)
constexpr int kXtGatherBlock = 1024;  // gather: 16 waves per CU, one tile of x in LDS
constexpr int kXtBlock = 256;         // reduce
constexpr int kXtRun = 16;            // reduce: nonzeros per thread (merge-path run)
constexpr int kXtM = kXtBlock * kXtRun;  // chunk capacity (nonzeros)
constexpr int kXtRmax = 512;             // rows owned per chunk
template <typename T> struct XtTile;
template <> struct XtTile<float> { static constexpr int W = 40960; };   // 160 KB
template <> struct XtTile<double> { static constexpr int W = 20480; };  // 160 KB


#ifndef LHPC_XT_GATHER_PRE
#define LHPC_XT_GATHER_PRE 1
#endif
// gather: block b streams pieces[3b..3b+1] of tile pieces[3b+2]; 8 nonzeros
// per thread and step (one 16-B col16 load, 8 LDS gathers, 8 contiguous xg
// stores), U steps in flight.  Piece bounds are multiples of 8.
template <typename T, int U>
__global__ __launch_bounds__(kXtGatherBlock) void k_xtile_gather(
    const int32_t *__restrict__ pieces, const uint16_t *__restrict__ col16,
    const T *__restrict__ x, int64_t n_cols, T *__restrict__ xg) {
  constexpr int W = XtTile<T>::W;
  __shared__ T xt[W];
  const int tid = threadIdx.x;
  const int g0 = pieces[3 * blockIdx.x], g1 = pieces[3 * blockIdx.x + 1];
  const int64_t c0 = static_cast<int64_t>(pieces[3 * blockIdx.x + 2]) * W;
  const int wlen = static_cast<int>((n_cols - c0) < W ? (n_cols - c0) : W);
  constexpr int PT = W / kXtGatherBlock;
  const int q0 = g0 >> 3, q1 = g1 >> 3;  // 8-entry groups
  const u32x4 *cv = reinterpret_cast<const u32x4 *>(col16);
  u32x4 w[U];
  auto load_w = [&](int q) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q + u * kXtGatherBlock;
      w[u] = qq < q1 ? __builtin_nontemporal_load(cv + qq) : u32x4{0, 0, 0, 0};
    }
  };
#if LHPC_XT_GATHER_PRE
  load_w(q0 + tid);  // the first col16 step does not depend on the tile: issue it under the tile load
#endif
  T tv[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int j = i * kXtGatherBlock + tid;
    tv[i] = j < wlen ? x[c0 + j] : T(0);
  }
#pragma unroll
  for (int i = 0; i < PT; ++i) xt[i * kXtGatherBlock + tid] = tv[i];
  __syncthreads();
  for (int q = q0 + tid; q < q1; q += U * kXtGatherBlock) {
#if LHPC_XT_GATHER_PRE
    if (q != q0 + tid) load_w(q);
#else
    load_w(q);
#endif
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q + u * kXtGatherBlock;
      T o[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        o[2 * h] = xt[w[u][h] & 0xFFFFu];
        o[2 * h + 1] = xt[w[u][h] >> 16];
      }
      if (qq < q1) {
        if constexpr (sizeof(T) == 4) {
          f32x4 *d = reinterpret_cast<f32x4 *>(xg + static_cast<int64_t>(qq) * 8);
          d[0] = f32x4{o[0], o[1], o[2], o[3]};
          d[1] = f32x4{o[4], o[5], o[6], o[7]};
        } else {
          typedef double f64x2 __attribute__((ext_vector_type(2)));
          f64x2 *d = reinterpret_cast<f64x2 *>(xg + static_cast<int64_t>(qq) * 8);
#pragma unroll
          for (int h = 0; h < 4; ++h) d[h] = f64x2{o[2 * h], o[2 * h + 1]};
        }
      }
    }
  }
}

// reduce: one block per chunk c = (b % 8)·Cx + b / 8, so each XCD walks a
// contiguous run of chunks and the xg lines two neighbouring chunks share
// stay in its L2.  PMC (profiles/r01/xtile_*): the stream equals the
// algorithmic bytes and the kernel is bound by instruction issue and load
// latency, so both phases are branch-free and every load that does not
// depend on another is issued together (three round trips per chunk: the
// 16-B chunk descriptor {e0, e1, r0, r1}; val run + row_ptr + segment table;
// xg/perm):
//   scan     the chunk's S segment lengths are prefix-summed (with a count of
//            non-empty segments packed in the high half), giving each
//            non-empty segment its rank, base_ne[rank] = segment start −
//            flat offset, and a bit at its flat offset in sbm (M bits).
//   phase A  flat position f of the segment concatenation lies in the
//            non-empty segment of rank popcount(sbm bits ≤ f) − 1: one wave
//            prefix-scan of the 64 sbm words gives each 64-position batch its
//            base rank, mbcnt gives the lane's; src = base_ne[rank] + f, and
//            xs[perm[src]] = xg[src].  Wave w owns batches [16w, 16w+16).
//   phase B  thread t owns the run [16t, 16t+16); a bitmap of row starts
//            (ds_or) drives a segmented scan (reset at a start, add), whose
//            running value rounded to T is written back in place: a row that
//            ends inside a run leaves its value at its last position.  Pieces
//            of rows crossing runs (hp: before the run's first start, tp:
//            after its last) are combined in run order, and the owned rows'
//            y is stored coalesced from their last positions.
// xs lives in LDS at pidx(i) = i + i/16 (thread t's run at [17t, 17t+16):
// conflict-free).  Dynamic LDS: xs[M+M/16] T, hp[256] f64, tp[256] f64,
// bm[M/32] u32, sbm[M/32] u32, rpl[Rmax+1] i32, base_ne[S] i32, wsum[4] i32.
#ifndef LHPC_XT_RBLK32
#define LHPC_XT_RBLK32 512
#endif
#ifndef LHPC_XT_RBLK64
#define LHPC_XT_RBLK64 1024
#endif
// reduce configurations: BLK threads, each owning one 64-B run of RUN =
// 64/sizeof(T) nonzeros (fp32 16, fp64 8); chunks of M = RUN·BLK nonzeros
// owning ≤ Rmax rows.  A 64-B run keeps LDS per wave at 4 KB for both types,
// so LDS never caps occupancy below 8 waves per SIMD.  fp32: BLK = 512 (C2
// reduce: 256 → 512 took 470 → 420 µs, 1024 was no faster).  fp64 with
// 16-nonzero runs held 8 KB per wave (73 KB per 512-thread block: 2 blocks,
// 16 waves per CU; C3 reduce 987 µs).
template <typename T> constexpr int xt_run() { return 64 / static_cast<int>(sizeof(T)); }
template <typename T, int BLK> struct XtRed {
  static constexpr int M = BLK * xt_run<T>(), Rmax = M / 8;
};
template <typename T> constexpr int xt_red_blk() { return sizeof(T) == 4 ? LHPC_XT_RBLK32 : LHPC_XT_RBLK64; }
// LDS slot of chunk position i for the seg reduce (lhpc_plan.hpp xtile_slot):
// run t = i/RUN occupies 64 B at 64·t and its 16-B slot q is stored at
// q ^ xt_swz(t), so the 16 lanes of a ds_read_b128 group hit 16 distinct
// bank quads (4 runs per 256-B bank row, swizzled by the row's index mod 4)
__device__ __forceinline__ int xt_swz(int t) { return (t >> 2) & 3; }
template <typename T> __device__ __forceinline__ int xt_slot(int i) {
  constexpr int VW = 16 / sizeof(T), RUN = xt_run<T>();
  return (i & ~(RUN - 1)) | ((((i & (RUN - 1)) / VW) ^ xt_swz(i / RUN)) * VW) | (i & (VW - 1));
}
__device__ __forceinline__ int xt_pidx(int i) { return i + (i >> 4); }

#ifndef LHPC_XT_IP_LATE
#define LHPC_XT_IP_LATE 1  // iperm loaded after phase A's xg loads are issued (not live during the rank math)
#endif
#ifndef LHPC_XT_IP_DMA
#define LHPC_XT_IP_DMA 1  // iperm reduce, fp32: xg → LDS by global_load_lds (no VGPRs)
#endif
#ifndef LHPC_XT_IP_WAVES
#define LHPC_XT_IP_WAVES 8  // iperm reduce: 8 waves/SIMD (fp32 66 → 64 VGPRs + 8 B spill: C2 593 → 580 µs)
#endif
template <typename T, int G, int BLK, int P>
__global__ __launch_bounds__(BLK, P == 3 ? LHPC_XT_IP_WAVES : 1) void k_xtile_reduce(
    const int32_t *__restrict__ cdesc, const int32_t *__restrict__ segoff, int S, int64_t c0, int64_t C,
    int64_t Cx, int total, const T *__restrict__ xg, const uint16_t *__restrict__ perm,
    const T *__restrict__ val, const int32_t *__restrict__ rp, T *__restrict__ y,
    double *__restrict__ carry) {
  constexpr int RUN = xt_run<T>(), M = XtRed<T, BLK>::M, RMAX = XtRed<T, BLK>::Rmax;
  constexpr int RPT = (RMAX + 1 + BLK - 1) / BLK;  // row_ptr loads per thread
  constexpr int NB = M / BLK;                      // 64-position batches per wave (= RUN)
  // P positions per lane in phase A (segments padded to multiples of P, so a
  // lane's P positions are one aligned vector of xg and of perm): NBP
  // batches of 64 lanes per wave, M/P bits in the segment-start bitmap
  // P = 3 (iperm mode): one position per lane; phase A stores xg in flat
  // (segment concatenation) order and phase B gathers each CSR position's x
  // through iperm (CSR order, read with val) instead of scattering by perm
  constexpr bool IP = P == 3;
  constexpr int PP = IP ? 1 : P;
  constexpr int NBP = NB / PP;
  static_assert((NB == 16 || NB == 8) && (PP == 1 || PP == 2) && M / PP <= 256 * kWave && M >= 4096,
                "8/16 batches per wave; ≤ 256 batches per chunk; sbm ≥ 128 words");
  typedef T tvec __attribute__((ext_vector_type(16 / sizeof(T)), aligned(sizeof(T))));
  constexpr int VW = 16 / sizeof(T), NV = RUN / VW;
  // dynamic LDS (xtile_lds_bytes): xs[M + VW] T (xt_slot layout; slot M is
  // the sentinel's spare), bt[BLK/64][NB] u32x4, ws[BLK/64] f64,
  // wsf[BLK/64] i32, bm[M/32] u32, sbm[M/32] u32, rpl[RMAX+1] u16 (padded to
  // 4 B), base_ne[S] i32, wsum[8] i32
  extern __shared__ __align__(16) unsigned char smem[];
  T *xs = reinterpret_cast<T *>(smem);
  u32x4 *bt0 = reinterpret_cast<u32x4 *>(xs + M + VW);
  double *ws = reinterpret_cast<double *>(bt0 + (BLK / kWave) * NB);  // per-wave segmented-scan totals
  int *wsf = reinterpret_cast<int *>(ws + BLK / kWave);
  uint32_t *bm = reinterpret_cast<uint32_t *>(wsf + BLK / kWave);
  uint32_t *sbm = bm + M / 32;
  uint16_t *rpl = reinterpret_cast<uint16_t *>(sbm + M / 32);
  int32_t *base_ne = reinterpret_cast<int32_t *>(rpl + ((RMAX + 2) & ~1));
  int32_t *wsum = base_ne + S;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int wv = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int i0 = tid * RUN;
  const int64_t c = c0 + static_cast<int64_t>(blockIdx.x % 8) * Cx + blockIdx.x / 8;  // chunk range [c0, C)
  if (c >= C) return;  // block-uniform
  // ---- round trip 1: the chunk descriptor and the segment table (both
  //      addressed by c alone), then — without waiting for them — round
  //      trip 2 (val run and row_ptr, addressed by the descriptor).  The
  //      segment scan and phase A need only the table, so phase A's xg/perm
  //      loads go out while val and row_ptr are still in flight.
  int sa[G], sb[G];
#pragma unroll
  for (int q = 0; q < G; ++q) {
    const int sI = tid * G + q;
    const int sc = sI < S ? sI : S - 1;
    sa[q] = segoff[c * S + sc];
    sb[q] = segoff[(c + 1) * S + sc];
  }
  const u32x4 d = *reinterpret_cast<const u32x4 *>(cdesc + 4 * c);
  const int e0 = static_cast<int>(d[0]), m = static_cast<int>(d[1]) - e0;
  const int r0 = static_cast<int>(d[2]), R = static_cast<int>(d[3]) - r0;
  tvec vv[NV];
  {
    // the val allocation is padded by one run, so a run may read past nnz
    const tvec *vp = reinterpret_cast<const tvec *>(val + e0 + (i0 < m ? i0 : 0));
#pragma unroll
    for (int q = 0; q < NV; ++q) vv[q] = __builtin_nontemporal_load(vp + q);
  }
  constexpr int NIP = IP ? RUN * 2 / 16 : 1;  // 16-B iperm vectors per run
  u32x4 ipv[NIP];
  // perm points at iperm ([chunk][M] u16, CSR order); loaded with phase A's
  // xg round trip (LHPC_XT_IP_LATE) or here with val
  auto load_ipv = [&]() {
    const u32x4 *ip = reinterpret_cast<const u32x4 *>(perm + c * M + i0);
#pragma unroll
    for (int q = 0; q < NIP; ++q) ipv[q] = __builtin_nontemporal_load(ip + q);
  };
  if constexpr (IP && !LHPC_XT_IP_LATE) load_ipv();
  int rv[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int j = q * BLK + tid;
    rv[q] = rp[r0 + (j <= R ? j : R)];
  }
  // ---- scan: segment ranks / bases and the segment-start bitmap
  if (tid < M / 32) {
    bm[tid] = 0u;
    sbm[tid] = 0u;
  }
  int lsum = 0;  // (length | non-empty count << 16) of this thread's segments
#pragma unroll
  for (int q = 0; q < G; ++q) {
    if (tid * G + q >= S) sb[q] = sa[q];
    lsum += (sb[q] - sa[q]) + (sb[q] > sa[q] ? 0x10000 : 0);
  }
  const int inc = wave_incl_scan(lsum);
  if (lane == kWave - 1) wsum[wv] = inc;
  __syncthreads();
  int mf = m;  // flat length of the chunk's (padded) segments
  if constexpr (PP > 1) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < BLK / kWave; ++w) tot += wsum[w];
    mf = tot & 0xFFFF;
  }
  {
    int run = inc - lsum;
    for (int w = 0; w < wv; ++w) run += wsum[w];
    int off = run & 0xFFFF, rank = run >> 16;
#pragma unroll
    for (int q = 0; q < G; ++q) {
      const int len = sb[q] - sa[q];
      if (len > 0) {
        base_ne[rank] = sa[q] - off;
        atomicOr(sbm + ((off / PP) >> 5), 1u << ((off / PP) & 31));
        ++rank;
      }
      off += len;
    }
  }
  __syncthreads();

  // ---- phase A: src = base_ne[rank] + f, loads of xg/perm (round trip 3);
  //      positions past mf load the sentinel entry `total` (perm: spare slot M)
  int src[NBP];
  {
    // lane q holds batch q's word (a batch = 64 lanes × P positions); its
    // wave-uniform rank terms (w >> 1, base) go to an LDS triple that the
    // owning wave reads back as a broadcast:
    //   rank = starts before the batch − 1 + (w & 1) + mbcnt(w >> 1)
    // lane q holds batch words q (and q + 64 … when M/P > 4096); wave w owns
    // batches [NBP·w, NBP·w + NBP)
    const int grp = (wv * NBP) >> 6;  // this wave's batches lie in 64-batch group grp
    uint64_t wl = 0;
    int cnt = 0, incl = 0, below = 0;
    for (int g2 = 0; g2 <= grp; ++g2) {  // wave-uniform
      wl = static_cast<uint64_t>(sbm[128 * g2 + 2 * lane]) | (static_cast<uint64_t>(sbm[128 * g2 + 2 * lane + 1]) << 32);
      cnt = __popcll(wl);
      incl = wave_incl_scan(cnt) + below;  // starts in batches ≤ 64·g2 + lane
      below = __builtin_amdgcn_readlane(incl, kWave - 1);
    }
    u32x4 *bt = bt0 + wv * NB;
    if (lane / NBP == wv % (kWave / NBP)) {  // lanes holding this wave's batches
      const uint64_t w1 = wl >> 1;
      bt[lane & (NBP - 1)] = u32x4{static_cast<uint32_t>(w1), static_cast<uint32_t>(w1 >> 32),
                                   static_cast<uint32_t>(incl - cnt - 1 + static_cast<int>(wl & 1u)), 0u};
    }
    __builtin_amdgcn_wave_barrier();  // LDS is in order within a wave: no block barrier needed
#pragma unroll
    for (int u = 0; u < NBP; ++u) {
      const u32x4 t = bt[u];  // uniform address: broadcast
      const int rk = __builtin_amdgcn_mbcnt_hi(t[1], __builtin_amdgcn_mbcnt_lo(t[0], t[2]));
      const int f = ((wv * NBP + u) * kWave + lane) * PP;
      const int sv = base_ne[rk] + f;  // mf > 0 ⇒ 0 ≤ rk < S; mf = 0: base_ne[−1] (in LDS), unused
      src[u] = f < mf ? sv : total;
    }
  }
  // plain loads: the segment lines a neighbouring chunk shares must stay in
  // L2 (non-temporal xg/perm loads: 433 → 555 µs)
  if constexpr (IP) {
    // flat order: lane-linear LDS stores (no perm loads, no scatter)
#if LHPC_XT_IP_DMA
    if constexpr (sizeof(T) == 4) {
      // LDS-DMA: each lane's xg element lands at the batch's base + 4·lane
      // (exactly the flat order), no VGPR destination; drained by the
      // vmcnt(0) before the barrier below
#pragma unroll
      for (int u = 0; u < NBP; ++u)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(xg + src[u]),
                                         (__attribute__((address_space(3))) void *)(xs + (wv * NBP + u) * kWave),
                                         4, 0, 0);
      if constexpr (LHPC_XT_IP_LATE) load_ipv();
    } else
#endif
    {
      T xv[NBP];
#pragma unroll
      for (int u = 0; u < NBP; ++u) xv[u] = xg[src[u]];
#pragma unroll
      for (int u = 0; u < NBP; ++u) xs[(wv * NBP + u) * kWave + lane] = xv[u];
      if constexpr (LHPC_XT_IP_LATE) load_ipv();
    }
  } else if constexpr (P == 1) {
    T xv[NBP];
    uint16_t pv[NBP];
#pragma unroll
    for (int u = 0; u < NBP; ++u) {
      xv[u] = xg[src[u]];
      pv[u] = perm[src[u]];  // LDS slot xt_slot(position); the sentinel's: M
    }
#pragma unroll
    for (int u = 0; u < NBP; ++u) xs[pv[u]] = xv[u];
  } else {
    // one 2·sizeof(T) xg load and one 4-B perm load per lane and batch
    typedef T t2 __attribute__((ext_vector_type(2)));
    t2 xv[NBP];
    uint32_t pv[NBP];
#pragma unroll
    for (int u = 0; u < NBP; ++u) {
      xv[u] = *reinterpret_cast<const t2 *>(xg + src[u]);
      pv[u] = *reinterpret_cast<const uint32_t *>(perm + src[u]);
    }
#pragma unroll
    for (int u = 0; u < NBP; ++u) {
      xs[pv[u] & 0xFFFFu] = xv[u][0];
      xs[pv[u] >> 16] = xv[u][1];
    }
  }
  // row_ptr (round trip 2) → local row offsets and the row-start bitmap
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int j = q * BLK + tid;
    rv[q] -= e0;
    if (j <= R) rpl[j] = static_cast<uint16_t>(rv[q] <= m ? rv[q] : m + 1);  // > m: continues
    if (j < R && rv[q] < m) atomicOr(bm + (rv[q] >> 5), 1u << (rv[q] & 31));  // empty rows share a bit
  }
  const int n = m - i0 < RUN ? (m - i0 > 0 ? m - i0 : 0) : RUN;  // valid entries in the run
  if (n < RUN) {  // the chunk's last run (and runs past m): val and x past m → 0 · 0
    if constexpr (!IP)
      for (int j = n; j < RUN; ++j) xs[xt_slot<T>(i0 + j)] = T(0);
#pragma unroll
    for (int j = 0; j < RUN; ++j) vv[j / VW][j % VW] = j < n ? vv[j / VW][j % VW] : T(0);
  }
  __syncthreads();

  // ---- phase B: branch-free segmented scan of the thread's run.  The fp32
  //      product is exact in fp64, so the fma equals the add of the product.
  const uint32_t mask = (bm[i0 >> 5] >> (i0 & 31)) & ((1u << RUN) - 1u);
  const int hl = mask ? __builtin_ctz(mask) : RUN;  // head length (entries before the first start)
  const int hend = (hl < n ? hl : n) - 1;                // last head position (−1: none)
  // the run is NV 16-B slots at RUN·tid, slot q stored at q ^ xt_swz (conflict-free ds_read_b128)
  typedef T lvec __attribute__((ext_vector_type(VW)));
  lvec *xr = reinterpret_cast<lvec *>(xs + i0);
  const int swz = xt_swz(tid);
  lvec xq[NV];
  if constexpr (IP) {
    // gather the run's x from the flat array, then (after every thread has
    // read) the running sums below go back in the CSR (xt_slot) layout
    // unconditional reads (iperm past m is 0, a valid slot), so all RUN
    // ds_reads issue before the first wait; then x past m → 0
    T gx[RUN];
#pragma unroll
    for (int j = 0; j < RUN; ++j) {
      const uint32_t w = ipv[j / 8][(j % 8) / 2];
      gx[j] = xs[static_cast<int>((j & 1) ? (w >> 16) : (w & 0xFFFFu))];
    }
#pragma unroll
    for (int j = 0; j < RUN; ++j) xq[j / VW][j % VW] = j < n ? gx[j] : T(0);
    __syncthreads();
  } else {
#pragma unroll
    for (int q = 0; q < NV; ++q) xq[q] = xr[q ^ swz];
  }
  double acc = 0.0, hsave = 0.0;
#pragma unroll
  for (int j = 0; j < RUN; ++j) {
    acc = ((mask >> j) & 1u) ? 0.0 : acc;
    acc = __builtin_fma(static_cast<double>(vv[j / VW][j % VW]), static_cast<double>(xq[j / VW][j % VW]), acc);
    hsave = j == hend ? acc : hsave;
    xq[j / VW][j % VW] = static_cast<T>(acc);  // in place; slots past m are never read
  }
#pragma unroll
  for (int q = 0; q < NV; ++q) xr[q ^ swz] = xq[q];
  const bool has_head = n > 0 && !(mask & 1u);
  const bool cont = rpl[R] > m;  // the row active at m−1 runs past the chunk
  // ---- rows that cross runs: segmented scan over threads (run order) of
  //      x(t) = tail piece if run t holds a row start, else its whole-run sum;
  //      the row open when run t begins is the exclusive value S(t−1)
  bool fl = n > 0 && mask != 0u;
  double sv = wave_seg_scan(fl ? acc : hsave, fl);
  if (lane == kWave - 1) {
    ws[wv] = sv;
    wsf[wv] = fl ? 1 : 0;
  }
  __syncthreads();
  double cw = 0.0;  // segmented carry of the waves before this one
  int gw = 0;
  for (int w = 0; w < wv; ++w) {
    cw = wsf[w] ? ws[w] : cw + ws[w];
    gw |= wsf[w];
  }
  if (!fl) sv = cw + sv;
  const int fin_incl = (fl ? 1 : 0) | gw;
  constexpr int kShr1 = 0x138;  // DPP wave_shr:1 (lane l ← lane l−1; lane 0 keeps `old`)
  const double oin = dpp_f64_old<kShr1>(cw, sv);                                 // S(t−1)
  const int fin = __builtin_amdgcn_update_dpp(gw, fin_incl, kShr1, 0xF, 0xF, false);  // starts before run t
  const int tlast = m > 0 ? (m - 1) / RUN : -1;
  if (tid == 0 && !(m > 0 && rpl[0] > 0)) carry[2 * c] = 0.0;  // no head piece
  if (has_head) {
    const int i1 = i0 + n;
    const bool end_i1 = i1 < m ? ((bm[i1 >> 5] >> (i1 & 31)) & 1u) != 0 : !cont;
    const bool ends = hl < n || end_i1;
    if (ends || tid == tlast) {
      const double sum = oin + hsave;
      if (!fin) {
        carry[2 * c] = sum;  // this chunk's piece of the previous chunk's row
      } else if (ends) {
        xs[xt_slot<T>(i0 + hend)] = static_cast<T>(sum);
      } else {
        carry[2 * c + 1] = sum;  // row continues into the next chunk
      }
    }
  }
  if (tid == tlast && mask && cont) carry[2 * c + 1] = acc;  // own tail row continues
  __syncthreads();
  // coalesced y store of the owned rows from their last positions (a row
  // continuing past the chunk is stored by k_xtile_fixup, later on the stream)
  for (int j = tid; j < R; j += BLK) {
    const int a0 = rpl[j], a1 = rpl[j + 1];
    if (a1 == a0) y[r0 + j] = T(0);
    else if (a1 <= m) y[r0 + j] = xs[xt_slot<T>(a1 - 1)];
  }
}

// rows cut by a chunk end: y[row] = tail piece + head pieces, chunk order
template <typename T>
__global__ __launch_bounds__(kXtBlock) void k_xtile_fixup(
    const int32_t *__restrict__ cont, int64_t n_cont, const int32_t *__restrict__ cr, int64_t C,
    const double *__restrict__ carry, T *__restrict__ y) {  // C: end of the chunk range (rows never cross it)
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kXtBlock + threadIdx.x;
  if (i >= n_cont) return;
  const int64_t c = cont[i];
  double s = carry[2 * c + 1];
  for (int64_t d = c + 1; d < C; ++d) {
    s += carry[2 * d];
    if (cr[d + 1] > cr[d]) break;
  }
  y[cr[c + 1] - 1] = static_cast<T>(s);
}

// ------------------------------------------------- XTILE, chunk-major xg
// (layout: lhpc_plan.hpp XtileHost::cm)
// gather: block b streams pieces[3b..3b+1] of tile pieces[3b+2] (idle when
// empty).  Per thread and step: one 16-B col16 load (a group of 8 entries of
// one segment, padding 0xFFFF at its end) and the group's xg position, 8 LDS
// gathers, and 8 contiguous xg stores — two unaligned 16-B stores for a full
// group (fp32), per-entry stores for a segment's last group.
template <typename T, int U>
__global__ __launch_bounds__(kXtGatherBlock) void k_xtile_gather_cm(
    const int32_t *__restrict__ pieces, const uint16_t *__restrict__ col16,
    const int32_t *__restrict__ gdst, const T *__restrict__ x, int64_t n_cols, T *__restrict__ xg) {
  constexpr int W = XtTile<T>::W;
  __shared__ T xt[W];
  const int tid = threadIdx.x;
  const int g0 = pieces[3 * blockIdx.x], g1 = pieces[3 * blockIdx.x + 1];
  if (g0 == g1) return;  // block-uniform: no entries of this tile in this chunk range
  const int64_t c0 = static_cast<int64_t>(pieces[3 * blockIdx.x + 2]) * W;
  const int wlen = static_cast<int>((n_cols - c0) < W ? (n_cols - c0) : W);
  constexpr int PT = W / kXtGatherBlock;
  T tv[PT];
#pragma unroll
  for (int i = 0; i < PT; ++i) {
    const int j = i * kXtGatherBlock + tid;
    tv[i] = j < wlen ? x[c0 + j] : T(0);
  }
#pragma unroll
  for (int i = 0; i < PT; ++i) xt[i * kXtGatherBlock + tid] = tv[i];
  __syncthreads();
  typedef T tvec4u __attribute__((ext_vector_type(16 / sizeof(T)), aligned(sizeof(T))));
  constexpr int VW = 16 / sizeof(T);
  const int q0 = g0 >> 3, q1 = g1 >> 3;  // 8-entry groups
  const u32x4 *cv = reinterpret_cast<const u32x4 *>(col16);
  for (int q = q0 + tid; q < q1; q += U * kXtGatherBlock) {
    u32x4 w[U];
    int dst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q + u * kXtGatherBlock;
      const int qc = qq < q1 ? qq : q0;  // clamped: the loads stay unconditional
      w[u] = __builtin_nontemporal_load(cv + qc);
      dst[u] = __builtin_nontemporal_load(gdst + qc);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int qq = q + u * kXtGatherBlock;
      T o[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const uint32_t lo = w[u][h] & 0xFFFFu, hi = w[u][h] >> 16;
        o[2 * h] = xt[lo < static_cast<uint32_t>(W) ? lo : 0u];
        o[2 * h + 1] = xt[hi < static_cast<uint32_t>(W) ? hi : 0u];
      }
      if (qq < q1) {
        T *d = xg + dst[u];
        if ((w[u][3] >> 16) != 0xFFFFu) {  // full group
#pragma unroll
          for (int v = 0; v < 8 / VW; ++v) {
            tvec4u t;
#pragma unroll
            for (int e = 0; e < VW; ++e) t[e] = o[v * VW + e];
            *reinterpret_cast<tvec4u *>(d + v * VW) = t;
          }
        } else {
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            if ((w[u][h] & 0xFFFFu) != 0xFFFFu) d[2 * h] = o[2 * h];
            if ((w[u][h] >> 16) != 0xFFFFu) d[2 * h + 1] = o[2 * h + 1];
          }
        }
      }
    }
  }
}

// reduce over chunk-major xg: block per chunk (XCD-blocked as k_xtile_reduce).
// Thread t loads its run [16t, 16t+16) of the chunk's val, xg and perm (all
// contiguous), scatters xs[perm] = xg, and phase B / the run combine / the y
// store are those of k_xtile_reduce.  Two round trips per chunk: the 16-B
// descriptor, then every other load.  LDS: xs[M+M/16] T, hp[256] f64,
// tp[256] f64, bm[M/32] u32, rpl[Rmax+1] i32 (static).
template <typename T>
__global__ __launch_bounds__(kXtBlock) void k_xtile_reduce_cm(
    const int32_t *__restrict__ cdesc, int64_t C, int64_t Cx, const T *__restrict__ xg,
    const uint16_t *__restrict__ perm, const T *__restrict__ val, const int32_t *__restrict__ rp,
    T *__restrict__ y, double *__restrict__ carry) {
  constexpr int MP = kXtM + kXtM / 16;
  constexpr int RPT = (kXtRmax + 1 + kXtBlock - 1) / kXtBlock;
  typedef T tvec __attribute__((ext_vector_type(16 / sizeof(T)), aligned(sizeof(T))));
  typedef uint16_t pvec __attribute__((ext_vector_type(8), aligned(2)));
  constexpr int VW = 16 / sizeof(T), NV = kXtRun / VW;
  __shared__ T xs[MP];
  __shared__ double hp[kXtBlock], tp[kXtBlock];
  __shared__ uint32_t bm[kXtM / 32];
  __shared__ int32_t rpl[kXtRmax + 1];

  const int tid = threadIdx.x;
  const int i0 = tid * kXtRun;
  const int64_t c = static_cast<int64_t>(blockIdx.x % 8) * Cx + blockIdx.x / 8;
  if (c >= C) return;  // block-uniform
  const u32x4 d = *reinterpret_cast<const u32x4 *>(cdesc + 4 * c);
  const int e0 = static_cast<int>(d[0]), m = static_cast<int>(d[1]) - e0;
  const int r0 = static_cast<int>(d[2]), R = static_cast<int>(d[3]) - r0;

  // ---- round trip 2: val / xg / perm runs and row_ptr (unconditional loads;
  //      the val, xg and perm allocations are padded by one run)
  const int64_t rb = static_cast<int64_t>(e0) + (i0 < m ? i0 : 0);
  tvec vv[NV], xv[NV];
  pvec pv[kXtRun / 8];
  {
    const tvec *vp = reinterpret_cast<const tvec *>(val + rb);
    const tvec *xp = reinterpret_cast<const tvec *>(xg + rb);
    const pvec *pp = reinterpret_cast<const pvec *>(perm + rb);
#pragma unroll
    for (int q = 0; q < NV; ++q) vv[q] = __builtin_nontemporal_load(vp + q);
#pragma unroll
    for (int q = 0; q < NV; ++q) xv[q] = __builtin_nontemporal_load(xp + q);
#pragma unroll
    for (int q = 0; q < kXtRun / 8; ++q) pv[q] = pp[q];
  }
  int rv[RPT];
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int j = q * kXtBlock + tid;
    rv[q] = rp[r0 + (j <= R ? j : R)] - e0;
  }
  if (tid < kXtM / 32) bm[tid] = 0u;
#pragma unroll
  for (int q = 0; q < RPT; ++q) {
    const int j = q * kXtBlock + tid;
    if (j <= R) rpl[j] = rv[q];
  }
  const int n = m - i0 < kXtRun ? (m - i0 > 0 ? m - i0 : 0) : kXtRun;  // valid entries in the run
#pragma unroll
  for (int j = 0; j < kXtRun; ++j)  // entries past m go to the spare slot MP−1 (never read)
    xs[j < n ? xt_pidx(pv[j / 8][j % 8]) : MP - 1] = xv[j / VW][j % VW];
  __syncthreads();  // bm zeroed before the ds_or below
#pragma unroll
  for (int q = 0; q < RPT; ++q) {  // row starts inside the chunk (empty rows share a bit)
    const int j = q * kXtBlock + tid;
    if (j < R && rv[q] < m) atomicOr(bm + (rv[q] >> 5), 1u << (rv[q] & 31));
  }
  __syncthreads();

  // ---- phase B: branch-free segmented scan of the thread's run
  const uint32_t mask = (bm[tid >> 1] >> ((tid & 1) * 16)) & 0xFFFFu;
  const int hl = mask ? __builtin_ctz(mask) : kXtRun;
  const int hend = (hl < n ? hl : n) - 1;
  double acc = 0.0, hsave = 0.0;
#pragma unroll
  for (int j = 0; j < kXtRun; ++j) {
    const double pr = static_cast<double>(vv[j / VW][j % VW]) * static_cast<double>(xs[17 * tid + j]);
    const double pj = j < n ? pr : 0.0;
    acc = ((mask >> j) & 1u) ? 0.0 : acc;
    acc += pj;
    hsave = j == hend ? acc : hsave;
    xs[17 * tid + j] = static_cast<T>(acc);
  }
  const bool has_head = n > 0 && !(mask & 1u);
  if (has_head) hp[tid] = hsave;
  if (n > 0 && mask) tp[tid] = acc;
  const bool cont = rpl[R] > m;
  __syncthreads();
  const int tlast = m > 0 ? (m - 1) / kXtRun : -1;
  if (tid == 0 && !(m > 0 && rpl[0] > 0)) carry[2 * c] = 0.0;
  if (has_head) {
    const int i1 = i0 + n;
    const bool end_i1 = i1 < m ? ((bm[i1 >> 5] >> (i1 & 31)) & 1u) != 0 : !cont;
    const bool ends = hl < n || end_i1;
    if (ends || tid == tlast) {
      int u = tid - 1;
      while (u >= 0 && ((bm[u >> 1] >> ((u & 1) * 16)) & 0xFFFFu) == 0u) --u;
      double sum = u >= 0 ? tp[u] : 0.0;
      for (int v = u + 1; v <= tid; ++v) sum += hp[v];
      if (u < 0) {
        carry[2 * c] = sum;
      } else if (ends) {
        xs[xt_pidx(i0 + hend)] = static_cast<T>(sum);
      } else {
        carry[2 * c + 1] = sum;
      }
    }
  }
  if (tid == tlast && mask && cont) carry[2 * c + 1] = tp[tid];
  __syncthreads();
  for (int j = tid; j < R; j += kXtBlock) {
    const int a0 = rpl[j], a1 = rpl[j + 1];
    if (a1 == a0) y[r0 + j] = T(0);
    else if (a1 <= m) y[r0 + j] = xs[xt_pidx(a1 - 1)];
  }
}

// ------------------------------------------------------------- host side
// Distinct 128-B x lines touched per nonzero, over up to 32 evenly spaced
// chunks of 8192 consecutive rows (1.0 = no reuse within a chunk).
template <typename RP>
double gather_lines_per_nnz(const RP &rp, const int32_t *col, int64_t n_rows, size_t tsz) {
  constexpr int64_t kChunk = 8192, kSamples = 32;
  const int shift = tsz == 8 ? 4 : 5;  // 16 doubles / 32 floats per line
  const int64_t chunks = (n_rows + kChunk - 1) / kChunk;
  const int64_t step = std::max<int64_t>(1, chunks / kSamples);
  int64_t lines = 0, nz = 0;
  std::vector<int32_t> buf;
  for (int64_t c = 0; c < chunks; c += step) {
    const int64_t r0 = c * kChunk, r1 = std::min(n_rows, r0 + kChunk);
    const int64_t k0 = rp[r0], k1 = rp[r1];
    buf.resize(static_cast<size_t>(k1 - k0));
    for (int64_t k = k0; k < k1; ++k) buf[static_cast<size_t>(k - k0)] = col[k] >> shift;
    std::sort(buf.begin(), buf.end());
    lines += std::unique(buf.begin(), buf.end()) - buf.begin();
    nz += k1 - k0;
  }
  return nz ? static_cast<double>(lines) / static_cast<double>(nz) : 1.0;
}

bool is_gfx950(int dev) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
  return std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

}  // namespace
}  // namespace lhpc

using namespace lhpc;

struct lhpc_spmv_plan {
  int dtype = LHPC_F32;
  int device = 0;
  int rp64 = 0;  // device row_ptr is int64
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  void *d_row_ptr = nullptr;
  int32_t *d_col = nullptr;
  void *d_val = nullptr;
  int64_t *d_blocks = nullptr;
  int64_t n_blocks = 0, n_long = 0;
  void *d_xstage = nullptr, *d_ystage = nullptr;
  double *d_dpart = nullptr;  // lhpc_spmv_dot: per-block partials (ADAPTIVE), allocated on first use
  int kernel = LHPC_KERNEL_ROWGROUP;
  int L = 16, R = 4;
  int64_t bytes = 0;
  // XSLICE
  int S = 0;
  int xs_jagged = 0, xs_nb = 2, xs_p64 = 0, xs_lens16 = 0, xs_fused = 0;
  int xs_persist = 0, xs_grid = 0, xs_g = 8;  // persistent partial-free kernel: grid, chunks/wave/pass
  unsigned *d_arrive = nullptr;  // XSLICE fused: arrival counter per 256-row block
  int64_t xs_width = 0, xs_chunks = 0, xs_rows_pad = 0, xs_bps = 0;
  void *d_lens = nullptr;
  int64_t *d_cbase = nullptr;
  void *d_partial = nullptr;
  // XTILE
  int64_t xt_C = 0, xt_pieces = 0, xt_cont = 0, xt_total = 0;
  size_t xt_lds = 0;
  int xt_u = 8;  // gather steps in flight (LHPC_XTILE_U; the chunk-major gather caps it at 4)
  // pipelined seg calls: K chunk ranges; range k's gather runs on the caller's
  // stream, its reduce on xt_s2 once the gather's event fires, so range k's
  // reduce overlaps range k+1's gather
  int xt_K = 1;
  // row ranges (lhpc_spmv_plan_create_split): range k = rows [xt_srow[k],
  // xt_srow[k+1]) = chunks [xt_src[k], xt_src[k+1]), cont entries [xt_sco[k], xt_sco[k+1])
  std::vector<int64_t> split_rows, xt_srow, xt_src, xt_sco;
  std::vector<int64_t> xt_rc;           // [K+1] chunk bounds
  std::vector<int64_t> xt_rpo;          // [K+1] offsets (in pieces) of each range's gather pieces
  int32_t *d_rpieces = nullptr;
  hipStream_t xt_s2 = nullptr;
  std::vector<hipEvent_t> xt_ev;        // [K+1]
  int32_t *d_cdesc = nullptr;
  int32_t *d_ce = nullptr, *d_cr = nullptr, *d_segoff = nullptr, *d_pieces = nullptr, *d_cont = nullptr;
  uint16_t *d_col16 = nullptr, *d_perm = nullptr;
  int xt_cm = 0;  // chunk-major xg (XtileHost::cm)
  int xt_p = 1;   // reduce phase A positions per lane (segments padded to multiples of xt_p)
  int32_t *d_gdst = nullptr;
  void *d_xg = nullptr;
  double *d_carry = nullptr;
};

namespace {

int dmalloc(void **p, size_t n, int64_t &acct) {
  if (n == 0) n = 16;
  hipError_t e = hipMalloc(p, n);
  if (e == hipErrorOutOfMemory) return LHPC_ERR_ALLOC;
  if (e != hipSuccess) return static_cast<int>(e);
  acct += static_cast<int64_t>(n);
  return LHPC_OK;
}

template <typename T, typename I, int L, int R>
int launch_rowgroup_t(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  constexpr int WR = (kWave / L) * R;
  const int64_t waves = (p->n_rows + WR - 1) / WR;
  const int64_t blocks = (waves * kWave + kBlock - 1) / kBlock;
  if (blocks == 0) return LHPC_OK;
  hipLaunchKernelGGL((k_spmv_rowgroup<T, I, L, R>), dim3(static_cast<unsigned>(blocks)),
                     dim3(kBlock), 0, s, static_cast<const I *>(p->d_row_ptr), p->d_col,
                     static_cast<const T *>(p->d_val), static_cast<const T *>(x),
                     static_cast<T *>(y), p->n_rows);
  return check_launch(s);
}

template <typename T, typename I>
int launch_rowgroup(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  switch (p->L * 100 + p->R) {
    case 101: return launch_rowgroup_t<T, I, 1, 1>(p, x, y, s);
    case 201: return launch_rowgroup_t<T, I, 2, 1>(p, x, y, s);
    case 202: return launch_rowgroup_t<T, I, 2, 2>(p, x, y, s);
    case 401: return launch_rowgroup_t<T, I, 4, 1>(p, x, y, s);
    case 402: return launch_rowgroup_t<T, I, 4, 2>(p, x, y, s);
    case 404: return launch_rowgroup_t<T, I, 4, 4>(p, x, y, s);
    case 802: return launch_rowgroup_t<T, I, 8, 2>(p, x, y, s);
    case 804: return launch_rowgroup_t<T, I, 8, 4>(p, x, y, s);
    case 1601: return launch_rowgroup_t<T, I, 16, 1>(p, x, y, s);
    case 1602: return launch_rowgroup_t<T, I, 16, 2>(p, x, y, s);
    case 1604: return launch_rowgroup_t<T, I, 16, 4>(p, x, y, s);
    case 1608: return launch_rowgroup_t<T, I, 16, 8>(p, x, y, s);
    case 3201: return launch_rowgroup_t<T, I, 32, 1>(p, x, y, s);
    case 3202: return launch_rowgroup_t<T, I, 32, 2>(p, x, y, s);
    case 6401: return launch_rowgroup_t<T, I, 64, 1>(p, x, y, s);
    default: return LHPC_ERR_UNSUPPORTED;
  }
}

template <typename T, typename I>
int launch_adaptive(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s, const void *w = nullptr,
                    double *dpart = nullptr) {
  if (p->n_blocks == 0) return LHPC_OK;
  hipLaunchKernelGGL((k_spmv_adaptive<T, I>), dim3(static_cast<unsigned>(p->n_blocks)),
                     dim3(kBlock), 0, s, static_cast<const I *>(p->d_row_ptr), p->d_col,
                     static_cast<const T *>(p->d_val), static_cast<const T *>(x),
                     static_cast<T *>(y), p->d_blocks, static_cast<const T *>(w), dpart);
  return check_launch(s);
}

// Fixed-order two-stage sum of the per-block dot partials: stage 1 reduces
// 2048 consecutive partials per block (8 independent loads per thread), stage
// 2 (one block) the ≤ ⌈nb/2048⌉ stage-1 sums.  One block looping over ~10^5
// partials would serialise on L2 latency.
constexpr int kFinTile = 2048;
__global__ __launch_bounds__(kBlock) void k_dpart_finish(const double *__restrict__ part, int64_t nb,
                                                         double *__restrict__ out) {
  __shared__ double wsum[kBlock / kWave];
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) * kFinTile;
  double v[kFinTile / kBlock];
#pragma unroll
  for (int k = 0; k < kFinTile / kBlock; ++k) {
    const int64_t i = b0 + k * kBlock + threadIdx.x;
    v[k] = i < nb ? part[i] : 0.0;
  }
  double a = 0.0;
#pragma unroll
  for (int k = 0; k < kFinTile / kBlock; ++k) a += v[k];
  a = group_sum<kWave>(a);
  if ((threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = a;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = wsum[0];
#pragma unroll
    for (int i = 1; i < kBlock / kWave; ++i) t += wsum[i];
    out[blockIdx.x] = t;
  }
}

template <typename T>
int launch_xslice(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  if (p->n_rows == 0) return LHPC_OK;
  const int64_t grid = p->S >= 8 ? 8 * (p->S / 8) * p->xs_bps : p->S * p->xs_bps;
  const int64_t nnz_last = p->nnz > 0 ? p->nnz - 1 : 0;
  const dim3 g(static_cast<unsigned>(grid)), blk(kBlock);
  const T *xv = static_cast<const T *>(x);
  const T *vv = static_cast<const T *>(p->d_val);
  if (p->xs_persist) {
#define LHPC_XS_P(LT, NB, GG)                                                                      \
  hipLaunchKernelGGL((k_spmv_xslice_persist<T, LT, NB, GG>), dim3(static_cast<unsigned>(p->xs_grid)), blk, \
                     0, s, static_cast<const LT *>(p->d_lens), p->d_cbase, p->d_col, vv, xv,           \
                     static_cast<T *>(y), p->n_rows, p->xs_rows_pad, p->xs_chunks, p->S)
#define LHPC_XS_PG(LT, NB)                    \
  do {                                        \
    if (p->xs_g == 16) LHPC_XS_P(LT, NB, 16); \
    else if (p->xs_g == 4) LHPC_XS_P(LT, NB, 4); \
    else LHPC_XS_P(LT, NB, 8);                \
  } while (0)
    if (p->xs_lens16) {
      if (p->xs_nb <= 2) LHPC_XS_PG(uint16_t, 2); else LHPC_XS_PG(uint16_t, 4);
    } else {
      if (p->xs_nb <= 2) LHPC_XS_PG(uint8_t, 2); else LHPC_XS_PG(uint8_t, 4);
    }
#undef LHPC_XS_PG
#undef LHPC_XS_P
    return check_launch(s);
  }
  if (p->xs_fused) {
    // counters zeroed on the stream before every launch (Guideline 16: re-initialise every call)
    LHPC_HIP_TRY(hipMemsetAsync(p->d_arrive, 0, static_cast<size_t>((p->xs_bps + 3) / 4 * 16), s));
#define LHPC_XS_FUSED(LT, NB)                                                                      \
  hipLaunchKernelGGL((k_spmv_xslice_fused<T, LT, NB>), g, blk, 0, s, static_cast<const LT *>(p->d_lens), \
                     p->d_cbase, p->d_col, vv, xv, static_cast<double *>(p->d_partial), p->d_arrive,   \
                     static_cast<T *>(y), p->n_rows, p->xs_rows_pad, p->xs_chunks, p->xs_bps, p->S)
#define LHPC_XS_FUSED_NB(LT)                 \
  switch (p->xs_nb) {                        \
    case 1: LHPC_XS_FUSED(LT, 1); break;     \
    case 2: LHPC_XS_FUSED(LT, 2); break;     \
    case 3: LHPC_XS_FUSED(LT, 3); break;     \
    default: LHPC_XS_FUSED(LT, 4); break;    \
  }
    if (p->xs_lens16) {
      LHPC_XS_FUSED_NB(uint16_t)
    } else {
      LHPC_XS_FUSED_NB(uint8_t)
    }
#undef LHPC_XS_FUSED_NB
#undef LHPC_XS_FUSED
    return check_launch(s);
  }
  if (p->xs_jagged) {
    hipLaunchKernelGGL((k_spmv_xslice<T, 4>), g, blk, 0, s, static_cast<const uint8_t *>(p->d_lens), p->d_cbase, p->d_col, vv, xv,
                       static_cast<T *>(p->d_partial), p->n_rows, p->xs_rows_pad, p->xs_chunks,
                       p->xs_bps, p->S, nnz_last);
  } else {
#define LHPC_XS_STREAM(P, NB)                                                                        \
  if (p->xs_lens16)                                                                                  \
    hipLaunchKernelGGL((k_spmv_xslice_stream<T, P, uint16_t, NB>), g, blk, 0, s,                      \
                       static_cast<const uint16_t *>(p->d_lens), p->d_cbase, p->d_col, vv, xv,         \
                       static_cast<P *>(p->d_partial), p->n_rows, p->xs_rows_pad, p->xs_chunks,        \
                       p->xs_bps, p->S);                                                              \
  else                                                                                               \
    hipLaunchKernelGGL((k_spmv_xslice_stream<T, P, uint8_t, NB>), g, blk, 0, s,                       \
                       static_cast<const uint8_t *>(p->d_lens), p->d_cbase, p->d_col, vv, xv,          \
                       static_cast<P *>(p->d_partial), p->n_rows, p->xs_rows_pad, p->xs_chunks,        \
                       p->xs_bps, p->S)
#define LHPC_XS_NB(P)                     \
  switch (p->xs_nb) {                     \
    case 1: LHPC_XS_STREAM(P, 1); break;  \
    case 2: LHPC_XS_STREAM(P, 2); break;  \
    case 3: LHPC_XS_STREAM(P, 3); break;  \
    default: LHPC_XS_STREAM(P, 4); break; \
  }
    if (p->xs_p64) {
      LHPC_XS_NB(double)
    } else {
      LHPC_XS_NB(T)
    }
#undef LHPC_XS_NB
#undef LHPC_XS_STREAM
  }
  LHPC_TRY(check_launch(s));
  const int64_t rgrid = (p->n_rows + 4 * kBlock - 1) / (4 * kBlock);
  const dim3 rg(static_cast<unsigned>(rgrid));
  if (p->xs_p64 && !p->xs_jagged)
    hipLaunchKernelGGL((k_xslice_reduce<T, double>), rg, blk, 0, s, static_cast<const double *>(p->d_partial),
                       static_cast<T *>(y), p->n_rows, p->xs_rows_pad, p->S);
  else
    hipLaunchKernelGGL((k_xslice_reduce<T, T>), rg, blk, 0, s, static_cast<const T *>(p->d_partial),
                       static_cast<T *>(y), p->n_rows, p->xs_rows_pad, p->S);
  return check_launch(s);
}

template <typename T>
size_t xtile_lds_bytes(int S) {
  constexpr int BLK = xt_red_blk<T>(), M = XtRed<T, BLK>::M, RMAX = XtRed<T, BLK>::Rmax, W = BLK / kWave;
  return static_cast<size_t>(M + 16 / sizeof(T)) * sizeof(T) + W * xt_run<T>() * 16 + W * (sizeof(double) + 4) +
         2 * M / 32 * sizeof(uint32_t) + ((RMAX + 2) & ~1) * sizeof(uint16_t) +
         sizeof(int32_t) * (static_cast<size_t>(S) + 8);
}

template <typename T>
int xtile_g(int S) {
  const int g = (S + xt_red_blk<T>() - 1) / xt_red_blk<T>();
  return g <= 1 ? 1 : g <= 2 ? 2 : g <= 4 ? 4 : g <= 8 ? 8 : 16;
}

template <typename T, int G, int P>
const void *xtile_reduce_fn() { return reinterpret_cast<const void *>(k_xtile_reduce<T, G, xt_red_blk<T>(), P>); }
template <typename T, int P>
const void *xtile_reduce_fn(int g) {
  return g == 1 ? xtile_reduce_fn<T, 1, P>() : g == 2 ? xtile_reduce_fn<T, 2, P>() : g == 4 ? xtile_reduce_fn<T, 4, P>()
         : g == 8 ? xtile_reduce_fn<T, 8, P>() : xtile_reduce_fn<T, 16, P>();
}

template <typename T>
int launch_xtile(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  if (p->n_rows == 0) return LHPC_OK;
  T *xg = static_cast<T *>(p->d_xg);
  if (p->xt_cm) {
    if (p->xt_pieces > 0) {
      const dim3 g(static_cast<unsigned>(p->xt_pieces)), b(kXtGatherBlock);
      if (p->xt_u == 1)
        hipLaunchKernelGGL((k_xtile_gather_cm<T, 1>), g, b, 0, s, p->d_pieces, p->d_col16, p->d_gdst,
                           static_cast<const T *>(x), p->n_cols, xg);
      else if (p->xt_u == 2)
        hipLaunchKernelGGL((k_xtile_gather_cm<T, 2>), g, b, 0, s, p->d_pieces, p->d_col16, p->d_gdst,
                           static_cast<const T *>(x), p->n_cols, xg);
      else
        hipLaunchKernelGGL((k_xtile_gather_cm<T, 4>), g, b, 0, s, p->d_pieces, p->d_col16, p->d_gdst,
                           static_cast<const T *>(x), p->n_cols, xg);
      LHPC_TRY(check_launch(s));
    }
    const int64_t Cx = (p->xt_C + 7) / 8;
    hipLaunchKernelGGL((k_xtile_reduce_cm<T>), dim3(static_cast<unsigned>(8 * Cx)), dim3(kXtBlock), 0, s,
                       p->d_cdesc, p->xt_C, Cx, xg, p->d_perm, static_cast<const T *>(p->d_val),
                       static_cast<const int32_t *>(p->d_row_ptr), static_cast<T *>(y), p->d_carry);
    LHPC_TRY(check_launch(s));
  } else {
  auto gather = [&](const int32_t *pieces, int64_t n) -> int {
    if (n <= 0) return LHPC_OK;
    const dim3 g(static_cast<unsigned>(n)), b(kXtGatherBlock);
    if (p->xt_u == 2)
      hipLaunchKernelGGL((k_xtile_gather<T, 2>), g, b, 0, s, pieces, p->d_col16,
                         static_cast<const T *>(x), p->n_cols, xg);
    else if (p->xt_u == 16)
      hipLaunchKernelGGL((k_xtile_gather<T, 16>), g, b, 0, s, pieces, p->d_col16,
                         static_cast<const T *>(x), p->n_cols, xg);
    else if (p->xt_u == 8)
      hipLaunchKernelGGL((k_xtile_gather<T, 8>), g, b, 0, s, pieces, p->d_col16,
                         static_cast<const T *>(x), p->n_cols, xg);
    else
      hipLaunchKernelGGL((k_xtile_gather<T, 4>), g, b, 0, s, pieces, p->d_col16,
                         static_cast<const T *>(x), p->n_cols, xg);
    return check_launch(s);
  };
  auto reduce = [&](int64_t c0, int64_t c1, hipStream_t rs) -> int {
    if (c1 <= c0) return LHPC_OK;
    const int64_t Cx = (c1 - c0 + 7) / 8;
    constexpr int BLK = xt_red_blk<T>();
    const dim3 rg(static_cast<unsigned>(8 * Cx)), rb(BLK);
#define LHPC_XT_RED1(GG, PP)                                                                             \
  hipLaunchKernelGGL((k_xtile_reduce<T, GG, BLK, PP>), rg, rb, p->xt_lds, rs, p->d_cdesc, p->d_segoff, p->S, \
                     c0, c1, Cx, static_cast<int>(p->xt_total), xg, p->d_perm,                         \
                     static_cast<const T *>(p->d_val),                                                 \
                     static_cast<const int32_t *>(p->d_row_ptr), static_cast<T *>(y), p->d_carry)
#define LHPC_XT_RED(GG) \
  do {                     \
    if (p->xt_p == 2)      \
      LHPC_XT_RED1(GG, 2); \
    else if (p->xt_p == 3) \
      LHPC_XT_RED1(GG, 3); \
    else                   \
      LHPC_XT_RED1(GG, 1); \
  } while (0)
    switch (xtile_g<T>(p->S)) {
      case 1: LHPC_XT_RED(1); break;
      case 2: LHPC_XT_RED(2); break;
      case 4: LHPC_XT_RED(4); break;
      case 8: LHPC_XT_RED(8); break;
      default: LHPC_XT_RED(16); break;
    }
#undef LHPC_XT_RED
#undef LHPC_XT_RED1
    return check_launch(rs);
  };
  if (p->xt_K <= 1) {
    LHPC_TRY(gather(p->d_pieces, p->xt_pieces));
    LHPC_TRY(reduce(0, p->xt_C, s));
  } else {
    for (int k = 0; k < p->xt_K; ++k) {
      LHPC_TRY(gather(p->d_rpieces + 3 * p->xt_rpo[k], p->xt_rpo[k + 1] - p->xt_rpo[k]));
      LHPC_HIP_TRY(hipEventRecord(p->xt_ev[k], s));
      LHPC_HIP_TRY(hipStreamWaitEvent(p->xt_s2, p->xt_ev[k], 0));
      LHPC_TRY(reduce(p->xt_rc[k], p->xt_rc[k + 1], p->xt_s2));
    }
    LHPC_HIP_TRY(hipEventRecord(p->xt_ev[p->xt_K], p->xt_s2));
    LHPC_HIP_TRY(hipStreamWaitEvent(s, p->xt_ev[p->xt_K], 0));
  }
  }
  if (p->xt_cont > 0) {
    hipLaunchKernelGGL((k_xtile_fixup<T>), dim3(static_cast<unsigned>((p->xt_cont + kXtBlock - 1) / kXtBlock)),
                       dim3(kXtBlock), 0, s, p->d_cont, p->xt_cont, p->d_cr, p->xt_C, p->d_carry,
                       static_cast<T *>(y));
    LHPC_TRY(check_launch(s));
  }
  return LHPC_OK;
}

// lhpc_spmv_stage: the gather of a split plan; lhpc_spmv_range: range k's
// reduce + fix-up into y_k (row xt_srow[k] at y_k[0]).
template <typename T>
int launch_xtile_stage(const lhpc_spmv_plan *p, const void *x, hipStream_t s) {
  if (p->xt_pieces <= 0) return LHPC_OK;
  const dim3 g(static_cast<unsigned>(p->xt_pieces)), b(kXtGatherBlock);
  T *xg = static_cast<T *>(p->d_xg);
  if (p->xt_u == 2)
    hipLaunchKernelGGL((k_xtile_gather<T, 2>), g, b, 0, s, p->d_pieces, p->d_col16,
                       static_cast<const T *>(x), p->n_cols, xg);
  else if (p->xt_u == 16)
    hipLaunchKernelGGL((k_xtile_gather<T, 16>), g, b, 0, s, p->d_pieces, p->d_col16,
                       static_cast<const T *>(x), p->n_cols, xg);
  else if (p->xt_u == 8)
    hipLaunchKernelGGL((k_xtile_gather<T, 8>), g, b, 0, s, p->d_pieces, p->d_col16,
                       static_cast<const T *>(x), p->n_cols, xg);
  else
    hipLaunchKernelGGL((k_xtile_gather<T, 4>), g, b, 0, s, p->d_pieces, p->d_col16,
                       static_cast<const T *>(x), p->n_cols, xg);
  return check_launch(s);
}

template <typename T>
int launch_xtile_range(const lhpc_spmv_plan *p, int k, void *yk, hipStream_t s) {
  const int64_t c0 = p->xt_src[k], c1 = p->xt_src[k + 1];
  T *y = static_cast<T *>(yk) - p->xt_srow[k];  // rows are written at their plan index
  T *xg = static_cast<T *>(p->d_xg);
  if (c1 > c0) {
    const int64_t Cx = (c1 - c0 + 7) / 8;
    constexpr int BLK = xt_red_blk<T>();
    const dim3 rg(static_cast<unsigned>(8 * Cx)), rb(BLK);
#define LHPC_XT_RED1(GG, PP)                                                                             \
  hipLaunchKernelGGL((k_xtile_reduce<T, GG, BLK, PP>), rg, rb, p->xt_lds, s, p->d_cdesc, p->d_segoff, p->S, \
                     c0, c1, Cx, static_cast<int>(p->xt_total), xg, p->d_perm,                         \
                     static_cast<const T *>(p->d_val), static_cast<const int32_t *>(p->d_row_ptr), y,  \
                     p->d_carry)
#define LHPC_XT_RED(GG) \
  do {                     \
    if (p->xt_p == 2)      \
      LHPC_XT_RED1(GG, 2); \
    else if (p->xt_p == 3) \
      LHPC_XT_RED1(GG, 3); \
    else                   \
      LHPC_XT_RED1(GG, 1); \
  } while (0)
    switch (xtile_g<T>(p->S)) {
      case 1: LHPC_XT_RED(1); break;
      case 2: LHPC_XT_RED(2); break;
      case 4: LHPC_XT_RED(4); break;
      case 8: LHPC_XT_RED(8); break;
      default: LHPC_XT_RED(16); break;
    }
#undef LHPC_XT_RED
#undef LHPC_XT_RED1
    LHPC_TRY(check_launch(s));
  }
  const int64_t n0 = p->xt_sco[k], n1 = p->xt_sco[k + 1];
  if (n1 > n0) {
    hipLaunchKernelGGL((k_xtile_fixup<T>), dim3(static_cast<unsigned>((n1 - n0 + kXtBlock - 1) / kXtBlock)),
                       dim3(kXtBlock), 0, s, p->d_cont + n0, n1 - n0, p->d_cr, c1, p->d_carry, y);
    LHPC_TRY(check_launch(s));
  }
  return LHPC_OK;
}

template <typename T>
int launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  if (p->kernel == LHPC_KERNEL_XTILE) return launch_xtile<T>(p, x, y, s);
  if (p->kernel == LHPC_KERNEL_XSLICE) return launch_xslice<T>(p, x, y, s);
  if (p->kernel == LHPC_KERNEL_ADAPTIVE)
    return p->rp64 ? launch_adaptive<T, int64_t>(p, x, y, s)
                   : launch_adaptive<T, int32_t>(p, x, y, s);
  return p->rp64 ? launch_rowgroup<T, int64_t>(p, x, y, s)
                 : launch_rowgroup<T, int32_t>(p, x, y, s);
}

// Host view of row_ptr regardless of width.
struct RowPtrView {
  const void *p;
  int bits;
  int64_t operator[](int64_t i) const {
    return bits == 64 ? static_cast<const int64_t *>(p)[i]
                      : static_cast<const int32_t *>(p)[i];
  }
};

// Row blocks for ADAPTIVE: greedy, each block <= kBlockNnz nonzeros and
// <= kBlock rows, or a single row of any length.
std::vector<int64_t> build_blocks(RowPtrView rp, int64_t n_rows, int64_t &n_long) {
  std::vector<int64_t> b;
  b.reserve(static_cast<size_t>(n_rows / 64 + 2));
  n_long = 0;
  int64_t r = 0;
  while (r < n_rows) {
    b.push_back(r);
    const int64_t start = rp[r];
    if (rp[r + 1] - start > kBlockNnz) {
      ++n_long;
      ++r;
      continue;
    }
    int64_t end = r + 1;
    while (end < n_rows && end - r < kBlock && rp[end + 1] - start <= kBlockNnz) ++end;
    r = end;
  }
  b.push_back(n_rows);
  return b;
}

}  // namespace

namespace {
// XTILE plan: re-encode A (lhpc_plan.cpp build_xtile) and copy it to HBM.
int build_xtile_plan(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val,
                     size_t tsz) {
  const int64_t W = tsz == 4 ? XtTile<float>::W : XtTile<double>::W;
  int cus = 256;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, p->device) == hipSuccess) cus = prop.multiProcessorCount;
  // ≈ 2 gather workgroups per CU (one resident per CU: 160 KB of LDS each)
  // and ≥ 4 tiles' worth of stream per piece, so the tile load (W·T bytes)
  // stays ≤ 1/4 of a piece's col16 + xg traffic on small (per-rank) matrices
  const int64_t min_piece = 4 * W * static_cast<int64_t>(tsz) / (2 + static_cast<int64_t>(tsz));
  int64_t piece = std::max<int64_t>(min_piece, p->nnz / (2 * static_cast<int64_t>(cus)) + 1);
  if (const char *env = std::getenv("LHPC_XTILE_PIECE")) piece = std::max<int64_t>(8, std::atoll(env));
  XtileHost xt;
  // LHPC_XTILE_LAYOUT=cm: chunk-major xg (opt-in: its scattered xg stores make
  // the gather 2.5x slower on C2 than the reduce saves, DESIGN.md §4 XTILE)
  int cm = 0;
  if (const char *env = std::getenv("LHPC_XTILE_LAYOUT")) cm = std::strcmp(env, "cm") == 0;
  p->xt_cm = cm;
  // chunking: the seg reduce's M / Rmax for this type; the cm reduce's fixed 4096 / 512
  const int cM = cm ? kXtM : (tsz == 4 ? XtRed<float, xt_red_blk<float>()>::M : XtRed<double, xt_red_blk<double>()>::M);
  const int cR = cm ? kXtRmax : (tsz == 4 ? XtRed<float, xt_red_blk<float>()>::Rmax : XtRed<double, xt_red_blk<double>()>::Rmax);
  // reduce positions per lane (LHPC_XTILE_PAIR=0/1): 2 pads every
  // (chunk, tile) segment to an even length, so phase A loads xg/perm as
  // aligned pairs (DESIGN.md §4 XTILE)
  // xt_p = 3 (default; LHPC_XTILE_IPERM=0 selects the perm scatter, 1): the
  // reduce keeps the chunk's segments in flat order in LDS and gathers each
  // CSR position's x through iperm (CSR order, read with val) instead of
  // scattering them by perm (DESIGN.md §4 XTILE: C2 589 → 580 µs, C3 1169 → 1086 µs)
  // Only for ≥ 32 chunks per CU: with fewer (per-rank matrices at N ≥ 4) the
  // perm reduce's shorter blocks win (W = 8 rank of C2: 0.088 against
  // 0.093 ms; W = 1: 0.626 against 0.611 ms; profiles/r01/explore_scaling_*)
  int pp = p->nnz >= 32LL * cus * cM ? 3 : 1;
  if (const char *env = std::getenv("LHPC_XTILE_IPERM")) pp = std::atoi(env) ? 3 : 1;
  if (const char *env = std::getenv("LHPC_XTILE_PAIR")) pp = std::atoi(env) ? 2 : pp;
  p->xt_p = cm ? 1 : pp;
  const int bst = build_xtile(rp.p, rp.bits, col_idx, p->n_rows, p->n_cols, W, cM, cR, piece,
                              cm != 0, static_cast<int>(tsz), p->split_rows.data(),
                              static_cast<int>(p->split_rows.size()), xt, p->xt_p == 2 ? 2 : 1,
                              p->xt_p == 3);
  if (bst != LHPC_OK) return bst;
  p->kernel = LHPC_KERNEL_XTILE;
  p->rp64 = 0;
  p->S = xt.S;
  p->xs_width = W;
  p->xt_C = xt.n_chunks;
  p->xt_pieces = static_cast<int64_t>(xt.pieces.size() / 3);
  p->xt_cont = static_cast<int64_t>(xt.cont.size());
  p->xt_total = xt.total;
  p->xt_lds = tsz == 4 ? xtile_lds_bytes<float>(xt.S) : xtile_lds_bytes<double>(xt.S);
  if (const char *env = std::getenv("LHPC_XTILE_U")) {
    const int u = std::atoi(env);
    p->xt_u = u <= 1 && cm ? 1 : u == 2 ? 2 : u >= 16 && !cm ? 16 : u >= 8 && !cm ? 8 : 4;  // U = 1: chunk-major gather only; 8: tile-stream only
  }
  if (!cm) {
    const int g = tsz == 4 ? xtile_g<float>(xt.S) : xtile_g<double>(xt.S);
    const void *kfn = tsz == 4 ? (p->xt_p == 2   ? xtile_reduce_fn<float, 2>(g)
                                  : p->xt_p == 3 ? xtile_reduce_fn<float, 3>(g)
                                                 : xtile_reduce_fn<float, 1>(g))
                               : (p->xt_p == 2   ? xtile_reduce_fn<double, 2>(g)
                                  : p->xt_p == 3 ? xtile_reduce_fn<double, 3>(g)
                                                 : xtile_reduce_fn<double, 1>(g));
    LHPC_HIP_TRY(hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(p->xt_lds)));
  }
  const int64_t n_rows = p->n_rows, nnz = p->nnz, C = xt.n_chunks;
  auto up = [&](void **d, const void *h, size_t n) -> int {
    LHPC_TRY(dmalloc(d, n, p->bytes));
    if (n && h) LHPC_HIP_TRY(hipMemcpy(*d, h, n, hipMemcpyHostToDevice));
    return LHPC_OK;
  };
  std::vector<int32_t> rp32(static_cast<size_t>(n_rows + 1));
  for (int64_t i = 0; i <= n_rows; ++i) rp32[static_cast<size_t>(i)] = static_cast<int32_t>(rp[i]);
  LHPC_TRY(up(&p->d_row_ptr, rp32.data(), rp32.size() * 4));
  // val padded by one run: a reduce thread loads its whole 16-nonzero run as vectors
  LHPC_TRY(dmalloc(&p->d_val, static_cast<size_t>(nnz + kXtRun) * tsz, p->bytes));
  LHPC_HIP_TRY(hipMemset(static_cast<unsigned char *>(p->d_val) + nnz * tsz, 0, kXtRun * tsz));
  if (nnz) LHPC_HIP_TRY(hipMemcpy(p->d_val, val, static_cast<size_t>(nnz) * tsz, hipMemcpyHostToDevice));
  {
    std::vector<int32_t> cd(static_cast<size_t>(4 * C + 4));
    for (int64_t c = 0; c < C; ++c) {
      cd[4 * c] = xt.ce[c];
      cd[4 * c + 1] = xt.ce[c + 1];
      cd[4 * c + 2] = xt.cr[c];
      cd[4 * c + 3] = xt.cr[c + 1];
    }
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_cdesc), cd.data(), cd.size() * 4));
  }
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_ce), xt.ce.data(), xt.ce.size() * 4));
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_cr), xt.cr.data(), xt.cr.size() * 4));
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_pieces), xt.pieces.data(), xt.pieces.size() * 4));
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_cont), xt.cont.data(), xt.cont.size() * 4));
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_col16), xt.col16.get(), static_cast<size_t>(xt.total) * 2));
  if (cm) {
    // xg and perm are indexed by nonzero, padded by one reduce run (never stored, read masked)
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_gdst), xt.gdst.get(), static_cast<size_t>(xt.total / 8) * 4));
    LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_perm), static_cast<size_t>(nnz + kXtRun) * 2, p->bytes));
    LHPC_HIP_TRY(hipMemset(p->d_perm + nnz, 0, kXtRun * 2));
    if (nnz) LHPC_HIP_TRY(hipMemcpy(p->d_perm, xt.perm.get(), static_cast<size_t>(nnz) * 2, hipMemcpyHostToDevice));
    LHPC_TRY(up(&p->d_xg, nullptr, static_cast<size_t>(nnz + kXtRun) * tsz));
  } else {
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_segoff), xt.segoff.data(), xt.segoff.size() * 4));
    // one sentinel entry past the stream: reduce loads it for positions past m,
    // and its perm is the byte offset of the spare LDS slot M + M/16 − 1
    // (xt_p entries: a pair-mode lane loads the sentinel pair)
    if (p->xt_p == 3) {  // iperm mode: the reduce reads iperm ([C][M], CSR order) in perm's place
      const size_t ni = static_cast<size_t>(C > 0 ? C : 1) * static_cast<size_t>(cM);
      LHPC_TRY(up(reinterpret_cast<void **>(&p->d_perm), xt.iperm.get(), ni * 2));
    } else {
      LHPC_TRY(up(reinterpret_cast<void **>(&p->d_perm), nullptr, static_cast<size_t>(xt.total + 2) * 2));
      if (xt.total) LHPC_HIP_TRY(hipMemcpy(p->d_perm, xt.perm.get(), static_cast<size_t>(xt.total) * 2, hipMemcpyHostToDevice));
      const uint16_t spare[2] = {static_cast<uint16_t>(cM), static_cast<uint16_t>(cM)};  // slot M: one 16-B slot past the chunk
      LHPC_HIP_TRY(hipMemcpy(p->d_perm + xt.total, spare, 4, hipMemcpyHostToDevice));
    }
    LHPC_TRY(up(&p->d_xg, nullptr, static_cast<size_t>(xt.total + 2) * tsz));
  }
  LHPC_TRY(up(reinterpret_cast<void **>(&p->d_carry), nullptr, static_cast<size_t>(2 * C + 2) * 8));
  LHPC_HIP_TRY(hipMemset(p->d_carry, 0, static_cast<size_t>(2 * C + 2) * 8));
  if (!p->split_rows.empty()) {
    const size_t K = p->split_rows.size() + 1;
    p->xt_srow.assign(1, 0);
    p->xt_srow.insert(p->xt_srow.end(), p->split_rows.begin(), p->split_rows.end());
    p->xt_srow.push_back(n_rows);
    p->xt_src.assign(xt.rchunk.begin(), xt.rchunk.end());
    p->xt_sco.assign(K + 1, 0);
    for (size_t k = 0; k <= K; ++k)
      p->xt_sco[k] = std::lower_bound(xt.cont.begin(), xt.cont.end(), static_cast<int32_t>(p->xt_src[k])) -
                     xt.cont.begin();
  }
  // pipelined ranges (seg): K chunk ranges, one gather piece per (range, tile):
  // [ceil8(segoff(s, c_k)), ceil8(segoff(s, c_k+1))) — the last range ends at
  // the tile's padded end.  The 8-entry group straddling a range bound is
  // gathered with the earlier range, which completes first on the caller's
  // stream, so every range's entries are written before its reduce starts.
  // Opt-in (LHPC_XTILE_RANGES=K): measured slower on C2 (K = 2/4/8/16: 0.68–0.73
  // ms against 0.63 ms at K = 1): the overlapped gather and reduce contend for
  // the same HBM stream rate instead of filling each other's gaps.
  int K = 1;
  if (const char *env = std::getenv("LHPC_XTILE_RANGES")) K = std::max(1, std::atoi(env));
  K = static_cast<int>(std::min<int64_t>(K, std::max<int64_t>(1, C)));
  if (!cm && K > 1) {
    const int64_t S = xt.S;
    std::vector<int32_t> rpcs;
    p->xt_rc.assign(static_cast<size_t>(K) + 1, 0);
    p->xt_rpo.assign(static_cast<size_t>(K) + 1, 0);
    for (int k = 0; k <= K; ++k) p->xt_rc[k] = C * k / K;
    for (int k = 0; k < K; ++k) {
      for (int64_t s = 0; s < S; ++s) {
        const int64_t g0 = (xt.segoff[static_cast<size_t>(p->xt_rc[k] * S + s)] + 7) & ~int64_t{7};
        const int64_t g1 = (xt.segoff[static_cast<size_t>(p->xt_rc[k + 1] * S + s)] + 7) & ~int64_t{7};
        if (g1 > g0) {
          rpcs.push_back(static_cast<int32_t>(g0));
          rpcs.push_back(static_cast<int32_t>(g1));
          rpcs.push_back(static_cast<int32_t>(s));
        }
      }
      p->xt_rpo[k + 1] = static_cast<int64_t>(rpcs.size() / 3);
    }
    LHPC_TRY(up(reinterpret_cast<void **>(&p->d_rpieces), rpcs.data(), rpcs.size() * 4));
    LHPC_HIP_TRY(hipStreamCreateWithFlags(&p->xt_s2, hipStreamNonBlocking));
    p->xt_ev.assign(static_cast<size_t>(K) + 1, nullptr);
    for (auto &e : p->xt_ev) LHPC_HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    p->xt_K = K;
  }
  return LHPC_OK;
}
}  // namespace

namespace {
int plan_create_impl(lhpc_spmv_plan **out, int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz,
                     const void *row_ptr, int row_ptr_bits, const int32_t *col_idx, const void *val,
                     const int *device_ids, int n_devices, unsigned flags, int n_splits,
                     const int64_t *split_rows) {
  if (!out) return LHPC_ERR_INVALID_ARG;
  *out = nullptr;
  if ((dtype != LHPC_F32 && dtype != LHPC_F64) || n_rows < 0 || n_cols < 0 || nnz < 0 ||
      !row_ptr || (row_ptr_bits != 32 && row_ptr_bits != 64) || n_cols > INT32_MAX ||
      (nnz > 0 && (!col_idx || !val)))
    return LHPC_ERR_INVALID_ARG;
  if (n_devices > 1) return LHPC_ERR_UNSUPPORTED;  // one process per GPU
  if (flags & LHPC_PLAN_DEVICE_INPUT) return LHPC_ERR_UNSUPPORTED;
  if (row_ptr_bits == 32 && nnz > INT32_MAX) return LHPC_ERR_INVALID_ARG;

  const RowPtrView rp{row_ptr, row_ptr_bits};
  if (rp[0] != 0 || rp[n_rows] != nnz) return LHPC_ERR_BAD_CSR;
  if (flags & LHPC_PLAN_VALIDATE) {
    for (int64_t i = 0; i < n_rows; ++i)
      if (rp[i + 1] < rp[i]) return LHPC_ERR_BAD_CSR;
    for (int64_t k = 0; k < nnz; ++k)
      if (col_idx[k] < 0 || col_idx[k] >= n_cols) return LHPC_ERR_BAD_CSR;
  }

  int dev = 0;
  if (device_ids && n_devices == 1) {
    dev = device_ids[0];
    LHPC_HIP_TRY(hipSetDevice(dev));
  } else {
    LHPC_HIP_TRY(hipGetDevice(&dev));
  }
  if (!is_gfx950(dev)) return LHPC_ERR_NO_DEVICE;

  auto *p = new (std::nothrow) lhpc_spmv_plan();
  if (!p) return LHPC_ERR_ALLOC;
  if (n_splits > 0) p->split_rows.assign(split_rows, split_rows + n_splits);
  p->dtype = dtype;
  p->device = dev;
  p->n_rows = n_rows;
  p->n_cols = n_cols;
  p->nnz = nnz;
  // int32 offsets whenever they fit: 4 B/row less HBM traffic
  p->rp64 = nnz > INT32_MAX ? 1 : 0;
  const size_t tsz = dtype == LHPC_F32 ? 4 : 8;

  // ---- kernel selection from row-length statistics
  int64_t maxlen = 0;
  double sum2 = 0;
  for (int64_t i = 0; i < n_rows; ++i) {
    const int64_t l = rp[i + 1] - rp[i];
    maxlen = std::max(maxlen, l);
    sum2 += static_cast<double>(l) * static_cast<double>(l);
  }
  const double mean = n_rows ? static_cast<double>(nnz) / static_cast<double>(n_rows) : 0;
  const double var = n_rows ? sum2 / static_cast<double>(n_rows) - mean * mean : 0;
  const double cv = mean > 0 ? std::sqrt(std::max(var, 0.0)) / mean : 0;
  // Off the XSLICE path ADAPTIVE (nnz-balanced blocks, coalesced col/val stream,
  // LDS row sums) is the default: measured equal or faster than ROWGROUP on
  // uniform rows of 3-40 nnz (within 4% at 8 and 24), and 1.26-1.5× faster on
  // C1 and the 2-D Laplacians (tools/explore_rowlen.py).
  // ROWGROUP stays selectable (FORCE_ROWGROUP); `cv`/`maxlen` are kept for info.
  (void)cv;
  bool adaptive = true;
  if (flags & LHPC_PLAN_FORCE_ROWGROUP) adaptive = false;
  if (flags & LHPC_PLAN_FORCE_ADAPTIVE) adaptive = true;
  // XSLICE when x outgrows one XCD's 4 MB L2 and rows are short enough for
  // the uint8 in-slice lengths (the builder re-checks per slice).
  const double x_bytes = static_cast<double>(n_cols) * static_cast<double>(tsz);
  double slice_mb = 5.0;
  if (const char *env = std::getenv("LHPC_XSLICE_MB")) slice_mb = std::max(0.25, std::atof(env));
  // ... and only when the gathers have no locality of their own: a banded or
  // structured matrix (stencil operators, the CG Laplacian) re-reads each x
  // line from neighbouring rows, which the row-local kernels already serve
  // from L2, while XSLICE would add S partials per row.  Measure it: distinct
  // 128-B x lines per nonzero over sampled 8192-row chunks (≈0.8 for C2's
  // uniform columns, ≈0.03 for a 2-D Laplacian); ≤ 0.25 counts as local.
  double locality_thr = 0.25;
  if (const char *env = std::getenv("LHPC_SPMV_LOCALITY")) locality_thr = std::atof(env);
  const bool auto_ok = !(flags & (LHPC_PLAN_FORCE_ROWGROUP | LHPC_PLAN_FORCE_ADAPTIVE |
                                   LHPC_PLAN_FORCE_XSLICE | LHPC_PLAN_FORCE_XTILE));
  const bool nolocal =
      auto_ok && x_bytes > 8.0e6 && gather_lines_per_nnz(rp, col_idx, n_rows, tsz) > locality_thr;
  // XTILE (x tiles in LDS) is the default for gathers without locality;
  // LHPC_SPMV_XTILE=0 selects XSLICE instead.
  bool xtile_env = true;
  if (const char *env = std::getenv("LHPC_SPMV_XTILE")) xtile_env = std::atoi(env) != 0;
  const bool want_xtile = (flags & LHPC_PLAN_FORCE_XTILE) || (nolocal && xtile_env);
  if (want_xtile && n_rows > 0) {
    int st = build_xtile_plan(p, rp, col_idx, val, tsz);
    if (st == LHPC_OK) {
      *out = p;
      return LHPC_OK;
    }
    if (st != LHPC_ERR_UNSUPPORTED) {
      lhpc_spmv_plan_destroy(p);
      return st;
    }
    // layout does not fit its index types: XSLICE / CSR kernels below
  }
  const bool want_xslice = (flags & LHPC_PLAN_FORCE_XSLICE) || nolocal;
  if (want_xslice && nnz > 0) {
    int P = static_cast<int>(std::ceil(x_bytes / (8.0 * slice_mb * 1.0e6)));
    P = std::max(1, std::min(P, 32));
    int S = 8 * P;
    if (const char *env = std::getenv("LHPC_XSLICE_S")) S = std::max(1, std::min(256, std::atoi(env)));
    if (S > 8) S = (S + 7) / 8 * 8;
    XsliceHost xs;
    bool jagged = false;
    if (const char *env = std::getenv("LHPC_XSLICE_LAYOUT")) jagged = std::strcmp(env, "jagged") == 0;
    const int bst = build_xslice(row_ptr, row_ptr_bits, col_idx, val, tsz, n_rows, n_cols, S, jagged, xs);
    if (bst == LHPC_OK) {
      p->kernel = LHPC_KERNEL_XSLICE;
      p->S = S;
      p->xs_jagged = jagged ? 1 : 0;
      // fp64 partials (exact-ish: one rounding per row overall) vs partials in
      // the value type (less traffic).  fp64 values always use fp64.
      p->xs_p64 = (tsz == 8 || ((flags & LHPC_PLAN_EXACT_PARTIALS) && !(flags & LHPC_PLAN_FAST_PARTIALS))) && !jagged
                      ? 1 : 0;
      if (const char *env = std::getenv("LHPC_XSLICE_PARTIAL")) p->xs_p64 = (tsz == 8 || !std::strcmp(env, "f64")) && !jagged;
      // fused slice reduction (fp64 partials only): opt-in.  Measured 2.5×
      // SLOWER than the separate reduce on C2 (3.07 vs 1.23 ms): every block
      // waits out its store drain + arrival atomic, which costs more than the
      // 123 µs reduce pass it removes.
      p->xs_fused = 0;
      if (const char *env = std::getenv("LHPC_XSLICE_FUSE"))
        if (!jagged && std::atoi(env) != 0) p->xs_fused = p->xs_p64 = 1;  // the hand-off is fp64
      // persistent partial-free kernel: opt-in.  Measured slower on C2/C3/C4
      // (1.65-2.3 ms vs 1.24 ms): each wave walks the S slices serially and
      // its dependent window round trips are not hidden at 4-5 waves/SIMD
      // (DESIGN.md §4).
      p->xs_persist = 0;
      if (const char *env = std::getenv("LHPC_XSLICE_PERSIST"))
        p->xs_persist = !jagged && !p->xs_fused && !(flags & LHPC_PLAN_FAST_PARTIALS) && std::atoi(env) != 0;
      if (p->xs_persist) {
        // G chunks per wave and pass (G fp64 accumulators per lane); window NB·64
        p->xs_g = 8;
        if (const char *env = std::getenv("LHPC_XSLICE_G")) p->xs_g = std::atoi(env);
        if (p->xs_g != 4 && p->xs_g != 16) p->xs_g = 8;
        p->xs_nb = 4;
        if (const char *env = std::getenv("LHPC_XSLICE_NB")) p->xs_nb = std::atoi(env) <= 2 ? 2 : 4;
        int cus = 256, per_cu = 4;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
        int occ = 0;
        const void *kfn = nullptr;
        if (tsz == 4)
          kfn = p->xs_g == 16 ? reinterpret_cast<const void *>(k_spmv_xslice_persist<float, uint8_t, 4, 16>)
                : p->xs_g == 4 ? reinterpret_cast<const void *>(k_spmv_xslice_persist<float, uint8_t, 4, 4>)
                               : reinterpret_cast<const void *>(k_spmv_xslice_persist<float, uint8_t, 4, 8>);
        else
          kfn = p->xs_g == 16 ? reinterpret_cast<const void *>(k_spmv_xslice_persist<double, uint8_t, 4, 16>)
                : p->xs_g == 4 ? reinterpret_cast<const void *>(k_spmv_xslice_persist<double, uint8_t, 4, 4>)
                               : reinterpret_cast<const void *>(k_spmv_xslice_persist<double, uint8_t, 4, 8>);
        const hipError_t oe = hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kfn, kBlock, 0);
        if (oe == hipSuccess && occ > 0) per_cu = std::min(occ, 8);
        if (const char *env = std::getenv("LHPC_XSLICE_BPC")) per_cu = std::max(1, std::atoi(env));
        p->xs_grid = cus * per_cu;
      }
      {  // window = NB·64 nonzeros: cover a typical chunk in one window
        const double mean_chunk = xs.n_chunks ? static_cast<double>(nnz) / (static_cast<double>(S) * xs.n_chunks) : 0;
        int nb = static_cast<int>(std::ceil(mean_chunk * 1.2 / kWave));
        if (const char *env = std::getenv("LHPC_XSLICE_NB")) nb = std::atoi(env);
        p->xs_nb = std::max(1, std::min(nb, 4));
      }
      p->xs_width = xs.width;
      p->xs_chunks = xs.n_chunks;
      p->xs_rows_pad = xs.n_rows_pad;
      p->xs_bps = (xs.n_chunks + (kBlock / kWave) - 1) / (kBlock / kWave);
      int st = LHPC_OK;
      do {
        const size_t lb = static_cast<size_t>(S) * xs.n_rows_pad;
        const size_t cb = (static_cast<size_t>(S) * xs.n_chunks + 1) * 8;
        p->xs_lens16 = xs.lens_bytes == 2 ? 1 : 0;
        if ((st = dmalloc(&p->d_lens, lb * xs.lens_bytes, p->bytes))) break;
        if ((st = dmalloc(reinterpret_cast<void **>(&p->d_cbase), cb, p->bytes))) break;
        if ((st = dmalloc(reinterpret_cast<void **>(&p->d_col), static_cast<size_t>(nnz) * 4, p->bytes))) break;
        if ((st = dmalloc(&p->d_val, static_cast<size_t>(nnz) * tsz, p->bytes))) break;
        if (!p->xs_persist && (st = dmalloc(&p->d_partial, lb * (p->xs_p64 ? 8 : tsz), p->bytes))) break;
        if (p->xs_fused) {
          const size_t ab = static_cast<size_t>((p->xs_bps + 3) / 4 * 16);  // 16-B multiple, from the allocation start
          if ((st = dmalloc(reinterpret_cast<void **>(&p->d_arrive), ab, p->bytes))) break;
          if ((st = static_cast<int>(hipMemset(p->d_arrive, 0, ab)))) break;
        }
        if ((st = static_cast<int>(hipMemcpy(p->d_lens, xs.lens.get(), lb * xs.lens_bytes, hipMemcpyHostToDevice)))) break;
        if ((st = static_cast<int>(hipMemcpy(p->d_cbase, xs.cbase.get(), cb, hipMemcpyHostToDevice)))) break;
        if ((st = static_cast<int>(hipMemcpy(p->d_col, xs.col.get(), static_cast<size_t>(nnz) * 4, hipMemcpyHostToDevice)))) break;
        if ((st = static_cast<int>(hipMemcpy(p->d_val, xs.val.get(), static_cast<size_t>(nnz) * tsz, hipMemcpyHostToDevice)))) break;
      } while (false);
      if (st != LHPC_OK) {
        lhpc_spmv_plan_destroy(p);
        return st;
      }
      *out = p;
      return LHPC_OK;
    }
    if (bst != LHPC_ERR_UNSUPPORTED) {
      lhpc_spmv_plan_destroy(p);
      return bst;
    }
    // some row too long for one slice: fall through to a CSR kernel
  }
  if (adaptive) {
    p->kernel = LHPC_KERNEL_ADAPTIVE;
  } else {
    p->kernel = LHPC_KERNEL_ROWGROUP;
    int L = 4;
    while (L < 64 && L < mean) L <<= 1;
    p->L = L;
    p->R = L <= 16 ? 4 : (L == 32 ? 2 : 1);
    if (L == 4) p->R = 1;
  }
  if (const char *env = std::getenv("LHPC_SPMV_ROWGROUP")) {  // "L,R" bench knob
    int L = 0, R = 0;
    if (std::sscanf(env, "%d,%d", &L, &R) == 2 && p->kernel == LHPC_KERNEL_ROWGROUP) {
      p->L = L;
      p->R = R;
    }
  }

  int st = LHPC_OK;
  do {
    const size_t rp_bytes = static_cast<size_t>(n_rows + 1) * (p->rp64 ? 8 : 4);
    if ((st = dmalloc(&p->d_row_ptr, rp_bytes, p->bytes))) break;
    if ((st = dmalloc(reinterpret_cast<void **>(&p->d_col), static_cast<size_t>(nnz) * 4,
                      p->bytes)))
      break;
    if ((st = dmalloc(&p->d_val, static_cast<size_t>(nnz) * tsz, p->bytes))) break;
    // row_ptr in the device width
    if (p->rp64 == (row_ptr_bits == 64 ? 1 : 0)) {
      if ((st = static_cast<int>(hipMemcpy(p->d_row_ptr, row_ptr, rp_bytes, hipMemcpyHostToDevice))))
        break;
    } else {
      std::vector<int32_t> tmp(static_cast<size_t>(n_rows + 1));
      for (int64_t i = 0; i <= n_rows; ++i) tmp[static_cast<size_t>(i)] = static_cast<int32_t>(rp[i]);
      if ((st = static_cast<int>(hipMemcpy(p->d_row_ptr, tmp.data(), rp_bytes, hipMemcpyHostToDevice))))
        break;
    }
    if (nnz) {
      if ((st = static_cast<int>(hipMemcpy(p->d_col, col_idx, static_cast<size_t>(nnz) * 4,
                                           hipMemcpyHostToDevice))))
        break;
      if ((st = static_cast<int>(hipMemcpy(p->d_val, val, static_cast<size_t>(nnz) * tsz,
                                           hipMemcpyHostToDevice))))
        break;
    }
    if (p->kernel == LHPC_KERNEL_ADAPTIVE) {
      std::vector<int64_t> b = build_blocks(rp, n_rows, p->n_long);
      p->n_blocks = static_cast<int64_t>(b.size()) - 1;
      if ((st = dmalloc(reinterpret_cast<void **>(&p->d_blocks), b.size() * 8, p->bytes))) break;
      if ((st = static_cast<int>(hipMemcpy(p->d_blocks, b.data(), b.size() * 8, hipMemcpyHostToDevice))))
        break;
    }
  } while (false);
  if (st != LHPC_OK) {
    lhpc_spmv_plan_destroy(p);
    return st;
  }
  *out = p;
  return LHPC_OK;
}
}  // namespace

extern "C" int lhpc_spmv_plan_create(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                                     int64_t n_cols, int64_t nnz, const void *row_ptr,
                                     int row_ptr_bits, const int32_t *col_idx,
                                     const void *val, const int *device_ids,
                                     int n_devices, unsigned flags) {
  return plan_create_impl(out, dtype, n_rows, n_cols, nnz, row_ptr, row_ptr_bits, col_idx, val,
                          device_ids, n_devices, flags, 0, nullptr);
}

extern "C" int lhpc_spmv_plan_create_split(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                                           int64_t n_cols, int64_t nnz, const void *row_ptr,
                                           int row_ptr_bits, const int32_t *col_idx,
                                           const void *val, const int *device_ids, int n_devices,
                                           unsigned flags, int n_splits, const int64_t *split_rows) {
  if (!out || n_splits < 1 || !split_rows) return LHPC_ERR_INVALID_ARG;
  for (int i = 0; i < n_splits; ++i)
    if (split_rows[i] <= 0 || split_rows[i] >= n_rows || (i > 0 && split_rows[i] <= split_rows[i - 1]))
      return LHPC_ERR_INVALID_ARG;
  const int st = plan_create_impl(out, dtype, n_rows, n_cols, nnz, row_ptr, row_ptr_bits, col_idx, val,
                                  device_ids, n_devices, flags, n_splits, split_rows);
  if (st != LHPC_OK) return st;
  const lhpc_spmv_plan *p = *out;
  if (p->kernel != LHPC_KERNEL_XTILE || p->xt_cm || p->xt_srow.size() != static_cast<size_t>(n_splits) + 2) {
    lhpc_spmv_plan_destroy(*out);  // ranges exist only in the XTILE tile-stream layout
    *out = nullptr;
    return LHPC_ERR_UNSUPPORTED;
  }
  return LHPC_OK;
}

extern "C" int lhpc_spmv_stage(const lhpc_spmv_plan *p, const void *x, void *stream) {
  if (!p || (p->n_cols > 0 && !x)) return LHPC_ERR_INVALID_ARG;
  if (p->xt_srow.empty()) return LHPC_ERR_UNSUPPORTED;
  LHPC_HIP_TRY(hipSetDevice(p->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  return p->dtype == LHPC_F32 ? launch_xtile_stage<float>(p, x, s) : launch_xtile_stage<double>(p, x, s);
}

extern "C" int lhpc_spmv_range(const lhpc_spmv_plan *p, int k, void *y_range, void *stream) {
  if (!p || p->xt_srow.empty() || k < 0 || k + 2 > static_cast<int>(p->xt_srow.size()))
    return LHPC_ERR_INVALID_ARG;
  if (p->xt_srow[k + 1] > p->xt_srow[k] && !y_range) return LHPC_ERR_INVALID_ARG;
  LHPC_HIP_TRY(hipSetDevice(p->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  return p->dtype == LHPC_F32 ? launch_xtile_range<float>(p, k, y_range, s)
                              : launch_xtile_range<double>(p, k, y_range, s);
}

extern "C" int lhpc_spmv(lhpc_spmv_plan *p, const void *x, void *y, int on_device,
                         void *stream) {
  if (!p || (p->n_cols > 0 && !x) || (p->n_rows > 0 && !y)) return LHPC_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  LHPC_HIP_TRY(hipSetDevice(p->device));
  const size_t tsz = p->dtype == LHPC_F32 ? 4 : 8;
  const void *dx = x;
  void *dy = y;
  if (!on_device) {
    if (!p->d_xstage) {
      LHPC_TRY(dmalloc(&p->d_xstage, static_cast<size_t>(p->n_cols) * tsz, p->bytes));
      LHPC_TRY(dmalloc(&p->d_ystage, static_cast<size_t>(p->n_rows) * tsz, p->bytes));
    }
    LHPC_HIP_TRY(hipMemcpyAsync(p->d_xstage, x, static_cast<size_t>(p->n_cols) * tsz,
                                hipMemcpyHostToDevice, s));
    dx = p->d_xstage;
    dy = p->d_ystage;
  }
  const int st = p->dtype == LHPC_F32 ? launch<float>(p, dx, dy, s) : launch<double>(p, dx, dy, s);
  if (st != LHPC_OK) return st;
  if (!on_device) {
    LHPC_HIP_TRY(hipMemcpyAsync(y, p->d_ystage, static_cast<size_t>(p->n_rows) * tsz,
                                hipMemcpyDeviceToHost, s));
    LHPC_HIP_TRY(hipStreamSynchronize(s));
  }
  return LHPC_OK;
}

extern "C" int lhpc_vec_dot(int dtype, int64_t n, const void *a, const void *b, double *out, void *stream);

extern "C" int lhpc_spmv_dot(lhpc_spmv_plan *p, const void *x, void *y, const void *w, double *dot_out,
                             void *stream) {
  if (!p || !dot_out || (p->n_cols > 0 && !x) || (p->n_rows > 0 && (!y || !w))) return LHPC_ERR_INVALID_ARG;
  hipStream_t s = static_cast<hipStream_t>(stream);
  LHPC_HIP_TRY(hipSetDevice(p->device));
  if (p->kernel == LHPC_KERNEL_ADAPTIVE && p->n_blocks > 0) {
    const int64_t n1 = (p->n_blocks + kFinTile - 1) / kFinTile;  // stage-1 sums, after the partials
    if (!p->d_dpart)
      LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_dpart), (p->n_blocks + n1) * sizeof(double), p->bytes));
    int st;
    if (p->dtype == LHPC_F32)
      st = p->rp64 ? launch_adaptive<float, int64_t>(p, x, y, s, w, p->d_dpart)
                   : launch_adaptive<float, int32_t>(p, x, y, s, w, p->d_dpart);
    else
      st = p->rp64 ? launch_adaptive<double, int64_t>(p, x, y, s, w, p->d_dpart)
                   : launch_adaptive<double, int32_t>(p, x, y, s, w, p->d_dpart);
    LHPC_TRY(st);
    double *stage1 = p->d_dpart + p->n_blocks;
    if (n1 == 1) {
      hipLaunchKernelGGL(k_dpart_finish, dim3(1), dim3(kBlock), 0, s, p->d_dpart, p->n_blocks, dot_out);
    } else {
      hipLaunchKernelGGL(k_dpart_finish, dim3(static_cast<unsigned>(n1)), dim3(kBlock), 0, s, p->d_dpart,
                         p->n_blocks, stage1);
      if (n1 > kFinTile) return LHPC_ERR_UNSUPPORTED;  // > 4M blocks (> 8·10^9 nonzeros)
      hipLaunchKernelGGL(k_dpart_finish, dim3(1), dim3(kBlock), 0, s, stage1, n1, dot_out);
    }
    return check_launch(s);
  }
  // other kernel families: SpMV, then a separate dot pass
  LHPC_TRY(lhpc_spmv(p, x, y, 1, stream));
  return lhpc_vec_dot(p->dtype, p->n_rows, w, y, dot_out, stream);
}

extern "C" int lhpc_spmv_plan_info_get(const lhpc_spmv_plan *p, lhpc_spmv_plan_info *info) {
  if (!p || !info) return LHPC_ERR_INVALID_ARG;
  info->dtype = p->dtype;
  info->kernel = p->kernel;
  info->lanes_per_row = p->kernel == LHPC_KERNEL_ROWGROUP ? p->L : 0;
  info->rows_per_group = p->kernel == LHPC_KERNEL_ROWGROUP ? p->R : 0;
  info->n_rows = p->n_rows;
  info->n_cols = p->n_cols;
  info->nnz = p->nnz;
  info->n_blocks = p->n_blocks;
  info->n_long_rows = p->n_long;
  info->device_bytes = p->bytes;
  info->device = p->device;
  info->launches = p->kernel == LHPC_KERNEL_XSLICE && !p->xs_fused && !p->xs_persist ? 2 : 1;
  if (p->kernel == LHPC_KERNEL_XTILE) {
    info->launches = (p->xt_pieces > 0 ? 1 : 0) + 1 + (p->xt_cont > 0 ? 1 : 0);
    info->n_blocks = p->xt_C;
    info->n_long_rows = p->xt_cont;
  }
  info->slices = p->S;
  info->slice_width = p->xs_width;
  return LHPC_OK;
}

extern "C" int lhpc_spmv_plan_destroy(lhpc_spmv_plan *p) {
  if (!p) return LHPC_OK;
  (void)hipSetDevice(p->device);
  for (void *q : {p->d_row_ptr, static_cast<void *>(p->d_col), p->d_val,
                  static_cast<void *>(p->d_blocks), p->d_xstage, p->d_ystage,
                  p->d_lens, static_cast<void *>(p->d_cbase), p->d_partial,
                  static_cast<void *>(p->d_arrive), static_cast<void *>(p->d_dpart),
                  static_cast<void *>(p->d_cdesc), static_cast<void *>(p->d_ce), static_cast<void *>(p->d_cr), static_cast<void *>(p->d_segoff),
                  static_cast<void *>(p->d_pieces), static_cast<void *>(p->d_cont),
                  static_cast<void *>(p->d_col16), static_cast<void *>(p->d_perm), p->d_xg,
                  static_cast<void *>(p->d_carry), static_cast<void *>(p->d_gdst),
                  static_cast<void *>(p->d_rpieces)})
    if (q) (void)hipFree(q);
  for (hipEvent_t e : p->xt_ev)
    if (e) (void)hipEventDestroy(e);
  if (p->xt_s2) (void)hipStreamDestroy(p->xt_s2);
  delete p;
  return LHPC_OK;
}
