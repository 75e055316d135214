// lhpc_spmv_csr.hip — CSR SpMV kernels that keep the caller's CSR layout
// (y[i] = Σ_{k=row_ptr[i]}^{row_ptr[i+1]-1} val[k]·x[col_idx[k]]; the
// reference has no SpMV).  Numerics: fp64 accumulation in
// registers, one rounding at the store (SURVEY §8c binding recommendation).
//   ROWGROUP  L lanes per row (L | 64), R rows per lane group per wave, all
//             loads hoisted so a wave keeps R gathers + R val/col loads in
//             flight; the row sum is a DPP butterfly inside one 16-lane DPP
//             row for L <= 16 (no LDS), then one coalesced y store per wave.
//   ADAPTIVE  nnz-balanced row blocks: a 256-thread workgroup streams up to
//             kBlockNnz contiguous nonzeros (coalesced), stages fp64 products
//             in LDS, and reduces each row with L = 256/rows lanes; a row
//             longer than kBlockNnz gets a workgroup to itself.  For skewed
//             (power-law) row lengths.  Deterministic: fixed trees only.
//   SELL      short rows (≤ kSellMaxW nonzeros) with x locality: rows in
//             64-row slices, lane = row, entry j of every row of a slice
//             stored together (64 cols, then 64 vals, per j; padding col −1),
//             so the wave streams W coalesced col/val loads and keeps W
//             gathers in flight with no row_ptr, LDS or barrier.  Bit-
//             identical to ADAPTIVE on the same matrix: with ≤ 8 nonzeros per
//             row ADAPTIVE's blocks are 256 rows with one lane per row, which
//             adds the same products in the same order (a last block of ≤ 128
//             rows uses L lanes per row: SELL then sums in that order), and
//             the dot epilogue has the same tree.
// All read val/col_idx with non-temporal loads (streamed once) so the
// gathered x keeps its place in L2 / Infinity Cache.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "lhpc_spmv_impl.hpp"

namespace lhpc {
namespace {

constexpr int kBlockNnz = 2048;  // ADAPTIVE: nonzeros per stream block

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
// blocks[2b] = first row of block b, blocks[2b + 1] = its row_ptr;
// blocks[2·n_blocks] = n_rows, blocks[2·n_blocks + 1] = nnz.
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
  const int64_t r0 = blocks[2 * blockIdx.x], base = blocks[2 * blockIdx.x + 1];
  const int64_t r1 = blocks[2 * blockIdx.x + 2];
  const int64_t cnt = blocks[2 * blockIdx.x + 3] - base;
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
  // the reduce's row bounds (and the dot's w) are loaded with the stream,
  // not after the barrier: L lanes per row, L = the largest power of two
  // with nrows·L ≤ 256
  int L = kWave;
  while (L > 1 && nrows * L > kBlock) L >>= 1;
  const int grp = tid / L, sub = tid & (L - 1);
  int64_t rs = 0, re = 0;
  T wv = T(0);
  if (grp < nrows) {
    rs = static_cast<int64_t>(row_ptr[r0 + grp]) - base;
    re = static_cast<int64_t>(row_ptr[r0 + grp + 1]) - base;
    if (w && sub == 0) wv = w[r0 + grp];
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
  // reduce: L lanes per row
  double a = 0.0;
  if (grp < nrows)
    for (int64_t k = rs + sub; k < re; k += L) a += prod[k];
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
    if (w) d = static_cast<double>(yv) * static_cast<double>(wv);
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

// ------------------------------------------------------------- SELL
// x[c] for one nonzero of a SELL wave whose rows start at base: a column in
// [base, base + 64) comes from the lane holding x[base + lane] (`own`) by a
// lane shuffle, any other column is gathered.  The diagonal band of a
// row-local matrix then costs one coalesced load per wave instead of one
// gather instruction per band diagonal; the values are the same.
template <typename T>
__device__ __forceinline__ T sell_x(const T *__restrict__ x, int32_t c, int64_t base, T own) {
#ifdef LHPC_SELL_NO_SHFL
  return c >= 0 ? x[c] : T(0);
#else
  const uint64_t d = static_cast<uint64_t>(static_cast<int64_t>(c) - base);
  const bool loc = d < static_cast<uint64_t>(kWave);
  T v = __shfl(own, loc ? static_cast<int>(d) : 0, kWave);
  if (c >= 0 && !loc) v = x[c];
  return c >= 0 ? v : T(0);
#endif
}

// Device build of the SELL layout from device CSR (sell_build_device): row i
// (one thread) writes its entries to soff[i / 64] + 64·j + i % 64; padding
// was set beforehand (col −1, val 0).  V: the value's bit pattern.
template <typename V>
__global__ __launch_bounds__(kBlock) void k_sell_scatter(const void *__restrict__ rp, int bits,
                                                         const int32_t *__restrict__ col, const V *__restrict__ val,
                                                         const int64_t *__restrict__ soff, int64_t n_rows,
                                                         int32_t *__restrict__ ocol, V *__restrict__ oval) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n_rows;
       i += static_cast<int64_t>(gridDim.x) * kBlock) {
    const int64_t k0 = bits == 64 ? static_cast<const int64_t *>(rp)[i] : static_cast<const int32_t *>(rp)[i];
    const int64_t k1 = bits == 64 ? static_cast<const int64_t *>(rp)[i + 1] : static_cast<const int32_t *>(rp)[i + 1];
    const int64_t b = soff[i / kWave] + (i % kWave);
    for (int64_t j = 0; j < k1 - k0; ++j) {
      ocol[b + j * kWave] = col[k0 + j];
      oval[b + j * kWave] = val[k0 + j];
    }
  }
}

// The value ADAPTIVE computes for a row of ≤ 8 products p[] with L ≥ 2 lanes
// per row: lane s sums p[s], p[s + L], … from 0.0, then group_sum<L> pairs the
// lane sums as the tree (0+1)+(2+3)… (its butterfly steps are symmetric, so
// every lane holds that tree).  Lanes ≥ 8 hold 0.0, which adds nothing.
__device__ __forceinline__ double adaptive_lane_order(const double (&p)[kSellMaxW], int L) {
#pragma clang fp contract(off)
  if (L == 2) {
    const double q0 = ((p[0] + p[2]) + p[4]) + p[6], q1 = ((p[1] + p[3]) + p[5]) + p[7];
    return q0 + q1;
  }
  if (L == 4) return ((p[0] + p[4]) + (p[1] + p[5])) + ((p[2] + p[6]) + (p[3] + p[7]));
  return ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
}

// The block's y·w partial in ADAPTIVE's order (k_spmv_adaptive's epilogue):
// thread t holds row t's product d (0 past n_rows).  A full block has one
// ADAPTIVE lane per row — the same lanes, one wave tree per 64 rows, the
// four wave sums folded left.  A last block of nb ≤ 128 rows has L ≥ 2 lanes
// per row: ADAPTIVE's row r sits at lane r·L with zeros between, so its
// waves hold 64/L rows each; the products are moved to those lanes through
// LDS and summed the same way ((A0 + A1) + A2) + A3 (SELL's own waves would
// give (A0 + A1) + (A2 + A3)).
__device__ __forceinline__ void sell_dot_partial(double d, int64_t nb, double *wsum, double *dl, double *dpart) {
  int L = kWave;
  while (L > 1 && nb * L > kBlock) L >>= 1;  // block-uniform
  if (L > 1) {
    dl[threadIdx.x] = 0.0;
    __syncthreads();
    if (threadIdx.x < nb) dl[threadIdx.x * L] = d;
    __syncthreads();
    d = dl[threadIdx.x];
  }
  d = group_sum<kWave>(d);
  if ((threadIdx.x & (kWave - 1)) == 0) wsum[threadIdx.x / kWave] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = wsum[0];
#pragma unroll
    for (int i = 1; i < kBlock / kWave; ++i) t += wsum[i];
    dpart[blockIdx.x] = t;
  }
}

// soff[s] = first entry of slice s (a multiple of 64); its width is
// (soff[s + 1] − soff[s]) / 64 ≤ kSellMaxW.  One block = 4 slices = the
// 256 rows of ADAPTIVE's block blockIdx.x.
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_sell(const int32_t *__restrict__ col, const T *__restrict__ val,
                                                      const int64_t *__restrict__ soff, const T *__restrict__ x,
                                                      T *__restrict__ y, int64_t n_rows, int64_t n_cols,
                                                      const T *__restrict__ w, double *__restrict__ dpart) {
#pragma clang fp contract(off)  // the product rounds before the add, as ADAPTIVE's LDS-staged products do
  __shared__ double wsum[kBlock / kWave];
  __shared__ double dl[kBlock];
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t slice = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + threadIdx.x / kWave;
  const int64_t row = slice * kWave + lane;
  double a = 0.0;
  T wv = T(0);
  if (slice * kWave < n_rows) {  // wave-uniform
    const int64_t o0 = soff[slice];
    const int W = static_cast<int>((soff[slice + 1] - o0) / kWave);
    if (w && row < n_rows) wv = w[row];
    int32_t c[kSellMaxW];
    T v[kSellMaxW];
#pragma unroll
    for (int j = 0; j < kSellMaxW; ++j) {
      c[j] = -1;
      v[j] = T(0);
      if (j < W) {
        c[j] = ld_stream(col + o0 + j * kWave + lane);
        v[j] = ld_stream(val + o0 + j * kWave + lane);
      }
    }
    const int64_t base = slice * kWave;
    const T own = base + lane < n_cols ? x[base + lane] : T(0);
    T xv[kSellMaxW];
#pragma unroll
    for (int j = 0; j < kSellMaxW; ++j) xv[j] = sell_x(x, c[j], base, own);
    double pr[kSellMaxW];  // padding: 0·0 = 0, which adds nothing
#pragma unroll
    for (int j = 0; j < kSellMaxW; ++j) pr[j] = static_cast<double>(v[j]) * static_cast<double>(xv[j]);
    // ADAPTIVE's lanes per row in this block: 1 for every full block (256
    // rows); a last block of ≤ 128 rows gives L = 2 … 64 — sum in its order
    const int64_t nb = n_rows - static_cast<int64_t>(blockIdx.x) * kBlock;
    int L = kWave;
    while (L > 1 && nb * L > kBlock) L >>= 1;
    if (L == 1) {
#pragma unroll
      for (int j = 0; j < kSellMaxW; ++j)
        if (j < W) a += pr[j];
    } else {
      a = adaptive_lane_order(pr, L);
    }
  }
  const T yv = static_cast<T>(a);
  if (row < n_rows) y[row] = yv;
  if (w)  // block-uniform: ADAPTIVE's epilogue tree
    sell_dot_partial(row < n_rows ? static_cast<double>(yv) * static_cast<double>(wv) : 0.0,
                     n_rows - static_cast<int64_t>(blockIdx.x) * kBlock, wsum, dl, dpart);
}

// CG step on a SELL plan (lhpc_cg_solve): the previous iteration's
// x += α·p and p = r + β·p (k_cg_xp) fused into this iteration's q = A·p and
// p·q.  Every gathered p[c] is formed as r[c] + β·p_old[c] — the value k_cg_xp
// would have stored, so q, the dot and x are bit-identical to the unfused
// loop — and each row stores its own p (p_new: the other buffer; blocks
// still gather p_old) and x.  Saves k_cg_xp's pass over x, p, r (5n) for one
// more gathered vector (r) and the x / p stores (3n).
template <typename T>
__global__ __launch_bounds__(kBlock) void k_spmv_sell_cg(
    const int32_t *__restrict__ col, const T *__restrict__ val, const int64_t *__restrict__ soff,
    const T *__restrict__ r, const T *__restrict__ p_old, T *__restrict__ p_new, T *__restrict__ x,
    T *__restrict__ q, int64_t n_rows, const double *__restrict__ anum, const double *__restrict__ aden,
    const double *__restrict__ bnum, const double *__restrict__ bden, double *__restrict__ dpart) {
  __shared__ double wsum[kBlock / kWave];
  __shared__ double dl[kBlock];
  const T a = static_cast<T>(*anum / *aden);   // k_cg_xp's α and β
  const T beta = static_cast<T>(*bnum / *bden);
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t slice = static_cast<int64_t>(blockIdx.x) * (kBlock / kWave) + threadIdx.x / kWave;
  const int64_t row = slice * kWave + lane;
  double acc = 0.0;
  T pn = T(0);
  if (slice * kWave < n_rows) {  // wave-uniform
    const int64_t o0 = soff[slice];
    const int W = static_cast<int>((soff[slice + 1] - o0) / kWave);
    int32_t c[kSellMaxW];
    T v[kSellMaxW];
#pragma unroll
    for (int j = 0; j < kSellMaxW; ++j) {
      c[j] = -1;
      v[j] = T(0);
      if (j < W) {
        c[j] = ld_stream(col + o0 + j * kWave + lane);
        v[j] = ld_stream(val + o0 + j * kWave + lane);
      }
    }
    if (row < n_rows) {
      const T po = p_old[row];
      pn = r[row] + beta * po;
      x[row] = x[row] + a * po;
      p_new[row] = pn;
    }
    // the gathered p[c] = r[c] + β·p_old[c]: from the lane of row c when c
    // is one of this wave's rows (its pn: the same expression), else formed
    // from two gathers
    const int64_t base = slice * kWave;
    T pv[kSellMaxW];
#pragma unroll
    for (int j = 0; j < kSellMaxW; ++j) {
#ifdef LHPC_SELL_NO_SHFL
      pv[j] = c[j] >= 0 ? r[c[j]] + beta * p_old[c[j]] : T(0);
#else
      const uint64_t d = static_cast<uint64_t>(static_cast<int64_t>(c[j]) - base);
      const bool loc = d < static_cast<uint64_t>(kWave);
      T v = __shfl(pn, loc ? static_cast<int>(d) : 0, kWave);
      if (c[j] >= 0 && !loc) v = r[c[j]] + beta * p_old[c[j]];
      pv[j] = c[j] >= 0 ? v : T(0);
#endif
    }
    double pr[kSellMaxW];
#pragma unroll
    for (int j = 0; j < kSellMaxW; ++j) pr[j] = static_cast<double>(v[j]) * static_cast<double>(pv[j]);
    const int64_t nb = n_rows - static_cast<int64_t>(blockIdx.x) * kBlock;
    int L = kWave;
    while (L > 1 && nb * L > kBlock) L >>= 1;
    if (L == 1) {
#pragma unroll
      for (int j = 0; j < kSellMaxW; ++j)
        if (j < W) acc += pr[j];
    } else {
      acc = adaptive_lane_order(pr, L);
    }
  }
  const T yv = static_cast<T>(acc);
  if (row < n_rows) q[row] = yv;
  sell_dot_partial(row < n_rows ? static_cast<double>(yv) * static_cast<double>(pn) : 0.0,
                   n_rows - static_cast<int64_t>(blockIdx.x) * kBlock, wsum, dl, dpart);
}

template <typename T>
int launch_sell(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s, const void *w = nullptr,
                double *dpart = nullptr) {
  if (p->n_blocks == 0) return LHPC_OK;
  hipLaunchKernelGGL((k_spmv_sell<T>), dim3(static_cast<unsigned>(p->n_blocks)), dim3(kBlock), 0, s, p->d_col,
                     static_cast<const T *>(p->d_val), p->d_blocks, static_cast<const T *>(x), static_cast<T *>(y),
                     p->n_rows, p->n_cols, static_cast<const T *>(w), dpart);
  return check_launch(s);
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

// *dot_out = Σ of the plan's n_blocks dot partials (fixed order)
int dpart_finish(const lhpc_spmv_plan *p, int64_t n1, double *dot_out, hipStream_t s) {
  double *stage1 = p->d_dpart + p->n_blocks;
  if (n1 == 1) {
    hipLaunchKernelGGL(k_dpart_finish, dim3(1), dim3(kBlock), 0, s, p->d_dpart, p->n_blocks, dot_out);
  } else {
    hipLaunchKernelGGL(k_dpart_finish, dim3(static_cast<unsigned>(n1)), dim3(kBlock), 0, s, p->d_dpart,
                       p->n_blocks, stage1);
    LHPC_TRY(check_launch(s));
    hipLaunchKernelGGL(k_dpart_finish, dim3(1), dim3(kBlock), 0, s, stage1, n1, dot_out);
  }
  return check_launch(s);
}

}  // namespace

// Row blocks for ADAPTIVE: greedy, each block <= kBlockNnz nonzeros and
// <= kBlock rows, or a single row of any length.
std::vector<int64_t> csr_build_blocks(RowPtrView rp, int64_t n_rows, int64_t &n_long) {
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

// SELL layout (see k_spmv_sell): LHPC_ERR_UNSUPPORTED when a row has more
// than kSellMaxW nonzeros, or (auto) when the padding would stream more
// bytes than CSR with its row_ptr.  Sets kernel, n_blocks (256-row blocks,
// ADAPTIVE's own for such rows) and d_blocks = the slice offsets.
// Slice offsets of the SELL layout (host): off[s] = first entry of slice s,
// off[S] = entries stored; LHPC_ERR_UNSUPPORTED past kSellMaxW nonzeros in a
// row, or (not forced) when the padded slices would stream more bytes than
// CSR with its row_ptr.
static int sell_offsets(RowPtrView rp, int64_t n, int64_t nnz, size_t tsz, bool forced, std::vector<int64_t> &off,
                        int &wmax) {
  const int64_t S = (n + kWave - 1) / kWave;
  off.assign(static_cast<size_t>(S) + 1, 0);
  wmax = 0;
  for (int64_t s = 0; s < S; ++s) {
    int64_t W = 0;
    for (int64_t i = s * kWave; i < std::min(n, (s + 1) * kWave); ++i) W = std::max(W, rp[i + 1] - rp[i]);
    if (W > kSellMaxW) return LHPC_ERR_UNSUPPORTED;
    wmax = std::max(wmax, static_cast<int>(W));
    off[static_cast<size_t>(s) + 1] = off[static_cast<size_t>(s)] + W * kWave;
  }
  const double sell_b = static_cast<double>(off[static_cast<size_t>(S)]) * static_cast<double>(4 + tsz) +
                        8.0 * static_cast<double>(S);
  const double csr_b = static_cast<double>(nnz) * static_cast<double>(4 + tsz) + 4.0 * static_cast<double>(n + 1);
  return !forced && sell_b > csr_b ? LHPC_ERR_UNSUPPORTED : LHPC_OK;
}

static int sell_finish(lhpc_spmv_plan *p, const std::vector<int64_t> &off, int wmax) {
  LHPC_HIP_TRY(hipMemcpy(p->d_blocks, off.data(), off.size() * 8, hipMemcpyHostToDevice));
  p->kernel = LHPC_KERNEL_SELL;
  p->n_blocks = (p->n_rows + kBlock - 1) / kBlock;
  p->n_long = 0;
  p->sell_w = wmax;
  return LHPC_OK;
}

int sell_build(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz, bool forced) {
  const int64_t n = p->n_rows;
  std::vector<int64_t> off;
  int wmax = 0;
  LHPC_TRY(sell_offsets(rp, n, p->nnz, tsz, forced, off, wmax));
  const int64_t total = off.back();
  std::vector<int32_t> c(static_cast<size_t>(total), -1);
  std::vector<unsigned char> v(static_cast<size_t>(total) * tsz, 0);
  const unsigned char *vin = static_cast<const unsigned char *>(val);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t b = off[static_cast<size_t>(i / kWave)] + (i % kWave), k0 = rp[i], len = rp[i + 1] - k0;
    for (int64_t j = 0; j < len; ++j) {
      c[static_cast<size_t>(b + j * kWave)] = col_idx[k0 + j];
      std::memcpy(&v[static_cast<size_t>(b + j * kWave) * tsz], vin + static_cast<size_t>(k0 + j) * tsz, tsz);
    }
  }
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_col), static_cast<size_t>(total) * 4, p->bytes));
  LHPC_TRY(dmalloc(&p->d_val, static_cast<size_t>(total) * tsz, p->bytes));
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_blocks), off.size() * 8, p->bytes));
  if (total) {
    LHPC_HIP_TRY(hipMemcpy(p->d_col, c.data(), c.size() * 4, hipMemcpyHostToDevice));
    LHPC_HIP_TRY(hipMemcpy(p->d_val, v.data(), v.size(), hipMemcpyHostToDevice));
  }
  return sell_finish(p, off, wmax);
}

int sell_build_device(lhpc_spmv_plan *p, RowPtrView rp_host, const void *d_rp, const int32_t *d_col,
                      const void *d_val, size_t tsz, bool forced) {
  const int64_t n = p->n_rows;
  std::vector<int64_t> off;
  int wmax = 0;
  LHPC_TRY(sell_offsets(rp_host, n, p->nnz, tsz, forced, off, wmax));
  const int64_t total = off.back();
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_col), static_cast<size_t>(total) * 4, p->bytes));
  LHPC_TRY(dmalloc(&p->d_val, static_cast<size_t>(total) * tsz, p->bytes));
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_blocks), off.size() * 8, p->bytes));
  LHPC_TRY(sell_finish(p, off, wmax));  // the slice offsets, which the scatter reads
  if (total) {
    LHPC_HIP_TRY(hipMemsetD32(reinterpret_cast<hipDeviceptr_t>(p->d_col), -1, static_cast<size_t>(total)));
    LHPC_HIP_TRY(hipMemset(p->d_val, 0, static_cast<size_t>(total) * tsz));
    const unsigned grid = static_cast<unsigned>(std::min<int64_t>((n + kBlock - 1) / kBlock, 65536));
    if (tsz == 4)
      hipLaunchKernelGGL((k_sell_scatter<uint32_t>), dim3(grid), dim3(kBlock), 0, nullptr, d_rp, rp_host.bits, d_col,
                         static_cast<const uint32_t *>(d_val), p->d_blocks, n, p->d_col,
                         static_cast<uint32_t *>(p->d_val));
    else
      hipLaunchKernelGGL((k_sell_scatter<uint64_t>), dim3(grid), dim3(kBlock), 0, nullptr, d_rp, rp_host.bits, d_col,
                         static_cast<const uint64_t *>(d_val), p->d_blocks, n, p->d_col,
                         static_cast<uint64_t *>(p->d_val));
    LHPC_HIP_TRY(hipGetLastError());
    LHPC_HIP_TRY(hipDeviceSynchronize());
  }
  return LHPC_OK;
}

int csr_launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  const bool f32 = p->dtype == LHPC_F32;
  if (p->kernel == LHPC_KERNEL_SELL) return f32 ? launch_sell<float>(p, x, y, s) : launch_sell<double>(p, x, y, s);
  if (p->kernel == LHPC_KERNEL_ADAPTIVE)
    return f32 ? (p->rp64 ? launch_adaptive<float, int64_t>(p, x, y, s) : launch_adaptive<float, int32_t>(p, x, y, s))
               : (p->rp64 ? launch_adaptive<double, int64_t>(p, x, y, s) : launch_adaptive<double, int32_t>(p, x, y, s));
  return f32 ? (p->rp64 ? launch_rowgroup<float, int64_t>(p, x, y, s) : launch_rowgroup<float, int32_t>(p, x, y, s))
             : (p->rp64 ? launch_rowgroup<double, int64_t>(p, x, y, s) : launch_rowgroup<double, int32_t>(p, x, y, s));
}

int csr_launch_dot(lhpc_spmv_plan *p, const void *x, void *y, const void *w, double *dot_out, hipStream_t s) {
  if ((p->kernel != LHPC_KERNEL_ADAPTIVE && p->kernel != LHPC_KERNEL_SELL) || p->n_blocks == 0)
    return LHPC_ERR_UNSUPPORTED;
  const int64_t n1 = (p->n_blocks + kFinTile - 1) / kFinTile;  // stage-1 sums, after the partials
  if (n1 > kFinTile) return LHPC_ERR_UNSUPPORTED;                // > 4M blocks (> 8·10^9 nonzeros)
  if (!p->d_dpart)
    LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_dpart), (p->n_blocks + n1) * sizeof(double), p->bytes));
  int st;
  if (p->kernel == LHPC_KERNEL_SELL)
    st = p->dtype == LHPC_F32 ? launch_sell<float>(p, x, y, s, w, p->d_dpart)
                              : launch_sell<double>(p, x, y, s, w, p->d_dpart);
  else if (p->dtype == LHPC_F32)
    st = p->rp64 ? launch_adaptive<float, int64_t>(p, x, y, s, w, p->d_dpart)
                 : launch_adaptive<float, int32_t>(p, x, y, s, w, p->d_dpart);
  else
    st = p->rp64 ? launch_adaptive<double, int64_t>(p, x, y, s, w, p->d_dpart)
                 : launch_adaptive<double, int32_t>(p, x, y, s, w, p->d_dpart);
  LHPC_TRY(st);
  return dpart_finish(p, n1, dot_out, s);
}

int sell_cg_step(lhpc_spmv_plan *p, const void *r, const void *p_old, void *p_new, void *x, void *q,
                 const double *anum, const double *aden, const double *bnum, const double *bden, double *pq,
                 hipStream_t s) {
  if (p->kernel != LHPC_KERNEL_SELL || p->n_blocks == 0) return LHPC_ERR_UNSUPPORTED;
  const int64_t n1 = (p->n_blocks + kFinTile - 1) / kFinTile;
  if (n1 > kFinTile) return LHPC_ERR_UNSUPPORTED;
  if (!p->d_dpart)
    LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_dpart), (p->n_blocks + n1) * sizeof(double), p->bytes));
  if (p->dtype == LHPC_F32)
    hipLaunchKernelGGL((k_spmv_sell_cg<float>), dim3(static_cast<unsigned>(p->n_blocks)), dim3(kBlock), 0, s,
                       p->d_col, static_cast<const float *>(p->d_val), p->d_blocks, static_cast<const float *>(r),
                       static_cast<const float *>(p_old), static_cast<float *>(p_new), static_cast<float *>(x),
                       static_cast<float *>(q), p->n_rows, anum, aden, bnum, bden, p->d_dpart);
  else
    hipLaunchKernelGGL((k_spmv_sell_cg<double>), dim3(static_cast<unsigned>(p->n_blocks)), dim3(kBlock), 0, s,
                       p->d_col, static_cast<const double *>(p->d_val), p->d_blocks, static_cast<const double *>(r),
                       static_cast<const double *>(p_old), static_cast<double *>(p_new), static_cast<double *>(x),
                       static_cast<double *>(q), p->n_rows, anum, aden, bnum, bden, p->d_dpart);
  LHPC_TRY(check_launch(s));
  return dpart_finish(p, n1, pq, s);
}

}  // namespace lhpc
