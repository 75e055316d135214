// lhpc_spmv_xslice.hip — XSLICE: column-sliced CSR SpMV (DESIGN.md §4
// XSLICE; selected by LHPC_PLAN_FORCE_XSLICE or LHPC_SPMV_XTILE=0 — XTILE is
// the default for gathers without locality).  Slice s = g + 8·phase is
// processed by the blocks with blockIdx % 8 == g (the blocks the dispatcher
// deals to one XCD), phase after phase, so each XCD's L2 holds one x slice
// (≈ 2.5–5 MB) and the random x gathers hit L2 instead of Infinity Cache /
// HBM (measured: 151–168 G gathers/s vs 59 unsliced, tools/probe_slices.py).
// Placement is a speed heuristic only: any block→XCD mapping gives the same
// result.  Each slice stores one partial per row; k_xslice_reduce adds the S
// partials in slice order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "lhpc_plan.hpp"
#include "lhpc_spmv_impl.hpp"

namespace lhpc {
namespace {

constexpr int kLongRow = 48;  // in-slice rows longer than this are wave-reduced

// One wave owns a 64-row chunk of one slice: the chunk's in-slice nonzeros
// are in CSR order and the whole wave streams them NB·64 at a time — every lane loads / gathers (full lane utilisation,
// NB gathers in flight per lane) — staging exact fp64 products in a
// wave-private LDS window; lane r then adds its row's products in CSR order.
// Row offsets inside the chunk come from a wave prefix sum of the uint8
// lengths.  A chunk with more than NB·64 nonzeros loops over windows (rows
// spanning windows keep accumulating in order, so the result is unchanged).
template <typename T, typename P, typename LT, int NB>
__device__ __forceinline__ void xslice_block(
    const LT *__restrict__ lens, const int64_t *__restrict__ cbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, const T *__restrict__ x,
    P *__restrict__ partial, int64_t n_rows, int64_t n_rows_pad, int64_t n_chunks,
    int64_t blocks_per_slice, int S, int64_t b, double (*prod)[NB * kWave]) {
  constexpr int CAP = NB * kWave;
  (void)CAP;
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
  if (s >= S || chunk >= n_chunks) return;  // wave-uniform (this logical block only)
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

template <typename T, typename P, typename LT, int NB>
__global__ __launch_bounds__(kBlock) void k_spmv_xslice_stream(
    const LT *__restrict__ lens, const int64_t *__restrict__ cbase,
    const int32_t *__restrict__ col, const T *__restrict__ val, const T *__restrict__ x,
    P *__restrict__ partial, int64_t n_rows, int64_t n_rows_pad, int64_t n_chunks,
    int64_t blocks_per_slice, int S, int64_t n_blocks) {
  constexpr int CAP = NB * kWave;
  __shared__ double prod[kBlock / kWave][CAP];
  // grid-stride over the logical blocks: a dispatch holds < 2^32 work-items,
  // and at n = 80M the slice grid alone is 20M blocks (5.1e9 work-items)
  for (int64_t b = blockIdx.x; b < n_blocks; b += gridDim.x)
    xslice_block<T, P, LT, NB>(lens, cbase, col, val, x, partial, n_rows, n_rows_pad, n_chunks, blocks_per_slice, S,
                               b, prod);
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

template <typename T>
int launch_xslice(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  if (p->n_rows == 0) return LHPC_OK;
  const int64_t grid = p->S >= 8 ? 8 * (p->S / 8) * p->xs_bps : p->S * p->xs_bps;
  // ≤ 2^20 workgroups per dispatch (a multiple of 8, so each XCD keeps its
  // slices); the kernel strides over the rest
  const dim3 g(static_cast<unsigned>(std::min<int64_t>(grid, int64_t{1} << 20))), blk(kBlock);
  const T *xv = static_cast<const T *>(x);
  const T *vv = static_cast<const T *>(p->d_val);
#define LHPC_XS_STREAM(P, NB)                                                                        \
  if (p->xs_lens16)                                                                                  \
    hipLaunchKernelGGL((k_spmv_xslice_stream<T, P, uint16_t, NB>), g, blk, 0, s,                      \
                       static_cast<const uint16_t *>(p->d_lens), p->d_cbase, p->d_col, vv, xv,         \
                       static_cast<P *>(p->d_partial), p->n_rows, p->xs_rows_pad, p->xs_chunks,        \
                       p->xs_bps, p->S, grid);                                                        \
  else                                                                                               \
    hipLaunchKernelGGL((k_spmv_xslice_stream<T, P, uint8_t, NB>), g, blk, 0, s,                       \
                       static_cast<const uint8_t *>(p->d_lens), p->d_cbase, p->d_col, vv, xv,          \
                       static_cast<P *>(p->d_partial), p->n_rows, p->xs_rows_pad, p->xs_chunks,        \
                       p->xs_bps, p->S, grid)
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
  LHPC_TRY(check_launch(s));
  const int64_t rgrid = (p->n_rows + 4 * kBlock - 1) / (4 * kBlock);
  const dim3 rg(static_cast<unsigned>(rgrid));
  if (p->xs_p64)
    hipLaunchKernelGGL((k_xslice_reduce<T, double>), rg, blk, 0, s, static_cast<const double *>(p->d_partial),
                       static_cast<T *>(y), p->n_rows, p->xs_rows_pad, p->S);
  else
    hipLaunchKernelGGL((k_xslice_reduce<T, T>), rg, blk, 0, s, static_cast<const T *>(p->d_partial),
                       static_cast<T *>(y), p->n_rows, p->xs_rows_pad, p->S);
  return check_launch(s);
}

}  // namespace

int xslice_launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  return p->dtype == LHPC_F32 ? launch_xslice<float>(p, x, y, s) : launch_xslice<double>(p, x, y, s);
}

// S = 8·P slices of width ⌈n_cols/S⌉, P chosen so one slice of x is ≤ 5 MB
// (LHPC_XSLICE_MB / LHPC_XSLICE_S override); partials in the value type
// (fp32: one extra rounding per partial, ≤ 2^-23·Σ|a·x|) or in
// fp64 (fp64 data, or LHPC_PLAN_EXACT_PARTIALS).
int xslice_build(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz,
                 unsigned flags) {
  const int64_t nnz = p->nnz;
  const double x_bytes = static_cast<double>(p->n_cols) * static_cast<double>(tsz);
  const double slice_mb = p->opt.xslice_mb > 0 ? std::max(0.25, p->opt.xslice_mb) : 5.0;
  int P = static_cast<int>(std::ceil(x_bytes / (8.0 * slice_mb * 1.0e6)));
  P = std::max(1, std::min(P, 32));
  int S = 8 * P;
  if (p->opt.xslice_slices > 0) S = std::min(256, p->opt.xslice_slices);
  if (S > 8) S = (S + 7) / 8 * 8;
  XsliceHost xs;
  LHPC_TRY(build_xslice(rp.p, rp.bits, col_idx, val, tsz, p->n_rows, p->n_cols, S, xs));
  p->kernel = LHPC_KERNEL_XSLICE;
  p->S = S;
  p->xs_p64 = (tsz == 8 || ((flags & LHPC_PLAN_EXACT_PARTIALS) && !(flags & LHPC_PLAN_FAST_PARTIALS))) ? 1 : 0;
  if (p->opt.xslice_partial > 0) p->xs_p64 = tsz == 8 || p->opt.xslice_partial == 2;
  {  // window = NB·64 nonzeros: cover a typical chunk in one window
    const double mean_chunk = xs.n_chunks ? static_cast<double>(nnz) / (static_cast<double>(S) * xs.n_chunks) : 0;
    int nb = static_cast<int>(std::ceil(mean_chunk * 1.2 / kWave));
    if (p->opt.xslice_window > 0) nb = p->opt.xslice_window;
    p->xs_nb = std::max(1, std::min(nb, 4));
  }
  p->xs_width = xs.width;
  p->xs_chunks = xs.n_chunks;
  p->xs_rows_pad = xs.n_rows_pad;
  p->xs_bps = (xs.n_chunks + (kBlock / kWave) - 1) / (kBlock / kWave);
  const size_t lb = static_cast<size_t>(S) * xs.n_rows_pad;
  const size_t cb = (static_cast<size_t>(S) * xs.n_chunks + 1) * 8;
  p->xs_lens16 = xs.lens_bytes == 2 ? 1 : 0;
  LHPC_TRY(dmalloc(&p->d_lens, lb * xs.lens_bytes, p->bytes));
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_cbase), cb, p->bytes));
  LHPC_TRY(dmalloc(reinterpret_cast<void **>(&p->d_col), static_cast<size_t>(nnz) * 4, p->bytes));
  LHPC_TRY(dmalloc(&p->d_val, static_cast<size_t>(nnz) * tsz, p->bytes));
  LHPC_TRY(dmalloc(&p->d_partial, lb * (p->xs_p64 ? 8 : tsz), p->bytes));
  LHPC_HIP_TRY(hipMemcpy(p->d_lens, xs.lens.get(), lb * xs.lens_bytes, hipMemcpyHostToDevice));
  LHPC_HIP_TRY(hipMemcpy(p->d_cbase, xs.cbase.get(), cb, hipMemcpyHostToDevice));
  LHPC_HIP_TRY(hipMemcpy(p->d_col, xs.col.get(), static_cast<size_t>(nnz) * 4, hipMemcpyHostToDevice));
  LHPC_HIP_TRY(hipMemcpy(p->d_val, xs.val.get(), static_cast<size_t>(nnz) * tsz, hipMemcpyHostToDevice));
  return LHPC_OK;
}

}  // namespace lhpc
