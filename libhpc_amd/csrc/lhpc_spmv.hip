// lhpc_spmv.hip — CSR SpMV y = A·x for gfx950 (MI355X), behind include/lhpc.h:
// plan creation (validation, kernel selection, the family builders) and the
// C ABI.  The kernels live in lhpc_spmv_{csr,xslice,xtile}.hip
// (lhpc_spmv_impl.hpp).
//
// The reference has no SpMV; the operator is defined
// here as y[i] = Σ_{k=row_ptr[i]}^{row_ptr[i+1]-1} val[k]·x[col_idx[k]].
// Numerics: every dtype accumulates in fp64 registers and rounds once at the
// store (SURVEY §8c "binding recommendation"), so fp32 results are within
// 2^-24·|y| + ~1e-16·Σ|a·x| of the exact sum for any row length.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <new>
#include <vector>

#include "lhpc_plan.hpp"
#include "lhpc_spmv_impl.hpp"

namespace lhpc {
namespace {

// Distinct 128-B x lines touched per nonzero, over up to 32 evenly spaced
// chunks of 8192 consecutive rows (1.0 = no reuse within a chunk).
// fetch(k0, k1, out): the columns of nonzeros [k0, k1) (host array or a copy
// from device-resident input)
template <typename RP, typename Fetch>
double gather_lines_per_nnz(const RP &rp, Fetch fetch, int64_t n_rows, int64_t n_cols, size_t tsz) {
  constexpr int64_t kChunk = 8192, kSamples = 32;
  const int shift = tsz == 8 ? 4 : 5;  // 16 doubles / 32 floats per line
  const int64_t chunks = (n_rows + kChunk - 1) / kChunk;
  const int64_t step = std::max<int64_t>(1, chunks / kSamples);
  int64_t lines = 0, nz = 0;
  std::vector<int32_t> buf;
  // distinct lines per sample with a bitmap over x's lines (set, count, then
  // clear what was set): O(nonzeros) where a sort + unique cost ≈ 0.2 s for C2
  std::vector<uint64_t> seen(static_cast<size_t>(((n_cols >> shift) + 64) / 64), 0);
  for (int64_t c = 0; c < chunks; c += step) {
    const int64_t r0 = c * kChunk, r1 = std::min(n_rows, r0 + kChunk);
    const int64_t k0 = rp[r0], k1 = rp[r1];
    buf.resize(static_cast<size_t>(k1 - k0));
    if (k1 > k0 && fetch(k0, k1, buf.data()) != LHPC_OK) return 1.0;
    for (const int32_t v : buf) {
      const uint64_t l = static_cast<uint64_t>(v) >> shift, bit = uint64_t{1} << (l & 63);
      uint64_t &w = seen[static_cast<size_t>(l >> 6)];
      lines += (w & bit) ? 0 : 1;
      w |= bit;
    }
    for (const int32_t v : buf) seen[static_cast<size_t>((static_cast<uint64_t>(v) >> shift) >> 6)] = 0;
    nz += k1 - k0;
  }
  return nz ? static_cast<double>(lines) / static_cast<double>(nz) : 1.0;
}

// device CSR checks for LHPC_PLAN_DEVICE_INPUT (validate_csr on the GPU):
// bit 0: row_ptr[0] != 0, decreasing, or row_ptr[n_rows] != nnz; bit 1: a
// column outside [0, n_cols)
__global__ void k_validate_device_csr(const void *rp, int bits, const int32_t *col, int64_t n_rows, int64_t n_cols,
                                      int64_t nnz, unsigned *flag) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x, T = static_cast<int64_t>(gridDim.x) * blockDim.x;
  auto at = [&](int64_t i) -> int64_t {
    return bits == 64 ? static_cast<const int64_t *>(rp)[i] : static_cast<const int32_t *>(rp)[i];
  };
  unsigned bad = 0;
  for (int64_t i = t; i < n_rows; i += T)
    if (at(i + 1) < at(i)) bad |= 1u;
  if (t == 0 && (at(0) != 0 || at(n_rows) != nnz)) bad |= 1u;
  for (int64_t k = t; k < nnz; k += T)
    if (col[k] < 0 || col[k] >= n_cols) bad |= 2u;
  if (bad) atomicOr(flag, bad);
}

// XTILE column blocks from device-resident CSR (build_parts with d_rp):
// rows [r0, r0 + nr) restricted to columns [c0, c1), rebased — the device
// twin of lhpc_plan.cpp csr_column_block (count per row, host scan, scatter)
__device__ __forceinline__ int64_t rp_dev(const void *rp, int bits, int64_t i) {
  return bits == 64 ? static_cast<const int64_t *>(rp)[i] : static_cast<const int32_t *>(rp)[i];
}
__global__ void k_colblock_count(const void *rp, int bits, const int32_t *col, int64_t r0, int64_t nr, int32_t c0,
                                 int32_t c1, int32_t *cnt) {
  const int64_t T = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < nr; r += T) {
    int32_t c = 0;
    for (int64_t k = rp_dev(rp, bits, r0 + r), e = rp_dev(rp, bits, r0 + r + 1); k < e; ++k)
      c += col[k] >= c0 && col[k] < c1;
    cnt[r] = c;
  }
}
template <typename T>
__global__ void k_colblock_scatter(const void *rp, int bits, const int32_t *col, const T *val, int64_t r0, int64_t nr,
                                   int32_t c0, int32_t c1, const int64_t *orp, int32_t *ocol, T *oval) {
  const int64_t G = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t r = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; r < nr; r += G) {
    int64_t o = orp[r];
    for (int64_t k = rp_dev(rp, bits, r0 + r), e = rp_dev(rp, bits, r0 + r + 1); k < e; ++k)
      if (col[k] >= c0 && col[k] < c1) {
        ocol[o] = col[k] - c0;
        oval[o] = val[k];
        ++o;
      }
  }
}

// one column block on the device: host row offsets in orp, device col/val in
// the returned buffers (freed by the caller)
int colblock_device(const void *d_rp, int bits, const int32_t *d_col, const void *d_val, size_t tsz, int64_t r0,
                    int64_t r1, int64_t c0, int64_t c1, std::vector<int64_t> &orp, void **d_ocol, void **d_oval) {
  const int64_t nr = r1 - r0;
  *d_ocol = *d_oval = nullptr;
  orp.assign(static_cast<size_t>(nr) + 1, 0);
  std::vector<int32_t> cnt(static_cast<size_t>(nr));
  int32_t *d_cnt = nullptr;
  int64_t *d_orp = nullptr;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(&d_cnt), static_cast<size_t>(std::max<int64_t>(nr, 1)) * 4);
  const unsigned grid = static_cast<unsigned>(std::min<int64_t>((nr + 255) / 256 + 1, 8192));
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_colblock_count, dim3(grid), dim3(256), 0, nullptr, d_rp, bits, d_col, r0, nr,
                       static_cast<int32_t>(c0), static_cast<int32_t>(c1), d_cnt);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(cnt.data(), d_cnt, static_cast<size_t>(nr) * 4, hipMemcpyDeviceToHost);
  (void)hipFree(d_cnt);
  if (e != hipSuccess) return static_cast<int>(e);
  for (int64_t r = 0; r < nr; ++r) orp[static_cast<size_t>(r) + 1] = orp[static_cast<size_t>(r)] + cnt[static_cast<size_t>(r)];
  const int64_t m = orp[static_cast<size_t>(nr)];
  if (m == 0) return LHPC_OK;
  e = hipMalloc(&d_orp, static_cast<size_t>(nr + 1) * 8);
  if (e == hipSuccess) e = hipMemcpy(d_orp, orp.data(), static_cast<size_t>(nr + 1) * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(d_ocol, static_cast<size_t>(m) * 4);
  if (e == hipSuccess) e = hipMalloc(d_oval, static_cast<size_t>(m) * tsz);
  if (e == hipSuccess) {
    if (tsz == 4)
      hipLaunchKernelGGL(k_colblock_scatter<float>, dim3(grid), dim3(256), 0, nullptr, d_rp, bits, d_col,
                         static_cast<const float *>(d_val), r0, nr, static_cast<int32_t>(c0), static_cast<int32_t>(c1),
                         d_orp, static_cast<int32_t *>(*d_ocol), static_cast<float *>(*d_oval));
    else
      hipLaunchKernelGGL(k_colblock_scatter<double>, dim3(grid), dim3(256), 0, nullptr, d_rp, bits, d_col,
                         static_cast<const double *>(d_val), r0, nr, static_cast<int32_t>(c0), static_cast<int32_t>(c1),
                         d_orp, static_cast<int32_t *>(*d_ocol), static_cast<double *>(*d_oval));
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipFree(d_orp);
  return static_cast<int>(e);
}

bool is_gfx950(int dev) {
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return false;
  return std::strncmp(p.gcnArchName, "gfx950", 6) == 0;
}

int launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s) {
  if (!p->parts.empty()) {
    const size_t tsz = p->dtype == LHPC_F32 ? 4 : 8;
    for (size_t i = 0; i < p->parts.size(); ++i)
      LHPC_TRY(xtile_launch(p->parts[i], static_cast<const unsigned char *>(x) + p->part_col[i] * tsz,
                            static_cast<unsigned char *>(y) + p->part_row[i] * tsz, s));
    return LHPC_OK;
  }
  if (p->kernel == LHPC_KERNEL_XTILE) return xtile_launch(p, x, y, s);
  if (p->kernel == LHPC_KERNEL_XSLICE) return xslice_launch(p, x, y, s);
  return csr_launch(p, x, y, s);
}

// XTILE column blocks (lhpc_options.xtile_col_blocks).  A reduce chunk holds
// M nonzeros and meets every one of the S tiles, so its segment per tile is
// M/S nonzeros: 32 for C2 (S = 256), 4 at n = 80M (S = 2048), and the
// reduce's cost per nonzero grows with S (DESIGN.md §4 "large n": 632 GFLOP/s
// at S = 256, 533 at 768, 408 at 1024, 244 at 2048).  Cutting the columns into
// B blocks gives each block's plan S/B tiles; the blocks run in turn on x's
// column ranges, every block after the first adding into y.  A chunk also
// holds ≤ M/8 rows, so as a block's rows get shorter its chunks shrink with
// the blocks.  Same box, fp32 15 per row, forced B (profiles/r04/col_blocks):
// n = 10M (256 tiles) B = 1 / 2: 601 / 534 GFLOP/s; 40M (1024) B = 2 / 3 /
// 4: 498 / 446 / 426; 80M (2048) B = 2 / 3 / 4 / 6: 378 / 417 / 365 / 314;
// 150M (3840, two row parts) B = 2 / 3 / 4: 316 / 371 / 342.  fp64 10M (489)
// B = 1 / 2: 318 / 304; 40M (1954) B = 2 / 3 / 4 / 6: 264 / 261 / 230 / 180.
// Hence B = ⌈S / 768⌉, at most mean row length / 5.
constexpr int64_t kColBlockTiles = 768;
int xtile_col_blocks_for(int64_t n_rows, int64_t n_cols, int64_t nnz, size_t tsz, const lhpc_options &o) {
  const int64_t most = std::max<int64_t>(1, n_cols / 64);  // ≥ 64 columns per block
  if (o.xtile_col_blocks > 0) return static_cast<int>(std::min<int64_t>(o.xtile_col_blocks, most));
  const int64_t W = tsz == 4 ? 40960 : 20480, S = (n_cols + W - 1) / W;
  if (S <= kColBlockTiles || n_rows <= 0) return 1;
  const double mean = static_cast<double>(nnz) / static_cast<double>(n_rows);
  const int64_t bmax = std::max<int64_t>(1, static_cast<int64_t>(mean / 5.0));
  return static_cast<int>(std::min({(S + kColBlockTiles - 1) / kColBlockTiles, bmax, most}));
}

// XTILE row parts: the tile stream of one plan is addressed with int32
// offsets (nnz + 8 padding entries per tile < 2^31, lhpc_plan.cpp
// build_xtile).  A larger matrix (n ≳ 143M rows at 15 nonzeros per row) is
// cut into nnz-balanced row parts of ≤ cap nonzeros, each an ordinary XTILE
// plan over its rows (row_ptr rebased, the caller's col/val at the part's
// offset) run in turn on the same x, instead of dropping to XSLICE.  With
// B > 1 column blocks every row part is further cut by column (above).
// LHPC_ERR_UNSUPPORTED when some single row exceeds the cap.
// d_rp non-null: device input (col_idx / val and d_rp in HBM, rp a host copy
// of row_ptr): every part's layout is built on the GPU (xtile_build_device).
int build_parts(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz,
                int64_t cap, int B, const void *d_rp = nullptr) {
  const int64_t n_rows = p->n_rows;
  int64_t n_parts = std::max<int64_t>(1, (p->nnz + cap - 1) / cap);
  std::vector<int64_t> cuts;
  for (;; ++n_parts) {  // nnz-balanced cuts; one more part until every part fits
    cuts.assign(static_cast<size_t>(n_parts) + 1, 0);
    LHPC_TRY(lhpc_csr_partition_rows(rp.p, rp.bits, n_rows, static_cast<int>(n_parts), cuts.data()));
    bool fit = true;
    for (int64_t i = 0; i < n_parts && fit; ++i) {
      const int64_t r0 = cuts[i], r1 = cuts[i + 1];
      if (r1 - r0 == 1 && rp[r1] - rp[r0] > cap) return LHPC_ERR_UNSUPPORTED;  // one row past the cap
      fit = rp[r1] - rp[r0] <= cap;
    }
    if (fit) break;
    if (n_parts > n_rows) return LHPC_ERR_UNSUPPORTED;
  }
  // column block bounds, 64-column aligned (x + bound stays 256-B aligned)
  std::vector<int64_t> cb(static_cast<size_t>(B) + 1, p->n_cols);
  for (int b = 0; b < B; ++b) cb[b] = p->n_cols * b / B / 64 * 64;
  auto add = [&](int64_t r0, int64_t r1, int64_t c0, int64_t c1, RowPtrView lrp, const int32_t *lc, const void *lv,
                 int64_t lnnz, int acc) -> int {
    auto *q = new (std::nothrow) lhpc_spmv_plan();
    if (!q) return LHPC_ERR_ALLOC;
    p->parts.push_back(q);
    p->part_row.push_back(r0);
    p->part_col.push_back(c0);
    q->opt = p->opt;
    q->dtype = p->dtype;
    q->device = p->device;
    q->n_rows = r1 - r0;
    q->n_cols = c1 - c0;
    q->nnz = lnnz;
    q->xt_acc = acc;
    LHPC_TRY(d_rp ? xtile_build_device(q, lrp, lc, lv, tsz) : xtile_build(q, lrp, lc, lv, tsz));
    p->bytes += q->bytes;
    return LHPC_OK;
  };
  std::vector<int64_t> lrp;
  std::vector<int32_t> lcol;
  std::vector<unsigned char> lval;
  for (int64_t i = 0; i < n_parts; ++i) {
    const int64_t r0 = cuts[i], r1 = cuts[i + 1];
    if (r1 == r0) continue;
    const int64_t e0 = rp[r0];
    if (B == 1 || rp[r1] == e0) {
      lrp.resize(static_cast<size_t>(r1 - r0 + 1));
      for (int64_t r = r0; r <= r1; ++r) lrp[static_cast<size_t>(r - r0)] = rp[r] - e0;
      LHPC_TRY(add(r0, r1, 0, p->n_cols, RowPtrView{lrp.data(), 64}, col_idx + e0,
                   static_cast<const unsigned char *>(val) + e0 * static_cast<int64_t>(tsz), rp[r1] - e0, 0));
      continue;
    }
    bool first = true;  // the first non-empty block stores every row of the part
    for (int b = 0; b < B; ++b) {
      if (d_rp) {
        struct Tmp {
          void *c = nullptr, *v = nullptr;
          ~Tmp() {
            if (c) (void)hipFree(c);
            if (v) (void)hipFree(v);
          }
        } t;
        LHPC_TRY(colblock_device(d_rp, rp.bits, col_idx, val, tsz, r0, r1, cb[b], cb[b + 1], lrp, &t.c, &t.v));
        const int64_t m = lrp.back();
        if (m == 0) continue;  // adds nothing
        LHPC_TRY(add(r0, r1, cb[b], cb[b + 1], RowPtrView{lrp.data(), 64}, static_cast<const int32_t *>(t.c), t.v, m,
                     first ? 0 : 1));
      } else {
        csr_column_block(rp.p, rp.bits, col_idx, val, tsz, r0, r1, cb[b], cb[b + 1], lrp, lcol, lval);
        if (lcol.empty()) continue;  // adds nothing
        LHPC_TRY(add(r0, r1, cb[b], cb[b + 1], RowPtrView{lrp.data(), 64}, lcol.data(), lval.data(),
                     static_cast<int64_t>(lcol.size()), first ? 0 : 1));
      }
      first = false;
    }
  }
  p->part_row.push_back(n_rows);
  p->kernel = LHPC_KERNEL_XTILE;
  p->S = p->parts.empty() ? 0 : p->parts[0]->S;
  p->xs_width = p->parts.empty() ? 0 : p->parts[0]->xs_width;
  return LHPC_OK;
}

int plan_create_device_input(lhpc_spmv_plan **out, int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz,
                             const void *row_ptr, int row_ptr_bits, const int32_t *col_idx, const void *val,
                             const int *device_ids, int n_devices, unsigned flags, int n_splits,
                             const int64_t *split_rows, const lhpc_options *opts);

// host A → HBM copies → the device layout build (xtile_build_device /
// build_parts on the device); LHPC_ERR_UNSUPPORTED when the device build
// does not apply (aligned segments) or the copies do not fit in HBM
int xtile_build_uploaded(lhpc_spmv_plan *p, RowPtrView rp, const void *row_ptr, const int32_t *col_idx,
                         const void *val, size_t tsz, bool parts, int64_t cap, int B) {
  if (p->opt.xtile_host_build == 1 || p->opt.xtile_align == LHPC_XTILE_ALIGN_UNITS || p->nnz == 0)
    return LHPC_ERR_UNSUPPORTED;
  struct Tmp {
    void *a = nullptr;
    ~Tmp() {
      if (a) (void)hipFree(a);
    }
  } d_rp, d_col, d_val;
  const size_t rpb = static_cast<size_t>(p->n_rows + 1) * (rp.bits / 8);
  const size_t nnz = static_cast<size_t>(p->nnz);
  if (hipMalloc(&d_rp.a, rpb) != hipSuccess || hipMalloc(&d_col.a, std::max<size_t>(nnz, 1) * 4) != hipSuccess ||
      hipMalloc(&d_val.a, std::max<size_t>(nnz, 1) * tsz) != hipSuccess) {
    (void)hipGetLastError();
    return LHPC_ERR_UNSUPPORTED;
  }
  LHPC_HIP_TRY(hipMemcpy(d_rp.a, row_ptr, rpb, hipMemcpyHostToDevice));
  if (nnz) {
    LHPC_HIP_TRY(hipMemcpy(d_col.a, col_idx, nnz * 4, hipMemcpyHostToDevice));
    LHPC_HIP_TRY(hipMemcpy(d_val.a, val, nnz * tsz, hipMemcpyHostToDevice));
  }
  const int32_t *dc = static_cast<const int32_t *>(d_col.a);
  return parts ? build_parts(p, rp, dc, d_val.a, tsz, cap, B, d_rp.a) : xtile_build_device(p, rp, dc, d_val.a, tsz);
}

int plan_create_impl(lhpc_spmv_plan **out, int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz,
                     const void *row_ptr, int row_ptr_bits, const int32_t *col_idx, const void *val,
                     const int *device_ids, int n_devices, unsigned flags, int n_splits,
                     const int64_t *split_rows, const lhpc_options *opts) {
  if (!out) return LHPC_ERR_INVALID_ARG;
  const lhpc_options o = resolve_options(opts);
  *out = nullptr;
  if ((dtype != LHPC_F32 && dtype != LHPC_F64) || n_rows < 0 || n_cols < 0 || nnz < 0 ||
      !row_ptr || (row_ptr_bits != 32 && row_ptr_bits != 64) || n_cols > INT32_MAX ||
      (nnz > 0 && (!col_idx || !val)))
    return LHPC_ERR_INVALID_ARG;
  if (n_devices < 0 || (n_devices > 1 && !device_ids)) return LHPC_ERR_INVALID_ARG;
  if (row_ptr_bits == 32 && nnz > INT32_MAX) return LHPC_ERR_INVALID_ARG;
  if (flags & LHPC_PLAN_DEVICE_INPUT)
    return plan_create_device_input(out, dtype, n_rows, n_cols, nnz, row_ptr, row_ptr_bits, col_idx, val, device_ids,
                                    n_devices, flags, n_splits, split_rows, opts);

  const RowPtrView rp{row_ptr, row_ptr_bits};
  // always: every layout pass below indexes host arrays by row_ptr / col_idx,
  // and every kernel indexes x by col_idx (LHPC_PLAN_VALIDATE is implied)
  LHPC_TRY(validate_csr(row_ptr, row_ptr_bits, col_idx, n_rows, n_cols, nnz));

  // several devices driven by this one host thread: one local
  // plan, stream, comm stream (and RCCL comm) per device (lhpc_multi.hip)
  if (n_devices > 1 || (o.multi_force && n_devices == 1 && device_ids)) {
    if (n_splits > 0) return LHPC_ERR_UNSUPPORTED;
    auto *p = new (std::nothrow) lhpc_spmv_plan();
    if (!p) return LHPC_ERR_ALLOC;
    p->opt = o;
    p->dtype = dtype;
    p->n_rows = n_rows;
    p->n_cols = n_cols;
    p->nnz = nnz;
    const int st = multi_create(p, rp, col_idx, val, device_ids, n_devices, flags);
    if (st != LHPC_OK) {
      lhpc_spmv_plan_destroy(p);
      return st;
    }
    *out = p;
    return LHPC_OK;
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
  p->opt = o;
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
  // XSLICE / XTILE when x outgrows one XCD's 4 MB L2
  const double x_bytes = static_cast<double>(n_cols) * static_cast<double>(tsz);
  // ... and only when the gathers have no locality of their own: a banded or
  // structured matrix (stencil operators, the CG Laplacian) re-reads each x
  // line from neighbouring rows, which the row-local kernels already serve
  // from L2, while XSLICE would add S partials per row.  Measure it: distinct
  // 128-B x lines per nonzero over sampled 8192-row chunks (≈0.8 for C2's
  // uniform columns, ≈0.03 for a 2-D Laplacian); ≤ 0.25 counts as local.
  const double locality_thr = o.spmv_locality > 0 ? o.spmv_locality : 0.25;
  const bool auto_ok = !(flags & (LHPC_PLAN_FORCE_ROWGROUP | LHPC_PLAN_FORCE_ADAPTIVE |
                                   LHPC_PLAN_FORCE_XSLICE | LHPC_PLAN_FORCE_XTILE | LHPC_PLAN_FORCE_SELL));
  const bool nolocal =
      auto_ok && x_bytes > 8.0e6 && gather_lines_per_nnz(
          rp,
          [&](int64_t k0, int64_t k1, int32_t *out) {
            std::memcpy(out, col_idx + k0, static_cast<size_t>(k1 - k0) * 4);
            return LHPC_OK;
          },
          n_rows, n_cols, tsz) > locality_thr;
  // XTILE (x tiles in LDS) is the default for gathers without locality;
  // options.spmv_no_xtile selects XSLICE instead.
  const bool want_xtile = (flags & LHPC_PLAN_FORCE_XTILE) || (nolocal && !o.spmv_no_xtile);
  if (want_xtile && n_rows > 0) {
    // row parts when the tile stream outgrows its int32 offsets (or a lower
    // cap is asked for); user row splits keep a single plan
    // and column blocks when x spans many tiles (xtile_col_blocks_for)
    const int64_t tiles = (n_cols + (tsz == 4 ? 40960 : 20480) - 1) / (tsz == 4 ? 40960 : 20480);
    int64_t cap = INT32_MAX - 8 * (tiles + 256) - (int64_t{1} << 16);
    if (o.xtile_part_nnz > 0) cap = std::min<int64_t>(cap, o.xtile_part_nnz);
    const int B = n_splits == 0 ? xtile_col_blocks_for(n_rows, n_cols, nnz, tsz, o) : 1;
    const bool parts = (nnz > cap || B > 1) && n_splits == 0 && (tiles + B - 1) / B <= 4096;
    // the layout is built on the GPU from uploaded copies of A (byte-identical
    // to the host build, DESIGN.md §4 device input; C2 0.57 → ≈ 0.15 s); the
    // host build when the device cannot (aligned segments, no memory)
    const std::vector<int64_t> splits_in = p->split_rows;  // a build may add cache-range cuts
    int st = xtile_build_uploaded(p, rp, row_ptr, col_idx, val, tsz, parts, cap, B);
    if (st == LHPC_ERR_UNSUPPORTED) {
      p->split_rows = splits_in;
      for (auto *q : p->parts) lhpc_spmv_plan_destroy(q);
      p->parts.clear();
      p->part_row.clear();
      p->part_col.clear();
      p->bytes = 0;
      st = parts ? build_parts(p, rp, col_idx, val, tsz, cap, B) : xtile_build(p, rp, col_idx, val, tsz);
    }
    if (st == LHPC_OK) {
      *out = p;
      return LHPC_OK;
    }
    if (st != LHPC_ERR_UNSUPPORTED) {
      lhpc_spmv_plan_destroy(p);
      return st;
    }
    for (auto *q : p->parts) lhpc_spmv_plan_destroy(q);
    p->parts.clear();
    p->part_row.clear();
    p->part_col.clear();
    p->bytes = 0;
    // layout does not fit its index types: XSLICE / CSR kernels below
  }
  const bool want_xslice = (flags & LHPC_PLAN_FORCE_XSLICE) || nolocal;
  if (want_xslice && nnz > 0) {
    const int st = xslice_build(p, rp, col_idx, val, tsz, flags);
    if (st == LHPC_OK) {
      *out = p;
      return LHPC_OK;
    }
    if (st != LHPC_ERR_UNSUPPORTED) {
      lhpc_spmv_plan_destroy(p);
      return st;
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
  if (p->kernel == LHPC_KERNEL_ROWGROUP && (o.rowgroup_lanes > 0 || o.rowgroup_rows > 0)) {
    // the (L, R) shapes lhpc_spmv_csr.hip instantiates
    static const int kShapes[] = {101, 201, 202, 401, 402, 404, 802, 804, 1601, 1602, 1604, 1608, 3201, 3202, 6401};
    const int want = o.rowgroup_lanes * 100 + o.rowgroup_rows;
    if (std::find(std::begin(kShapes), std::end(kShapes), want) == std::end(kShapes)) {
      lhpc_spmv_plan_destroy(p);
      return LHPC_ERR_INVALID_ARG;
    }
    p->L = o.rowgroup_lanes;
    p->R = o.rowgroup_rows;
  }

  // SELL for short rows (≤ 8 nonzeros) whose padded slices stream no more
  // bytes than CSR + row_ptr: bit-identical to ADAPTIVE, no row_ptr stream,
  // LDS or barrier (the CG Laplacian: DESIGN.md §4)
  const bool force_sell = (flags & LHPC_PLAN_FORCE_SELL) != 0;
  if (p->kernel == LHPC_KERNEL_ADAPTIVE && (force_sell || (auto_ok && !o.spmv_no_sell)) && maxlen <= kSellMaxW &&
      n_rows > 0) {
    const int st = sell_build(p, rp, col_idx, val, tsz, force_sell);
    if (st == LHPC_OK) {
      *out = p;
      return LHPC_OK;
    }
    if (st != LHPC_ERR_UNSUPPORTED) {
      lhpc_spmv_plan_destroy(p);
      return st;
    }
  }
  if (force_sell) {
    lhpc_spmv_plan_destroy(p);
    return LHPC_ERR_UNSUPPORTED;  // a row longer than kSellMaxW (or no rows)
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
      std::vector<int64_t> b = csr_build_blocks(rp, n_rows, p->n_long);
      p->n_blocks = static_cast<int64_t>(b.size()) - 1;
      // device table: {first row, its row_ptr} per block boundary, so a block
      // reads its row and nonzero range with one 32-B load (no dependent
      // row_ptr round trip)
      std::vector<int64_t> bp(2 * b.size());
      for (size_t k = 0; k < b.size(); ++k) {
        bp[2 * k] = b[k];
        bp[2 * k + 1] = rp[b[k]];
      }
      if ((st = dmalloc(reinterpret_cast<void **>(&p->d_blocks), bp.size() * 8, p->bytes))) break;
      if ((st = static_cast<int>(hipMemcpy(p->d_blocks, bp.data(), bp.size() * 8, hipMemcpyHostToDevice))))
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
// LHPC_PLAN_DEVICE_INPUT: row_ptr / col_idx / val in HBM of the plan's
// device (e.g. straight from lhpc_coo_to_csr on the device).  Validated on
// the GPU; row_ptr (n_rows + 1 words) and the 32 locality samples come back
// to the host, which makes every layout decision.  The XTILE layout — the
// default for gathers without locality — is then built on the GPU from the
// device arrays (xtile_build_device: byte-identical to the host build); any
// other family, aligned segments or several devices copy A to the host and
// take the host path; row parts and column blocks are built on the GPU too.
int plan_create_device_input(lhpc_spmv_plan **out, int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz,
                             const void *row_ptr, int row_ptr_bits, const int32_t *col_idx, const void *val,
                             const int *device_ids, int n_devices, unsigned flags, int n_splits,
                             const int64_t *split_rows, const lhpc_options *opts) {
  RocTxRange rx("lhpc_spmv_plan_create: device input");
  const lhpc_options o = resolve_options(opts);
  int dev = 0;
  if (device_ids && n_devices >= 1) {
    dev = device_ids[0];
    LHPC_HIP_TRY(hipSetDevice(dev));
  } else {
    LHPC_HIP_TRY(hipGetDevice(&dev));
  }
  if (!is_gfx950(dev)) return LHPC_ERR_NO_DEVICE;
  // the arrays may still be in flight on any stream of the caller (plan
  // creation is synchronous anyway)
  LHPC_HIP_TRY(hipDeviceSynchronize());
  const size_t tsz = dtype == LHPC_F32 ? 4 : 8;
  {
    unsigned *flag = nullptr;
    LHPC_HIP_TRY(hipMalloc(reinterpret_cast<void **>(&flag), 4));
    hipError_t e = hipMemset(flag, 0, 4);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_validate_device_csr, dim3(1024), dim3(256), 0, nullptr, row_ptr, row_ptr_bits, col_idx,
                         n_rows, n_cols, nnz, flag);
      e = hipGetLastError();
    }
    unsigned bad = 0;
    if (e == hipSuccess) e = hipMemcpy(&bad, flag, 4, hipMemcpyDeviceToHost);
    (void)hipFree(flag);
    if (e != hipSuccess) return static_cast<int>(e);
    if (bad) return LHPC_ERR_BAD_CSR;
  }
  const size_t rpb = static_cast<size_t>(n_rows + 1) * (row_ptr_bits / 8);
  std::vector<unsigned char> hrp(rpb);
  LHPC_HIP_TRY(hipMemcpy(hrp.data(), row_ptr, rpb, hipMemcpyDeviceToHost));
  const RowPtrView rp{hrp.data(), row_ptr_bits};
  // the host path's XTILE decision (plan_create_impl), on the copied row_ptr
  // and device-fetched locality samples
  const double x_bytes = static_cast<double>(n_cols) * static_cast<double>(tsz);
  const double locality_thr = o.spmv_locality > 0 ? o.spmv_locality : 0.25;
  const bool auto_ok = !(flags & (LHPC_PLAN_FORCE_ROWGROUP | LHPC_PLAN_FORCE_ADAPTIVE | LHPC_PLAN_FORCE_XSLICE |
                                   LHPC_PLAN_FORCE_XTILE | LHPC_PLAN_FORCE_SELL));
  const int64_t tiles = (n_cols + (tsz == 4 ? 40960 : 20480) - 1) / (tsz == 4 ? 40960 : 20480);
  int64_t cap = INT32_MAX - 8 * (tiles + 256) - (int64_t{1} << 16);
  if (o.xtile_part_nnz > 0) cap = std::min<int64_t>(cap, o.xtile_part_nnz);
  // row parts and column blocks as plan_create_impl chooses them
  const int B = n_splits == 0 ? xtile_col_blocks_for(n_rows, n_cols, nnz, tsz, o) : 1;
  const bool parts = (nnz > cap || B > 1) && n_splits == 0;
  const bool single = n_devices <= 1 && !o.multi_force && n_rows > 0 &&
                      (parts ? (tiles + B - 1) / B <= 4096 : nnz <= cap && tiles <= 4096);
  bool want_xtile = single && (flags & LHPC_PLAN_FORCE_XTILE);
  // the host path's locality test (plan_create_impl's `nolocal`), on
  // device-fetched samples: XTILE here, and the SELL decision below
  bool nolocal = false;
  if (auto_ok && x_bytes > 8.0e6)
    nolocal = gather_lines_per_nnz(
                  rp,
                  [&](int64_t k0, int64_t k1, int32_t *dst) {
                    return static_cast<int>(hipMemcpy(dst, col_idx + k0, static_cast<size_t>(k1 - k0) * 4,
                                                      hipMemcpyDeviceToHost));
                  },
                  n_rows, n_cols, tsz) > locality_thr;
  if (single && auto_ok && !o.spmv_no_xtile && x_bytes > 8.0e6) want_xtile = nolocal;
  if (want_xtile) {
    auto *p = new (std::nothrow) lhpc_spmv_plan();
    if (!p) return LHPC_ERR_ALLOC;
    p->opt = o;
    if (n_splits > 0) p->split_rows.assign(split_rows, split_rows + n_splits);
    p->dtype = dtype;
    p->device = dev;
    p->n_rows = n_rows;
    p->n_cols = n_cols;
    p->nnz = nnz;
    const int st = parts ? build_parts(p, rp, col_idx, val, tsz, cap, B, row_ptr)
                         : xtile_build_device(p, rp, col_idx, val, tsz);
    if (st == LHPC_OK) {
      *out = p;
      return LHPC_OK;
    }
    lhpc_spmv_plan_destroy(p);
    if (st != LHPC_ERR_UNSUPPORTED) return st;
  }
  // SELL (short rows with x locality, as plan_create_impl selects it) built
  // on the GPU from the device arrays; when the padding rule refuses it, the
  // host path below chooses again (ADAPTIVE)
  const bool force_sell = (flags & LHPC_PLAN_FORCE_SELL) != 0;
  if (n_devices <= 1 && !o.multi_force && n_splits == 0 && n_rows > 0 &&
      (force_sell || (auto_ok && !o.spmv_no_sell && !nolocal))) {
    int64_t maxlen = 0;
    for (int64_t i = 0; i < n_rows; ++i) maxlen = std::max<int64_t>(maxlen, rp[i + 1] - rp[i]);
    if (maxlen <= kSellMaxW) {
      auto *p = new (std::nothrow) lhpc_spmv_plan();
      if (!p) return LHPC_ERR_ALLOC;
      p->opt = o;
      p->dtype = dtype;
      p->device = dev;
      p->n_rows = n_rows;
      p->n_cols = n_cols;
      p->nnz = nnz;
      const int st = sell_build_device(p, rp, row_ptr, col_idx, val, tsz, force_sell);
      if (st == LHPC_OK) {
        *out = p;
        return LHPC_OK;
      }
      lhpc_spmv_plan_destroy(p);
      if (st != LHPC_ERR_UNSUPPORTED) return st;
    }
  }
  // every other case: A to the host, the host path
  std::vector<int32_t> hcol(static_cast<size_t>(nnz));
  std::vector<unsigned char> hval(static_cast<size_t>(nnz) * tsz);
  if (nnz) {
    LHPC_HIP_TRY(hipMemcpy(hcol.data(), col_idx, static_cast<size_t>(nnz) * 4, hipMemcpyDeviceToHost));
    LHPC_HIP_TRY(hipMemcpy(hval.data(), val, static_cast<size_t>(nnz) * tsz, hipMemcpyDeviceToHost));
  }
  return plan_create_impl(out, dtype, n_rows, n_cols, nnz, hrp.data(), row_ptr_bits, hcol.data(), hval.data(),
                          device_ids, n_devices, flags & ~static_cast<unsigned>(LHPC_PLAN_DEVICE_INPUT), n_splits,
                          split_rows, opts);
}

}  // namespace
}  // namespace lhpc

using namespace lhpc;

extern "C" int lhpc_spmv_plan_create(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                                     int64_t n_cols, int64_t nnz, const void *row_ptr,
                                     int row_ptr_bits, const int32_t *col_idx,
                                     const void *val, const int *device_ids,
                                     int n_devices, unsigned flags) {
  try {
    RocTxRange rx("lhpc_spmv_plan_create");
    return plan_create_impl(out, dtype, n_rows, n_cols, nnz, row_ptr, row_ptr_bits, col_idx, val,
                            device_ids, n_devices, flags, 0, nullptr, nullptr);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_plan_create_opts(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                                          int64_t n_cols, int64_t nnz, const void *row_ptr,
                                          int row_ptr_bits, const int32_t *col_idx,
                                          const void *val, const int *device_ids, int n_devices,
                                          unsigned flags, int n_splits, const int64_t *split_rows,
                                          const lhpc_options *opts) {
  try {
    if (!out || n_splits < 0 || (n_splits > 0 && !split_rows)) return LHPC_ERR_INVALID_ARG;
    for (int i = 0; i < n_splits; ++i)
      if (split_rows[i] <= 0 || split_rows[i] >= n_rows || (i > 0 && split_rows[i] <= split_rows[i - 1]))
        return LHPC_ERR_INVALID_ARG;
    RocTxRange rx("lhpc_spmv_plan_create");
    const int st = plan_create_impl(out, dtype, n_rows, n_cols, nnz, row_ptr, row_ptr_bits, col_idx, val,
                                    device_ids, n_devices, flags, n_splits, split_rows, opts);
    if (st != LHPC_OK || n_splits == 0) return st;
    const lhpc_spmv_plan *p = *out;
    if (p->kernel != LHPC_KERNEL_XTILE || p->xt_srow.size() != static_cast<size_t>(n_splits) + 2) {
      lhpc_spmv_plan_destroy(*out);  // ranges exist only in the XTILE tile-stream layout
      *out = nullptr;
      return LHPC_ERR_UNSUPPORTED;
    }
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_plan_create_split(lhpc_spmv_plan **out, int dtype, int64_t n_rows,
                                           int64_t n_cols, int64_t nnz, const void *row_ptr,
                                           int row_ptr_bits, const int32_t *col_idx,
                                           const void *val, const int *device_ids, int n_devices,
                                           unsigned flags, int n_splits, const int64_t *split_rows) {
  try {
    if (n_splits < 1) return LHPC_ERR_INVALID_ARG;
    return lhpc_spmv_plan_create_opts(out, dtype, n_rows, n_cols, nnz, row_ptr, row_ptr_bits, col_idx, val,
                                      device_ids, n_devices, flags, n_splits, split_rows, nullptr);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_stage(const lhpc_spmv_plan *p, const void *x, void *stream) {
  try {
    if (!p || (p->n_cols > 0 && !x)) return LHPC_ERR_INVALID_ARG;
    if (p->xt_srow.empty() || p->xt_ring) return LHPC_ERR_UNSUPPORTED;  // a ring holds one range's xg
    RocTxRange rx("lhpc_spmv_stage");
    LHPC_HIP_TRY(hipSetDevice(p->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    return xtile_stage(p, x, s);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_range(const lhpc_spmv_plan *p, int k, void *y_range, void *stream) {
  try {
    if (!p || p->xt_srow.empty() || k < 0 || k + 2 > static_cast<int>(p->xt_srow.size()))
      return LHPC_ERR_INVALID_ARG;
    if (p->xt_ring) return LHPC_ERR_UNSUPPORTED;
    if (p->xt_srow[k + 1] > p->xt_srow[k] && !y_range) return LHPC_ERR_INVALID_ARG;
    RocTxRange rx("lhpc_spmv_range");
    LHPC_HIP_TRY(hipSetDevice(p->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    return xtile_range(p, k, y_range, s);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv(lhpc_spmv_plan *p, const void *x, void *y, int on_device,
                         void *stream) {
  try {
    if (!p || (p->n_cols > 0 && !x) || (p->n_rows > 0 && !y)) return LHPC_ERR_INVALID_ARG;
    RocTxRange rx("lhpc_spmv");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (p->multi) return multi_home(p, x, y, on_device, s);
    LHPC_HIP_TRY(hipSetDevice(p->device));
    const size_t tsz = p->dtype == LHPC_F32 ? 4 : 8;
    const void *dx = x;
    void *dy = y;
    if (!on_device) {
      if (!p->d_xstage) {
        LHPC_TRY(dmalloc(&p->d_xstage, static_cast<size_t>(p->n_cols) * tsz, p->bytes));
        LHPC_TRY(dmalloc(&p->d_ystage, static_cast<size_t>(p->n_rows) * tsz, p->bytes));
      }
      // host buffers: synchronous copies (see lhpc_sort.hip HostStage); the
      // staging buffers are only touched by host-buffer calls, which end synced
      LHPC_HIP_TRY(hipMemcpy(p->d_xstage, x, static_cast<size_t>(p->n_cols) * tsz, hipMemcpyHostToDevice));
      dx = p->d_xstage;
      dy = p->d_ystage;
    }
    const int st = launch(p, dx, dy, s);
    if (st != LHPC_OK) return st;
    if (!on_device) {
      LHPC_HIP_TRY(hipStreamSynchronize(s));
      LHPC_HIP_TRY(hipMemcpy(y, p->d_ystage, static_cast<size_t>(p->n_rows) * tsz, hipMemcpyDeviceToHost));
    }
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_vec_dot(int dtype, int64_t n, const void *a, const void *b, double *out, void *stream);

extern "C" int lhpc_spmv_dot(lhpc_spmv_plan *p, const void *x, void *y, const void *w, double *dot_out,
                             void *stream) {
  try {
    if (!p || !dot_out || (p->n_cols > 0 && !x) || (p->n_rows > 0 && (!y || !w))) return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    LHPC_HIP_TRY(hipSetDevice(p->device));
    if ((p->kernel == LHPC_KERNEL_ADAPTIVE || p->kernel == LHPC_KERNEL_SELL) && p->n_blocks > 0) {
      const int st = csr_launch_dot(p, x, y, w, dot_out, s);
      if (st != LHPC_ERR_UNSUPPORTED) return st;
    }
    // other kernel families: SpMV, then a separate dot pass
    LHPC_TRY(lhpc_spmv(p, x, y, 1, stream));
    return lhpc_vec_dot(p->dtype, p->n_rows, w, y, dot_out, stream);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_plan_info_get(const lhpc_spmv_plan *p, lhpc_spmv_plan_info *info) {
  try {
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
    info->launches = p->kernel == LHPC_KERNEL_XSLICE ? 2 : 1;
    if (p->kernel == LHPC_KERNEL_XTILE) {
      info->launches = p->xt_mall > 1 ? 2 * p->xt_mall + (p->xt_cont > 0 ? 1 : 0)
                                      : (p->xt_pieces > 0 ? 1 : 0) + 1 + (p->xt_cont > 0 ? 1 : 0);
      info->n_blocks = p->xt_C;
      info->n_long_rows = p->xt_cont;
    }
    info->slices = p->S;
    info->slice_width = p->xs_width;
    if (p->kernel == LHPC_KERNEL_SELL) {  // 64-row slices, widest slice in nonzeros
      info->slices = static_cast<int>((p->n_rows + kWave - 1) / kWave);
      info->slice_width = p->sell_w;
    }
    if (!p->parts.empty()) {  // XTILE row parts: totals over the parts
      info->launches = 0;
      info->n_blocks = 0;
      info->n_long_rows = 0;
      for (const auto *q : p->parts) {
        lhpc_spmv_plan_info qi{};
        LHPC_TRY(lhpc_spmv_plan_info_get(q, &qi));
        info->launches += qi.launches;
        info->n_blocks += qi.n_blocks;
        info->n_long_rows += qi.n_long_rows;
      }
    }
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_spmv_plan_destroy(lhpc_spmv_plan *p) {
  try {
    if (!p) return LHPC_OK;
    if (p->multi) multi_free(p);
    for (auto *q : p->parts) lhpc_spmv_plan_destroy(q);
    (void)hipSetDevice(p->device);
    for (void *q : {p->d_row_ptr, static_cast<void *>(p->d_col), p->d_val, static_cast<void *>(p->d_blocks),
                    p->d_xstage, p->d_ystage, p->d_lens, static_cast<void *>(p->d_cbase), p->d_partial,
                    static_cast<void *>(p->d_dpart), static_cast<void *>(p->d_cdesc), static_cast<void *>(p->d_cr),
                    static_cast<void *>(p->d_seghi), static_cast<void *>(p->d_seg), static_cast<void *>(p->d_pieces), static_cast<void *>(p->d_cont),
                    static_cast<void *>(p->d_col16), static_cast<void *>(p->d_perm), p->d_xg,
                    static_cast<void *>(p->d_pieces_cp), static_cast<void *>(p->d_pext),
                    static_cast<void *>(p->d_carry)})
      if (q) (void)hipFree(q);
    if (p->h_scalars) (void)hipHostFree(p->h_scalars);
    for (hipGraphExec_t g : p->cg_graph)
      if (g) (void)hipGraphExecDestroy(g);
    if (p->cg_vecs) (void)hipFree(p->cg_vecs);
    if (p->cg_scal) (void)hipFree(p->cg_scal);
    delete p;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

// Test support: FNV-1a digests of an XTILE plan's device layout, in the
// order row_ptr, col16, perm/iperm, val runs, chunk descriptors, cr, segment
// table (lo/len, hi), gather pieces, cont — so a test can byte-compare the
// layout built on the GPU from device input with the host build's.
extern "C" int lhpc_spmv_plan_layout_digest(const lhpc_spmv_plan *p, uint64_t *out, int cap, int *n_out) {
  try {
    if (!p || !out || !n_out || cap < 10) return LHPC_ERR_INVALID_ARG;
    if (p->kernel != LHPC_KERNEL_XTILE || p->multi) return LHPC_ERR_UNSUPPORTED;
    if (!p->parts.empty()) {  // row parts / column blocks: the parts' digests folded in order
      for (int i = 0; i < 10; ++i) out[i] = 0xcbf29ce484222325ull;
      for (size_t j = 0; j < p->parts.size(); ++j) {
        uint64_t d[10];
        int n = 0;
        LHPC_TRY(lhpc_spmv_plan_layout_digest(p->parts[j], d, 10, &n));
        const uint64_t where = static_cast<uint64_t>(p->part_row[j]) * 0x9E3779B97F4A7C15ull ^
                               static_cast<uint64_t>(p->part_col[j]) ^ static_cast<uint64_t>(p->parts[j]->xt_acc) << 63;
        for (int i = 0; i < 10; ++i) out[i] = (out[i] ^ d[i] ^ where) * 0x100000001b3ull;
      }
      *n_out = 10;
      return LHPC_OK;
    }
    LHPC_HIP_TRY(hipSetDevice(p->device));
    const size_t tsz = p->dtype == LHPC_F32 ? 4 : 8;
    const int64_t C = p->xt_C;
    const std::pair<const void *, size_t> arr[10] = {
        {p->d_row_ptr, static_cast<size_t>(p->n_rows + 1) * 4},
        {p->d_col16, static_cast<size_t>(p->xt_total) * 2},
        {p->d_perm, static_cast<size_t>(p->xt_p == 3 ? p->xt_nrun : p->xt_total + 2) * 2},
        {p->d_val, static_cast<size_t>(p->xt_nrun) * tsz},
        {p->d_cdesc, static_cast<size_t>(8 * C + 8) * 4},
        {p->d_cr, static_cast<size_t>(C + 1) * 4},
        {p->d_seg, static_cast<size_t>(p->xt_seg_n) * 4},  // segment table (or PRE: batch rank terms)
        {p->d_seghi, static_cast<size_t>(p->xt_seghi_n) * 4},
        {p->d_pieces, static_cast<size_t>(p->xt_pieces) * 12},
        {p->d_cont, static_cast<size_t>(p->xt_cont) * 4}};
    std::vector<unsigned char> h;
    for (int i = 0; i < 10; ++i) {
      h.resize(arr[i].second);
      if (arr[i].second) LHPC_HIP_TRY(hipMemcpy(h.data(), arr[i].first, arr[i].second, hipMemcpyDeviceToHost));
      uint64_t x = 0xcbf29ce484222325ull;
      for (unsigned char b : h) x = (x ^ b) * 0x100000001b3ull;
      out[i] = x ^ static_cast<uint64_t>(arr[i].second);
    }
    *n_out = 10;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
