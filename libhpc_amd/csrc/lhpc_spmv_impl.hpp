// lhpc_spmv_impl.hpp — the SpMV plan object and the interface between the
// kernel-family translation units:
//   lhpc_spmv.hip         plan creation (kernel selection), the C ABI
//   lhpc_spmv_csr.hip     ROWGROUP / ADAPTIVE (CSR kept as is), SELL (short rows)
//   lhpc_spmv_xslice.hip  XSLICE (XCD-local column slices + partial reduce)
//   lhpc_spmv_xtile.hip   XTILE (x tiles in LDS: tile gather + chunk reduce)
// The reference has no SpMV: the operator is
// y[i] = Σ_{k=row_ptr[i]}^{row_ptr[i+1]-1} val[k]·x[col_idx[k]].
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <vector>

#include "lhpc_common.hpp"

struct lhpc_spmv_plan {
  lhpc_options opt{};  // resolved variant options (lhpc::resolve_options)
  int dtype = LHPC_F32;
  int device = 0;
  int rp64 = 0;  // device row_ptr is int64
  int64_t n_rows = 0, n_cols = 0, nnz = 0;
  void *d_row_ptr = nullptr;
  int32_t *d_col = nullptr;
  void *d_val = nullptr;
  int64_t *d_blocks = nullptr;  // ADAPTIVE: the block table; SELL: the slice offsets
  int64_t n_blocks = 0, n_long = 0;
  int sell_w = 0;              // SELL: widest slice
  void *d_xstage = nullptr, *d_ystage = nullptr;
  double *h_scalars = nullptr;  // lhpc_cg_solve: 2 pinned host scalars, allocated on first use
  // lhpc_cg_solve's work (first solve; freed with the plan): r, p, q and x
  // vectors, device scalars + dot partials, and the captured iteration blocks
  // (graph c starts at rr parity c and holds cg_graph_iters[c] iterations)
  void *cg_vecs = nullptr;
  double *cg_scal = nullptr;
  hipGraphExec_t cg_graph[2] = {nullptr, nullptr};
  int cg_graph_iters[2] = {0, 0};
  std::atomic<int> cg_busy{0};  // a solve holds the work above (LHPC_ERR_BUSY for a second one)
  double *d_dpart = nullptr;  // lhpc_spmv_dot: per-block partials (ADAPTIVE / SELL), allocated on first use
  int kernel = LHPC_KERNEL_ROWGROUP;
  int L = 16, R = 4;
  int64_t bytes = 0;
  // XSLICE
  int S = 0;
  int xs_nb = 2, xs_p64 = 0, xs_lens16 = 0;
  int64_t xs_width = 0, xs_chunks = 0, xs_rows_pad = 0, xs_bps = 0;
  void *d_lens = nullptr;
  int64_t *d_cbase = nullptr;
  void *d_partial = nullptr;
  // XTILE
  int64_t xt_C = 0, xt_pieces = 0, xt_cont = 0, xt_total = 0, xt_nrun = 0;
  size_t xt_lds = 0;
  int xt_u = 8;  // gather steps in flight (lhpc_options.xtile_steps)
  int xt_nt = 0;  // gather: non-temporal xg stores (lhpc_options.xtile_store)
  // cache-sized ranges (lhpc_options.xtile_ranges = K): a call runs gather k, reduce k
  // for k < K so range k's xg is still in the Infinity Cache when its reduce
  // reads it; range k's gather pieces are [xt_rpc[k], xt_rpc[k+1])
  int xt_mall = 0;
  std::vector<int64_t> xt_rpc;
  // row ranges (lhpc_spmv_plan_create_split): range k = rows [xt_srow[k],
  // xt_srow[k+1]) = chunks [xt_src[k], xt_src[k+1]), cont entries [xt_sco[k], xt_sco[k+1])
  std::vector<int64_t> split_rows, xt_srow, xt_src, xt_sco;
  int32_t *d_cdesc = nullptr;
  int32_t *d_cr = nullptr, *d_seghi = nullptr, *d_pieces = nullptr, *d_cont = nullptr;
  uint32_t *d_seg = nullptr;  // segment table (lhpc_plan.hpp xtile_segment_table)
  uint16_t *d_col16 = nullptr, *d_perm = nullptr;
  int xt_p = 1;  // reduce: 1 perm scatter, 3 iperm gather (DESIGN.md §4 XTILE)
  int xt_al = 0;  // aligned segments: 16-B units (lhpc_options.xtile_align)
  void *d_xg = nullptr;
  // xg ring (cache-sized ranges without user splits, lhpc_plan.hpp
  // xtile_ring_pieces): d_xg holds xt_ring_len + 2 entries reused by every
  // range; per piece {ring delta, flags} in d_pext; range k's segment-table hi
  // rows start at xt_hrow[k]
  int xt_ring = 0;
  int xt_pre = 0;
  int64_t xt_seg_n = 0, xt_seghi_n = 0;  // entries of d_seg / d_seghi  // the reduce reads the plan's phase-A tables (d_seg = bt, d_seghi = base_ne)
  int64_t xt_ring_len = 0;
  int32_t *d_pext = nullptr;
  std::vector<int64_t> xt_hrow;
  double *d_carry = nullptr;
  // column parts (xtile_column_parts): the gather pieces reordered so that
  // part j = pieces [xt_cpf[j], xt_cpf[j+1]) of d_pieces_cp reads x only
  // below column xt_cpe[j] (a chained distributed call gathers part j as
  // soon as exchange j of the previous call has landed)
  int32_t *d_pieces_cp = nullptr;
  std::vector<int64_t> xt_cpf, xt_cpe;
  // XTILE row parts (lhpc_options.xtile_part_nnz): a matrix whose tile stream
  // exceeds the int32 stream offsets is cut into nnz-balanced row parts, one
  // XTILE plan each (rows [part_row[i], part_row[i+1]) of y), run in turn on
  // the same x; this plan then holds no arrays of its own
  std::vector<lhpc_spmv_plan *> parts;
  std::vector<int64_t> part_row;
  // XTILE column blocks (lhpc_options.xtile_col_blocks): parts may also cover a
  // column range [part_col[i], …) of x; a part whose xt_acc is set adds its
  // sums into y instead of storing them (every block of a row part after the
  // first one, run after it on the same stream)
  std::vector<int64_t> part_col;
  int xt_acc = 0;
  // single-process multi-device plan (n_devices > 1; lhpc_multi.hip)
  struct lhpc_multi *multi = nullptr;
};

namespace lhpc {

constexpr int kBlock = 256;
constexpr int kSellMaxW = 8;  // SELL: nonzeros per row at most (ADAPTIVE's 2048 / 256)

// Host view of row_ptr regardless of width.
struct RowPtrView {
  const void *p;
  int bits;
  int64_t operator[](int64_t i) const {
    return bits == 64 ? static_cast<const int64_t *>(p)[i] : static_cast<const int32_t *>(p)[i];
  }
};

// hipMalloc that books the bytes on the plan; LHPC_ERR_ALLOC on OOM.
inline int dmalloc(void **p, size_t n, int64_t &acct) {
  if (n == 0) n = 16;
  hipError_t e = hipMalloc(p, n);
  if (e == hipErrorOutOfMemory) return LHPC_ERR_ALLOC;
  if (e != hipSuccess) return static_cast<int>(e);
  acct += static_cast<int64_t>(n);
  return LHPC_OK;
}

// ---- lhpc_multi.hip: one rank's (or one device's) share of a row-block
// split.  Its K blocks (block k·nranks + rank of the global cuts) stacked in
// chunk order form a local CSR (row_ptr rebased, global columns); one
// row-range XTILE plan over them (split at every block start) stages x once
// and reduces chunk k on its own, else (the matrix does not select XTILE,
// or a single block) one plan per non-empty block.
struct LocalPlans {
  int K = 0;
  std::vector<int64_t> ls;                  // local row offset of chunk k (K + 1)
  lhpc_spmv_plan *split = nullptr;          // row-range plan over the K blocks (XTILE)
  std::vector<int> range_of;                // chunk k → range index of `split` (−1: empty)
  std::vector<lhpc_spmv_plan *> block_plan; // otherwise one plan per non-empty block
  // a split plan with per-range gather pieces (its xg exceeds the Infinity
  // Cache) gathers each range right before reducing it; else one stage
  bool range_gather() const { return split && !split->xt_rpc.empty(); }
  bool column_parts() const { return split && !split->xt_cpf.empty(); }
};
// ls: K + 1 local row offsets; row_ptr/col/val: the local CSR (host)
int local_plans_create(LocalPlans &lp, int dtype, int64_t n_cols, int K, const int64_t *ls, const void *row_ptr,
                       int row_ptr_bits, const int32_t *col_idx, const void *val, int device, unsigned flags,
                       const lhpc_options &o);
void local_plans_destroy(LocalPlans &lp);
// the call's stage (all of x's tiles; no-op for range-gather and block plans)
int local_plans_stage(const LocalPlans &lp, const void *x, hipStream_t s);
// column parts of the stage (a split plan without range gathers only):
// col_end as for xtile_column_parts; false when unavailable
bool local_plans_column_parts(LocalPlans &lp, const int64_t *col_end, int n_parts);
int local_plans_stage_part(const LocalPlans &lp, const void *x, int j, hipStream_t s);
// chunk k's rows into yk (its first row at yk[0]); `gathered` counts the
// ranges a range-gather plan has gathered so far in this call (start at 0)
int local_plans_chunk(const LocalPlans &lp, const void *x, int k, void *yk, int &gathered, hipStream_t s);
// the rank's local CSR from the GLOBAL one: rows of blocks k·nranks + rank,
// stacked (K + 1 local offsets in ls); no copy of col/val for one block
struct LocalCsr {
  std::vector<int64_t> ls, rp;
  std::vector<int32_t> col;
  std::vector<unsigned char> val;
  const int32_t *colp = nullptr;
  const void *valp = nullptr;
};
// the single-process multi-device plan (n_devices > 1 or options.multi_force)
int multi_create(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, const int *device_ids,
                 int n_devices, unsigned flags);
void multi_free(lhpc_spmv_plan *p);
// lhpc_spmv on it: x, y on device_ids[0] (on_device) or host buffers
int multi_home(lhpc_spmv_plan *p, const void *x, void *y, int on_device, hipStream_t s);
void local_csr_from_global(LocalCsr &out, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz,
                           const int64_t *cuts, int nranks, int K, int rank);

// ---- lhpc_spmv_csr.hip
int csr_launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s);
// ADAPTIVE with the fused y·w epilogue: *dot_out = Σ y[i]·w[i] (fixed order)
int csr_launch_dot(lhpc_spmv_plan *p, const void *x, void *y, const void *w, double *dot_out, hipStream_t s);
// lhpc_cg_solve on a SELL plan: x += α·p_old, p_new = r + β·p_old (α = *anum / *aden,
// β = *bnum / *bden), q = A·p_new, *pq = p_new·q — k_cg_xp fused into the next
// iteration's SpMV + dot, bit-identical to the unfused steps
int sell_cg_step(lhpc_spmv_plan *p, const void *r, const void *p_old, void *p_new, void *x, void *q,
                 const double *anum, const double *aden, const double *bnum, const double *bden, double *pq,
                 hipStream_t s);
// SELL layout; LHPC_ERR_UNSUPPORTED when the rows do not suit it (caller falls back)
int sell_build(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz, bool forced);
// the same layout from device CSR (d_rp: row_ptr of rp_host.bits on the device; rp_host: its host copy)
int sell_build_device(lhpc_spmv_plan *p, RowPtrView rp_host, const void *d_rp, const int32_t *d_col,
                      const void *d_val, size_t tsz, bool forced);
// ADAPTIVE row blocks (≤ 2048 nonzeros and ≤ 256 rows, or one long row)
std::vector<int64_t> csr_build_blocks(RowPtrView rp, int64_t n_rows, int64_t &n_long);

// ---- lhpc_spmv_xslice.hip
int xslice_launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s);
// LHPC_ERR_UNSUPPORTED: some row too long for the slice layout (caller falls back)
int xslice_build(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz,
                 unsigned flags);

// ---- lhpc_spmv_xtile.hip
int xtile_launch(const lhpc_spmv_plan *p, const void *x, void *y, hipStream_t s);
int xtile_stage(const lhpc_spmv_plan *p, const void *x, hipStream_t s);
int xtile_range_gather(const lhpc_spmv_plan *p, const void *x, int k, hipStream_t s);
int xtile_range(const lhpc_spmv_plan *p, int k, void *yk, hipStream_t s);
// column parts: col_end[j] ascending, col_end[n_parts-1] ≥ n_cols; tile t goes
// to the first part whose bound covers its last column.  LHPC_ERR_UNSUPPORTED
// for plans that gather per row range (cache-sized ranges).
int xtile_column_parts(lhpc_spmv_plan *p, const int64_t *col_end, int n_parts);
// the first part whose bound covers the tile's last column (host rule shared
// with lhpc_dist_chain_parts)
int xtile_part_of_tile(int64_t tile, int64_t tile_width, int64_t n_cols, const int64_t *col_end, int n_parts);
int xtile_stage_part(const lhpc_spmv_plan *p, const void *x, int j, hipStream_t s);
// LHPC_ERR_UNSUPPORTED: the layout does not fit its index types (caller falls back)
int xtile_build(lhpc_spmv_plan *p, RowPtrView rp, const int32_t *col_idx, const void *val, size_t tsz);
// the same layout from device-resident col/val (rp: a host copy of row_ptr);
// LHPC_ERR_UNSUPPORTED for options the device build lacks (aligned segments)
int xtile_build_device(lhpc_spmv_plan *p, RowPtrView rp_host, const int32_t *d_col, const void *d_val, size_t tsz);

}  // namespace lhpc
