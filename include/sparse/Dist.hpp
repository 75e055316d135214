// sparse/Dist.hpp — multi-GPU SpMV and stencil in the reference's idiom, one
// process per GPU, RCCL over xGMI behind the C ABI (include/lhpc.h lhpc_dist_*).
//
//   sparse::DistComm              RAII RCCL communicator + comm stream of this rank
//   sparse::interleaved_cuts(A, nranks, K)        nnz-balanced cuts (nranks·K blocks)
//   sparse::interleaved_local(A, cuts, nranks, K, rank)   the rank's stacked blocks
//   sparse::DistSpMVPlan<T>       RAII distributed plan (the rank's local CSR)
//   sparse::spmv(plan, d_x, d_y, stream)          full y on every rank (device)
//   sparse::dist_stencil7(comm, d_u, d_out, ...)  z-slab step with RCCL halo planes
//   DistComm::local(nranks, rank, device), p2p_export(d_y, bytes) / p2p_import(blobs)
//                                 direct xGMI peer exchange of y into registered
//                                 windows (up to LHPC_DIST_P2P_MAX_WINDOWS: a
//                                 ping-pong pair), p2p_reset()
//   sparse::exchange(plan, d_y, stream)           the y exchange alone
//   sparse::exchange_schedule(cuts, nranks, K, rank, kind)   the transfers, as data
// Non-zero status → std::system_error (include/lhpc_error.hpp).  The
// reference has no multi-device code; the rank-0 unique id must
// reach every rank through the launcher's own channel (MPI_Bcast, a file, …).
#pragma once
#ifndef LHPC_SPARSE_DIST_HPP_
#define LHPC_SPARSE_DIST_HPP_

#include <array>
#include <cstdint>
#include <type_traits>
#include <utility>
#include <vector>

#include "../lhpc.h"
#include "../lhpc_error.hpp"
#include "CSRMatrix.hpp"

namespace sparse {

class DistComm {
 public:
  using unique_id_t = std::array<unsigned char, LHPC_DIST_UNIQUE_ID_BYTES>;
  static unique_id_t unique_id() {
    unique_id_t id{};
    lhpc::checkLhpc(lhpc_dist_get_unique_id(id.data()));
    return id;
  }
  DistComm(const unique_id_t &id, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
    lhpc::checkLhpc(lhpc_dist_comm_create(&comm_, id.data(), nranks, rank, device));
  }
  // RCCL-free communicator: only the direct peer exchange of a registered y
  struct local_t {};
  DistComm(local_t, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
    lhpc::checkLhpc(lhpc_dist_comm_create_local(&comm_, nranks, rank, device));
  }
  static DistComm local(int nranks, int rank, int device) { return DistComm(local_t{}, nranks, rank, device); }
  DistComm(DistComm &&o) noexcept : comm_(std::exchange(o.comm_, nullptr)), nranks_(o.nranks_), rank_(o.rank_) {}
  DistComm(const DistComm &) = delete;
  DistComm &operator=(const DistComm &) = delete;
  using p2p_blob_t = std::array<unsigned char, LHPC_DIST_P2P_BLOB_BYTES>;
  // this rank's y window (device, n_rows values) as a blob for every rank;
  // all-gather the blobs (rank order) through the launcher, then p2p_import:
  // sparse::spmv(plan, d_x, d_y) with that d_y exchanges by peer stores
  p2p_blob_t p2p_export(void *d_y, std::int64_t bytes) {
    p2p_blob_t b{};
    lhpc::checkLhpc(lhpc_dist_p2p_export(comm_, d_y, bytes, b.data()));
    return b;
  }
  void p2p_import(const std::vector<p2p_blob_t> &blobs) {
    std::vector<unsigned char> flat;
    for (const auto &b : blobs) flat.insert(flat.end(), b.begin(), b.end());
    lhpc::checkLhpc(lhpc_dist_p2p_import(comm_, flat.data()));
  }
  void p2p_reset() { lhpc::checkLhpc(lhpc_dist_p2p_reset(comm_)); }
  // LHPC_ERR_INTERNAL after a peer flag wait timed out (check after a stream sync)
  int p2p_status() const { return lhpc_dist_p2p_status(comm_); }
  ~DistComm() {
    if (comm_) lhpc_dist_comm_destroy(comm_);
  }
  int nranks() const noexcept { return nranks_; }
  int rank() const noexcept { return rank_; }
  lhpc_dist_comm *native() noexcept { return comm_; }
  // in-place sum over ranks (device doubles), asynchronous on `stream`
  void allreduce_sum(double *d_buf, std::int64_t count, void *stream = nullptr) {
    lhpc::checkLhpc(lhpc_dist_allreduce_sum_f64(comm_, d_buf, count, stream));
  }

 private:
  lhpc_dist_comm *comm_ = nullptr;
  int nranks_ = 1, rank_ = 0;
};

// nnz-balanced cuts of A's rows into nranks·K blocks; block k·nranks + r is
// rank r's chunk k (lhpc_csr_partition_rows with nranks·K parts).
template <typename T, typename IndexT, typename OffsetT>
std::vector<std::int64_t> interleaved_cuts(const CSRMatrix<T, IndexT, OffsetT> &A, int nranks, int K) {
  std::vector<std::int64_t> cuts(static_cast<std::size_t>(nranks) * K + 1);
  lhpc::checkLhpc(lhpc_csr_partition_rows(A.row_ptr.data(), sizeof(OffsetT) * 8, A.n_rows, nranks * K, cuts.data()));
  return cuts;
}

// The rank's K blocks stacked in chunk order: row_ptr rebased, global columns.
template <typename T, typename IndexT, typename OffsetT>
CSRMatrix<T, IndexT, std::int64_t> interleaved_local(const CSRMatrix<T, IndexT, OffsetT> &A,
                                                     const std::vector<std::int64_t> &cuts, int nranks, int K,
                                                     int rank) {
  std::int64_t rows = 0;
  for (int k = 0; k < K; ++k) rows += cuts[std::size_t(k) * nranks + rank + 1] - cuts[std::size_t(k) * nranks + rank];
  CSRMatrix<T, IndexT, std::int64_t> L(rows, A.n_cols);
  std::int64_t at = 0;
  for (int k = 0; k < K; ++k) {
    const std::int64_t r0 = cuts[std::size_t(k) * nranks + rank], r1 = cuts[std::size_t(k) * nranks + rank + 1];
    for (std::int64_t i = r0; i < r1; ++i) {
      const auto s = A.row_ptr[std::size_t(i)], e = A.row_ptr[std::size_t(i + 1)];
      L.col_idx.insert(L.col_idx.end(), A.col_idx.begin() + s, A.col_idx.begin() + e);
      L.val.insert(L.val.end(), A.val.begin() + s, A.val.begin() + e);
      L.row_ptr[std::size_t(++at)] = static_cast<std::int64_t>(L.col_idx.size());
    }
  }
  return L;
}

template <typename T>
class DistSpMVPlan {
  static_assert(std::is_same_v<T, float> || std::is_same_v<T, double>, "SpMV is fp32 or fp64");

 public:
  // `local`: this rank's K blocks of the n_rows × n_cols matrix, stacked
  // (interleaved_local); `cuts`: the nranks·K + 1 global row cuts.
  template <typename OffsetT>
  DistSpMVPlan(DistComm &comm, std::int64_t n_rows, std::int64_t n_cols, int K, const std::vector<std::int64_t> &cuts,
               const CSRMatrix<T, std::int32_t, OffsetT> &local, unsigned flags = LHPC_PLAN_DEFAULT,
               const lhpc_options *opts = nullptr)
      : n_rows_(n_rows), n_cols_(n_cols) {
    lhpc::checkLhpc(lhpc_dist_spmv_plan_create_opts(
        &plan_, comm.native(), std::is_same_v<T, float> ? LHPC_F32 : LHPC_F64, n_rows, n_cols, K, cuts.data(),
        local.row_ptr.data(), sizeof(OffsetT) * 8, local.col_idx.data(), local.val.data(), flags, opts));
  }
  DistSpMVPlan(const DistSpMVPlan &) = delete;
  DistSpMVPlan &operator=(const DistSpMVPlan &) = delete;
  ~DistSpMVPlan() {
    if (plan_) lhpc_dist_spmv_plan_destroy(plan_);
  }
  std::int64_t rows() const noexcept { return n_rows_; }
  std::int64_t cols() const noexcept { return n_cols_; }
  lhpc_dist_spmv_plan *native() noexcept { return plan_; }

 private:
  lhpc_dist_spmv_plan *plan_ = nullptr;
  std::int64_t n_rows_ = 0, n_cols_ = 0;
};

// y (all n_rows, device) = A·x (all n_cols, device) on every rank; y != x.
template <typename T>
void spmv(DistSpMVPlan<T> &plan, const T *d_x, T *d_y, void *stream = nullptr) {
  lhpc::checkLhpc(lhpc_dist_spmv(plan.native(), d_x, d_y, stream));
}

// Iterative use (y of call n is x of call n+1): begin leaves the exchange of y
// in flight; a begin whose x is the previous begin's y gathers x by column
// part as each exchange chunk lands (cross-step overlap); end waits for it
template <typename T>
void spmv_begin(DistSpMVPlan<T> &plan, const T *d_x, T *d_y, void *stream = nullptr) {
  lhpc::checkLhpc(lhpc_dist_spmv_begin(plan.native(), d_x, d_y, stream));
}
template <typename T>
void spmv_end(DistSpMVPlan<T> &plan, void *stream = nullptr) {
  lhpc::checkLhpc(lhpc_dist_spmv_end(plan.native(), stream));
}

// Conjugate gradient over the distributed plan (lhpc_dist_cg_solve): b, x
// (initial guess in, whole solution out on every rank) and p_work are
// full-length device vectors; returns {iterations, ‖r‖/‖b‖}
template <typename T>
std::pair<int, double> cg(DistSpMVPlan<T> &plan, const T *d_b, T *d_x, T *d_p_work, double tol = 1e-8,
                          int max_iter = 1000, int check_every = 1, void *stream = nullptr) {
  int it = 0;
  double res = 0.0;
  lhpc::checkLhpc(lhpc_dist_cg_solve(plan.native(), d_b, d_x, d_p_work, tol, max_iter, check_every, &it, &res,
                                     stream));
  return {it, res};
}

// the y exchange of a call alone (every chunk; y holds this rank's blocks)
template <typename T>
void exchange(DistSpMVPlan<T> &plan, T *d_y, void *stream = nullptr) {
  lhpc::checkLhpc(lhpc_dist_exchange(plan.native(), d_y, stream));
}

// the transfers lhpc_dist_spmv issues on `rank` (kind LHPC_DIST_EXCHANGE_RCCL / _P2P)
inline std::vector<lhpc_dist_xfer> exchange_schedule(const std::vector<std::int64_t> &cuts, int nranks, int K,
                                                     int rank, int kind = LHPC_DIST_EXCHANGE_RCCL,
                                                     bool broadcast = false) {
  std::vector<lhpc_dist_xfer> v(static_cast<std::size_t>(nranks) * K);
  std::int64_t n = 0;
  lhpc::checkLhpc(lhpc_dist_exchange_schedule(cuts.data(), nranks, K, rank, kind, broadcast ? 1 : 0, v.data(),
                                              static_cast<std::int64_t>(v.size()), &n));
  v.resize(static_cast<std::size_t>(n));
  return v;
}

// One 7-point step on this rank's z-slab (HPCHighDimensionFlatArray<3,float,ghost>
// layout of logical (nzl, ny, nx), device buffers), halo planes over RCCL, or
// stored into the neighbours' ghost planes when d_u is a registered P2P window
// (exchange LHPC_DIST_EXCHANGE_AUTO / _RCCL / _P2P; lhpc_dist_stencil7_f32_x).
inline void dist_stencil7(DistComm &comm, float *d_u, float *d_out, std::int64_t nzl, std::int64_t ny,
                          std::int64_t nx, std::int64_t ghost, float c0, float c1, void *stream = nullptr,
                          int exchange = LHPC_DIST_EXCHANGE_AUTO) {
  lhpc::checkLhpc(lhpc_dist_stencil7_f32_x(comm.native(), d_u, d_out, nzl, ny, nx, ghost, c0, c1, exchange, stream));
}

}  // namespace sparse
#endif  // LHPC_SPARSE_DIST_HPP_
