// sparse/SpMV.hpp — y = A·x on MI355X behind the reference's host types.
//
//   sparse::SpMVPlan<T>  RAII owner of the HBM copy of A (one per GPU)
//   sparse::spmv(plan, x, y)  with x, y hpc::HPCHighDimensionFlatArray<1,T,...>
//   sparse::default_options()  lhpc_options for pinning a kernel variant
//                             (host, synchronous) or raw HBM pointers (async)
// Forwards to the C ABI (include/lhpc.h); non-zero status → std::system_error
// (include/lhpc_error.hpp).  The reference has no SpMV; the
// operator and its numerics are defined in DESIGN.md.
#pragma once
#ifndef LHPC_SPARSE_SPMV_HPP_
#define LHPC_SPARSE_SPMV_HPP_

#include <cstdint>
#include <type_traits>
#include <utility>
#include <vector>

#include "../hpc/HPCHighDimensionFlatArray.hpp"
#include "../lhpc.h"
#include "../lhpc_error.hpp"
#include "CSRMatrix.hpp"

namespace sparse {

// Variant options (include/lhpc.h lhpc_options), initialised to automatic:
//   auto o = sparse::default_options(); o.xtile_reduce = LHPC_XTILE_REDUCE_PERM;
inline lhpc_options default_options() {
  lhpc_options o;
  lhpc_options_init(&o);
  return o;
}

// A CSR matrix whose arrays already live in HBM of one device (e.g. the
// output of lhpc_coo_to_csr on the device, sparse/DeviceCSR.hpp): the plan is
// built from it without a host round trip (LHPC_PLAN_DEVICE_INPUT).
template <typename T>
struct DeviceCSRView {
  std::int64_t n_rows = 0, n_cols = 0, nnz = 0;
  const void *row_ptr = nullptr;  // n_rows + 1 offsets, int32 or int64
  int row_ptr_bits = 32;
  const std::int32_t *col_idx = nullptr;
  const T *val = nullptr;
  int device = 0;
};

template <typename T>
class SpMVPlan {
  static_assert(std::is_same_v<T, float> || std::is_same_v<T, double>, "SpMV is fp32 or fp64");

 public:
  // One host thread driving several GPUs: the rows are split into
  // devices.size()·K nnz-balanced blocks, one local plan, stream and comm
  // stream per device (lhpc_spmv_plan_create with n_devices > 1).  spmv(plan,
  // x, y) then takes host vectors (or device pointers on devices[0]);
  // spmv_multi keeps full replicas on every device.
  template <typename OffsetT>
  SpMVPlan(const CSRMatrix<T, std::int32_t, OffsetT> &A, const std::vector<int> &devices,
           unsigned flags = LHPC_PLAN_DEFAULT, const lhpc_options *opts = nullptr)
      : n_rows_(A.n_rows), n_cols_(A.n_cols), n_devices_(static_cast<int>(devices.size())) {
    lhpc::checkLhpc(lhpc_spmv_plan_create_opts(&plan_, std::is_same_v<T, float> ? LHPC_F32 : LHPC_F64, A.n_rows,
                                               A.n_cols, A.nnz(), A.row_ptr.data(), sizeof(OffsetT) * 8,
                                               A.col_idx.data(), A.val.data(), devices.data(),
                                               static_cast<int>(devices.size()), flags, 0, nullptr, opts));
  }
  explicit SpMVPlan(const DeviceCSRView<T> &A, unsigned flags = LHPC_PLAN_DEFAULT,
                    const lhpc_options *opts = nullptr)
      : n_rows_(A.n_rows), n_cols_(A.n_cols) {
    const int dev[1] = {A.device};
    lhpc::checkLhpc(lhpc_spmv_plan_create_opts(&plan_, std::is_same_v<T, float> ? LHPC_F32 : LHPC_F64, A.n_rows,
                                               A.n_cols, A.nnz, A.row_ptr, A.row_ptr_bits, A.col_idx, A.val, dev, 1,
                                               flags | LHPC_PLAN_DEVICE_INPUT, 0, nullptr, opts));
  }
  template <typename OffsetT>
  explicit SpMVPlan(const CSRMatrix<T, std::int32_t, OffsetT> &A, int device = -1,
                    unsigned flags = LHPC_PLAN_DEFAULT, const lhpc_options *opts = nullptr)
      : n_rows_(A.n_rows), n_cols_(A.n_cols) {
    const int dev[1] = {device};
    lhpc::checkLhpc(lhpc_spmv_plan_create_opts(&plan_, std::is_same_v<T, float> ? LHPC_F32 : LHPC_F64,
                                               A.n_rows, A.n_cols, A.nnz(), A.row_ptr.data(),
                                               sizeof(OffsetT) * 8, A.col_idx.data(), A.val.data(),
                                               device >= 0 ? dev : nullptr, device >= 0 ? 1 : 0, flags, 0, nullptr,
                                               opts));
  }
  SpMVPlan(const SpMVPlan &) = delete;
  SpMVPlan &operator=(const SpMVPlan &) = delete;
  SpMVPlan(SpMVPlan &&o) noexcept
      : plan_(std::exchange(o.plan_, nullptr)), n_rows_(o.n_rows_), n_cols_(o.n_cols_), n_devices_(o.n_devices_) {}
  SpMVPlan &operator=(SpMVPlan &&o) noexcept {
    if (this != &o) {
      reset();
      plan_ = std::exchange(o.plan_, nullptr);
      n_rows_ = o.n_rows_;
      n_cols_ = o.n_cols_;
      n_devices_ = o.n_devices_;
    }
    return *this;
  }
  ~SpMVPlan() { reset(); }

  lhpc_spmv_plan_info info() const {
    lhpc_spmv_plan_info i{};
    lhpc::checkLhpc(lhpc_spmv_plan_info_get(plan_, &i));
    return i;
  }
  std::int64_t rows() const noexcept { return n_rows_; }
  std::int64_t cols() const noexcept { return n_cols_; }
  int devices() const noexcept { return n_devices_; }
  lhpc_spmv_plan *native() noexcept { return plan_; }

 private:
  void reset() noexcept {
    if (plan_) lhpc_spmv_plan_destroy(plan_);
    plan_ = nullptr;
  }
  lhpc_spmv_plan *plan_ = nullptr;
  std::int64_t n_rows_ = 0, n_cols_ = 0;
  int n_devices_ = 1;
};

// Host vectors: the logical cells [0, n) of 1-D flat arrays (ghost cells, if
// any, are skipped and left untouched).  Synchronous.
template <typename T, std::size_t LX, std::size_t HX, std::size_t AX, class AlX, std::size_t LY,
          std::size_t HY, std::size_t AY, class AlY>
void spmv(SpMVPlan<T> &plan, const hpc::HPCHighDimensionFlatArray<1, T, LX, HX, AX, AlX> &x,
          hpc::HPCHighDimensionFlatArray<1, T, LY, HY, AY, AlY> &y) {
  if (static_cast<std::int64_t>(x.dims()[0]) < plan.cols() ||
      static_cast<std::int64_t>(y.dims()[0]) < plan.rows())
    lhpc::throwLhpcError(LHPC_ERR_INVALID_ARG, __FILE__, __LINE__);
  lhpc::checkLhpc(lhpc_spmv(plan.native(), x.data() + LX, y.data() + LY, 0, nullptr));
}

// Device vectors (HBM pointers), asynchronous on `stream` (a hipStream_t).
template <typename T>
void spmv(SpMVPlan<T> &plan, const T *d_x, T *d_y, void *stream = nullptr) {
  lhpc::checkLhpc(lhpc_spmv(plan.native(), d_x, d_y, 1, stream));
}

// Multi-device plan, full replicas: d_x[d] / d_y[d] on device d; afterwards
// every d_y[d] holds the whole y (lhpc_spmv_multi).  streams: one per device
// (nullptr: the plan's own streams).
template <typename T>
void spmv_multi(SpMVPlan<T> &plan, const std::vector<const T *> &d_x, const std::vector<T *> &d_y,
                const std::vector<void *> *streams = nullptr) {
  if (static_cast<int>(d_x.size()) != plan.devices() || static_cast<int>(d_y.size()) != plan.devices() ||
      (streams && static_cast<int>(streams->size()) != plan.devices()))
    lhpc::throwLhpcError(LHPC_ERR_INVALID_ARG, __FILE__, __LINE__);
  std::vector<const void *> xs(d_x.begin(), d_x.end());
  std::vector<void *> ys(d_y.begin(), d_y.end());
  lhpc::checkLhpc(lhpc_spmv_multi(plan.native(), xs.data(), ys.data(), streams ? streams->data() : nullptr));
}

}  // namespace sparse
#endif  // LHPC_SPARSE_SPMV_HPP_
