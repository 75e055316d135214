// sparse/DeviceCSR.hpp — a CSR matrix resident in HBM, assembled on the GPU
// from the reference's sparse grid, and handed to the SpMV without a host
// round trip (RootGrid → COO → GPU radix sort → CSR → SpMV).
//
//   auto b  = sparse::bounds(grid);
//   auto dA = sparse::to_csr_device<float>(grid, b, /*device=*/0);  // DeviceCSR<float>
//   sparse::SpMVPlan<float> plan(dA.view());   // XTILE layout built on the GPU
//
// The grid walk (foreach, reference lib/sparse/include/RootGrid.hpp:20-22)
// is host code; its COO triples go to HBM once, lhpc_coo_to_csr sorts and
// assembles them there, and LHPC_PLAN_DEVICE_INPUT builds the plan from the
// device arrays.  Needs the HIP runtime (the arrays are hipMalloc'd).
#pragma once
#ifndef LHPC_SPARSE_DEVICECSR_HPP_
#define LHPC_SPARSE_DEVICECSR_HPP_

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <stdexcept>
#include <type_traits>
#include <utility>
#include <vector>

#include "../lhpc.h"
#include "../lhpc_error.hpp"
#include "RootGrid.hpp"
#include "SpMV.hpp"
#include "ToCSR.hpp"

namespace sparse {

// RAII owner of device row_ptr (int32), col_idx and val on one device
template <typename T>
class DeviceCSR {
  static_assert(std::is_same_v<T, float> || std::is_same_v<T, double>, "DeviceCSR is fp32 or fp64");

 public:
  DeviceCSR() = default;
  DeviceCSR(std::int64_t n_rows, std::int64_t n_cols, std::int64_t nnz_capacity, int device)
      : n_rows_(n_rows), n_cols_(n_cols), device_(device) {
    hip(hipSetDevice(device));
    hip(hipMalloc(&row_ptr_, sizeof(std::int32_t) * static_cast<std::size_t>(n_rows + 1)));
    hip(hipMalloc(&col_, sizeof(std::int32_t) * static_cast<std::size_t>(nnz_capacity > 0 ? nnz_capacity : 1)));
    hip(hipMalloc(&val_, sizeof(T) * static_cast<std::size_t>(nnz_capacity > 0 ? nnz_capacity : 1)));
  }
  DeviceCSR(const DeviceCSR &) = delete;
  DeviceCSR &operator=(const DeviceCSR &) = delete;
  DeviceCSR(DeviceCSR &&o) noexcept { swap(o); }
  DeviceCSR &operator=(DeviceCSR &&o) noexcept {
    if (this != &o) {
      release();
      swap(o);
    }
    return *this;
  }
  ~DeviceCSR() { release(); }

  DeviceCSRView<T> view() const {
    DeviceCSRView<T> v;
    v.n_rows = n_rows_;
    v.n_cols = n_cols_;
    v.nnz = nnz_;
    v.row_ptr = row_ptr_;
    v.row_ptr_bits = 32;
    v.col_idx = col_;
    v.val = val_;
    v.device = device_;
    return v;
  }
  std::int64_t nnz() const noexcept { return nnz_; }
  std::int32_t *row_ptr() noexcept { return row_ptr_; }
  std::int32_t *col_idx() noexcept { return col_; }
  T *val() noexcept { return val_; }
  void set_nnz(std::int64_t nnz) noexcept { nnz_ = nnz; }

 private:
  static void hip(hipError_t e) {
    if (e != hipSuccess) lhpc::throwLhpcError(static_cast<int>(e), __FILE__, __LINE__);
  }
  void release() noexcept {
    if (row_ptr_ || col_ || val_) (void)hipSetDevice(device_);
    if (row_ptr_) (void)hipFree(row_ptr_);
    if (col_) (void)hipFree(col_);
    if (val_) (void)hipFree(val_);
    row_ptr_ = col_ = nullptr;
    val_ = nullptr;
  }
  void swap(DeviceCSR &o) noexcept {
    std::swap(n_rows_, o.n_rows_);
    std::swap(n_cols_, o.n_cols_);
    std::swap(nnz_, o.nnz_);
    std::swap(device_, o.device_);
    std::swap(row_ptr_, o.row_ptr_);
    std::swap(col_, o.col_);
    std::swap(val_, o.val_);
  }
  std::int64_t n_rows_ = 0, n_cols_ = 0, nnz_ = 0;
  int device_ = 0;
  std::int32_t *row_ptr_ = nullptr, *col_ = nullptr;
  T *val_ = nullptr;
};

// The grid's kept cells inside the window → COO in HBM → lhpc_coo_to_csr on
// the device (duplicates cannot occur: the grid is a map)
template <typename V, typename T, typename Layout, typename Keep = NonZero>
DeviceCSR<V> to_csr_device(const RootGrid<T, Layout> &grid, std::intptr_t row0, std::intptr_t col0,
                           std::int64_t n_rows, std::int64_t n_cols, int device = 0, Keep keep = {}) {
  if (n_rows < 0 || n_cols < 0 || n_rows > INT32_MAX || n_cols > INT32_MAX)
    throw std::invalid_argument("to_csr_device: window dimensions must be in [0, 2^31)");
  std::vector<std::int32_t> rows, cols;
  std::vector<V> vals;
  grid.foreach ([&](std::intptr_t x, std::intptr_t y, const T &v) {
    if (!keep(v)) return;
    const std::intptr_t r = x - row0, c = y - col0;
    if (r < 0 || r >= n_rows || c < 0 || c >= n_cols)
      throw std::out_of_range("to_csr_device: grid cell outside the window");
    rows.push_back(static_cast<std::int32_t>(r));
    cols.push_back(static_cast<std::int32_t>(c));
    vals.push_back(static_cast<V>(v));
  });
  const std::int64_t nnz = static_cast<std::int64_t>(rows.size());
  DeviceCSR<V> A(n_rows, n_cols, nnz, device);
  void *dr = nullptr, *dc = nullptr, *dv = nullptr;
  auto hip = [](hipError_t e) {
    if (e != hipSuccess) lhpc::throwLhpcError(static_cast<int>(e), __FILE__, __LINE__);
  };
  const std::size_t b = static_cast<std::size_t>(nnz > 0 ? nnz : 1);
  hip(hipMalloc(&dr, 4 * b));
  hip(hipMalloc(&dc, 4 * b));
  hip(hipMalloc(&dv, sizeof(V) * b));
  struct Free {
    void *a, *b, *c;
    ~Free() {
      (void)hipFree(a);
      (void)hipFree(b);
      (void)hipFree(c);
    }
  } fr{dr, dc, dv};
  if (nnz) {
    hip(hipMemcpy(dr, rows.data(), 4 * static_cast<std::size_t>(nnz), hipMemcpyHostToDevice));
    hip(hipMemcpy(dc, cols.data(), 4 * static_cast<std::size_t>(nnz), hipMemcpyHostToDevice));
    hip(hipMemcpy(dv, vals.data(), sizeof(V) * static_cast<std::size_t>(nnz), hipMemcpyHostToDevice));
  }
  std::int64_t merged = 0;
  lhpc::checkLhpc(lhpc_coo_to_csr(std::is_same_v<V, float> ? LHPC_F32 : LHPC_F64, n_rows, n_cols, nnz,
                                  static_cast<const std::int32_t *>(dr), static_cast<const std::int32_t *>(dc), dv,
                                  A.row_ptr(), 32, A.col_idx(), A.val(), &merged, /*on_device=*/1, nullptr));
  A.set_nnz(merged);
  return A;
}

template <typename V, typename T, typename Layout, typename Keep = NonZero>
DeviceCSR<V> to_csr_device(const RootGrid<T, Layout> &grid, const GridBounds &b, int device = 0, Keep keep = {}) {
  return to_csr_device<V>(grid, b.row_min, b.col_min, b.n_rows(), b.n_cols(), device, keep);
}

}  // namespace sparse
#endif  // LHPC_SPARSE_DEVICECSR_HPP_
