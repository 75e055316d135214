// sparse/ToCSR.hpp — RootGrid → CSRMatrix assembly.
//
// Connects the reference's sparse-grid API (lib/sparse/include/RootGrid.hpp:20-22,
// foreach) to the SpMV path: foreach → COO triples → GPU radix sort by
// (row, col) → CSR (lhpc_coo_to_csr, include/lhpc.h).  Grid coordinate x is
// the row and y the column (the leaf tile is x-major, DenseBlock.hpp), shifted
// by a caller-chosen window origin.
//
//   auto A = sparse::to_csr<float>(grid, row0, col0, n_rows, n_cols);
//   auto b = sparse::bounds(grid);             // bounding box of the kept cells
//   auto B = sparse::to_csr<double>(grid, b);  // window = bounding box
//
// A cell is kept when keep(value) is true (default: value != T{} — the
// reference benchmarks count `if (value)`, test_hpc_benchmark.cpp:873-876);
// the stored value is static_cast<V>(value).  Kept cells outside the window
// throw std::out_of_range (like HPCHighDimensionFlatArray::at).  The grid is
// a map, so there are no duplicate coordinates.
#pragma once
#ifndef LHPC_SPARSE_TOCSR_HPP_
#define LHPC_SPARSE_TOCSR_HPP_

#include <cstdint>
#include <limits>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "../lhpc.h"
#include "../lhpc_error.hpp"
#include "CSRMatrix.hpp"
#include "RootGrid.hpp"

namespace sparse {

struct NonZero {
  template <typename T>
  bool operator()(const T &v) const {
    return !(v == T{});
  }
};

struct GridBounds {
  std::intptr_t row_min = 0, row_max = -1;  // inclusive; empty when row_max < row_min
  std::intptr_t col_min = 0, col_max = -1;
  std::int64_t count = 0;
  std::int64_t n_rows() const { return count ? row_max - row_min + 1 : 0; }
  std::int64_t n_cols() const { return count ? col_max - col_min + 1 : 0; }
};

template <typename T, typename Layout, typename Keep = NonZero>
GridBounds bounds(const RootGrid<T, Layout> &grid, Keep keep = {}) {
  GridBounds b;
  b.row_min = b.col_min = std::numeric_limits<std::intptr_t>::max();
  b.row_max = b.col_max = std::numeric_limits<std::intptr_t>::min();
  grid.foreach ([&](std::intptr_t x, std::intptr_t y, const T &v) {
    if (!keep(v)) return;
    ++b.count;
    if (x < b.row_min) b.row_min = x;
    if (x > b.row_max) b.row_max = x;
    if (y < b.col_min) b.col_min = y;
    if (y > b.col_max) b.col_max = y;
  });
  if (!b.count) b = GridBounds{};
  return b;
}

template <typename V, typename IndexT = std::int32_t, typename OffsetT = std::int32_t, typename T, typename Layout,
          typename Keep = NonZero>
CSRMatrix<V, IndexT, OffsetT> to_csr(const RootGrid<T, Layout> &grid, std::intptr_t row0, std::intptr_t col0,
                                     std::int64_t n_rows, std::int64_t n_cols, Keep keep = {}) {
  static_assert(std::is_same_v<V, float> || std::is_same_v<V, double>, "to_csr: V is float or double");
  if (n_rows < 0 || n_cols < 0 || n_rows > std::numeric_limits<std::int32_t>::max() ||
      n_cols > std::numeric_limits<std::int32_t>::max())
    throw std::invalid_argument("to_csr: window dimensions must be in [0, 2^31)");
  std::vector<std::int32_t> rows, cols;
  std::vector<V> vals;
  grid.foreach ([&](std::intptr_t x, std::intptr_t y, const T &v) {
    if (!keep(v)) return;
    const std::intptr_t r = x - row0, c = y - col0;
    if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) throw std::out_of_range("to_csr: grid cell outside the window");
    rows.push_back(static_cast<std::int32_t>(r));
    cols.push_back(static_cast<std::int32_t>(c));
    vals.push_back(static_cast<V>(v));
  });
  CSRMatrix<V, IndexT, OffsetT> A(n_rows, n_cols);
  const std::int64_t nnz = static_cast<std::int64_t>(rows.size());
  A.col_idx.resize(static_cast<std::size_t>(nnz));
  A.val.resize(static_cast<std::size_t>(nnz));
  std::int64_t merged = 0;
  lhpc::checkLhpc(lhpc_coo_to_csr(std::is_same_v<V, float> ? LHPC_F32 : LHPC_F64, n_rows, n_cols, nnz, rows.data(),
                            cols.data(), vals.data(), A.row_ptr.data(), static_cast<int>(sizeof(OffsetT) * 8),
                            reinterpret_cast<std::int32_t *>(A.col_idx.data()), A.val.data(), &merged,
                            /*on_device=*/0, /*stream=*/nullptr));
  A.col_idx.resize(static_cast<std::size_t>(merged));
  A.val.resize(static_cast<std::size_t>(merged));
  return A;
}

template <typename V, typename IndexT = std::int32_t, typename OffsetT = std::int32_t, typename T, typename Layout,
          typename Keep = NonZero>
CSRMatrix<V, IndexT, OffsetT> to_csr(const RootGrid<T, Layout> &grid, const GridBounds &b, Keep keep = {}) {
  return to_csr<V, IndexT, OffsetT>(grid, b.row_min, b.col_min, b.n_rows(), b.n_cols(), keep);
}

}  // namespace sparse
#endif  // LHPC_SPARSE_TOCSR_HPP_
