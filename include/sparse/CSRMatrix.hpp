// sparse/CSRMatrix.hpp — CSR matrix type in the reference's `sparse` namespace.
//
// The reference has no CSR; this follows its idiom: header-only,
// namespace sparse (lib/sparse/include/RootGrid.hpp:10), storage in
// std::vector with hpc::AlignedAllocator<_, 64> (lib/hpc/include/AlignedAlloc.hpp:29).
// Canonical form: row_ptr[0] == 0, non-decreasing, row_ptr[n_rows] == nnz,
// and column indices strictly ascending inside each row.
#pragma once
#ifndef LHPC_SPARSE_CSR_MATRIX_HPP_
#define LHPC_SPARSE_CSR_MATRIX_HPP_

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

#include "../hpc/AlignedAlloc.hpp"

namespace sparse {

template <typename T>
using aligned_vector = std::vector<T, hpc::AlignedAllocator<T, 64>>;

template <typename T, typename IndexT = std::int32_t, typename OffsetT = std::int32_t>
struct CSRMatrix {
  static_assert(sizeof(IndexT) == 4, "column indices are int32 on the device path");
  static_assert(sizeof(OffsetT) == 4 || sizeof(OffsetT) == 8, "row_ptr is int32 or int64");
  using value_type = T;
  using index_type = IndexT;
  using offset_type = OffsetT;

  std::int64_t n_rows = 0;
  std::int64_t n_cols = 0;
  aligned_vector<OffsetT> row_ptr;  // n_rows + 1
  aligned_vector<IndexT> col_idx;   // nnz
  aligned_vector<T> val;            // nnz

  CSRMatrix() : row_ptr(1, OffsetT(0)) {}
  CSRMatrix(std::int64_t rows, std::int64_t cols)
      : n_rows(rows), n_cols(cols), row_ptr(static_cast<std::size_t>(rows + 1), OffsetT(0)) {}

  std::int64_t nnz() const noexcept { return static_cast<std::int64_t>(col_idx.size()); }

  // Throws std::invalid_argument describing the first violation.
  void validate(bool require_sorted = true) const {
    if (static_cast<std::int64_t>(row_ptr.size()) != n_rows + 1)
      throw std::invalid_argument("row_ptr size != n_rows + 1");
    if (row_ptr.front() != 0 || static_cast<std::int64_t>(row_ptr.back()) != nnz())
      throw std::invalid_argument("row_ptr must start at 0 and end at nnz");
    if (val.size() != col_idx.size()) throw std::invalid_argument("val/col_idx size mismatch");
    for (std::int64_t i = 0; i < n_rows; ++i) {
      const auto s = row_ptr[static_cast<std::size_t>(i)], e = row_ptr[static_cast<std::size_t>(i + 1)];
      if (e < s) throw std::invalid_argument("row_ptr not monotone at row " + std::to_string(i));
      for (auto k = s; k < e; ++k) {
        const auto c = col_idx[static_cast<std::size_t>(k)];
        if (c < 0 || c >= n_cols) throw std::invalid_argument("column out of range in row " + std::to_string(i));
        if (require_sorted && k > s && col_idx[static_cast<std::size_t>(k - 1)] >= c)
          throw std::invalid_argument("columns not strictly ascending in row " + std::to_string(i));
      }
    }
  }
};

}  // namespace sparse
#endif  // LHPC_SPARSE_CSR_MATRIX_HPP_
