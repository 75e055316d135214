// sparse/IO.hpp — CSRMatrix file I/O: the .lcsr
// container and Matrix Market input, over include/lhpc.h.
//
//   sparse::save_csr("A.lcsr", A);
//   auto B = sparse::load_csr<float, std::int64_t>("A.lcsr");   // dtype/widths must match
//   auto M = sparse::read_matrix_market<double>("matrix.mtx");   // GPU assembly (lhpc_coo_to_csr)
#pragma once
#ifndef LHPC_SPARSE_IO_HPP_
#define LHPC_SPARSE_IO_HPP_

#include <cstdint>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../lhpc.h"
#include "../lhpc_error.hpp"
#include "CSRMatrix.hpp"

namespace sparse {

template <typename T>
constexpr int lhpc_dtype_of() {
  static_assert(std::is_same_v<T, float> || std::is_same_v<T, double>, "float or double");
  return std::is_same_v<T, float> ? LHPC_F32 : LHPC_F64;
}

template <typename T, typename IndexT, typename OffsetT>
void save_csr(const std::string &path, const CSRMatrix<T, IndexT, OffsetT> &A) {
  lhpc::checkLhpc(lhpc_csr_save(path.c_str(), lhpc_dtype_of<T>(), A.n_rows, A.n_cols, A.nnz(), A.row_ptr.data(),
                                static_cast<int>(sizeof(OffsetT) * 8),
                                reinterpret_cast<const std::int32_t *>(A.col_idx.data()), A.val.data()));
}

template <typename T, typename OffsetT = std::int32_t, typename IndexT = std::int32_t>
CSRMatrix<T, IndexT, OffsetT> load_csr(const std::string &path) {
  int dtype = 0, rpbits = 0;
  std::int64_t n_rows = 0, n_cols = 0, nnz = 0;
  lhpc::checkLhpc(lhpc_csr_load_header(path.c_str(), &dtype, &n_rows, &n_cols, &nnz, &rpbits));
  if (dtype != lhpc_dtype_of<T>() || rpbits != static_cast<int>(sizeof(OffsetT) * 8))
    throw std::invalid_argument("load_csr: file dtype / row_ptr width differ from the requested CSRMatrix type");
  CSRMatrix<T, IndexT, OffsetT> A(n_rows, n_cols);
  A.col_idx.resize(static_cast<std::size_t>(nnz));
  A.val.resize(static_cast<std::size_t>(nnz));
  lhpc::checkLhpc(lhpc_csr_load(path.c_str(), A.row_ptr.data(), reinterpret_cast<std::int32_t *>(A.col_idx.data()),
                                A.val.data()));
  return A;
}

template <typename T, typename OffsetT = std::int32_t, typename IndexT = std::int32_t>
CSRMatrix<T, IndexT, OffsetT> read_matrix_market(const std::string &path) {
  std::int64_t n_rows = 0, n_cols = 0, zmax = 0, count = 0;
  int sym = 0, field = 0;
  lhpc::checkLhpc(lhpc_mm_read_header(path.c_str(), &n_rows, &n_cols, &zmax, &sym, &field));
  std::vector<std::int32_t> rows(static_cast<std::size_t>(zmax)), cols(static_cast<std::size_t>(zmax));
  std::vector<double> v64(static_cast<std::size_t>(zmax));
  lhpc::checkLhpc(lhpc_mm_read_coo(path.c_str(), rows.data(), cols.data(), v64.data(), &count));
  std::vector<T> vals(v64.begin(), v64.begin() + count);
  CSRMatrix<T, IndexT, OffsetT> A(n_rows, n_cols);
  A.col_idx.resize(static_cast<std::size_t>(count));
  A.val.resize(static_cast<std::size_t>(count));
  std::int64_t merged = 0;
  lhpc::checkLhpc(lhpc_coo_to_csr(lhpc_dtype_of<T>(), n_rows, n_cols, count, rows.data(), cols.data(), vals.data(),
                                  A.row_ptr.data(), static_cast<int>(sizeof(OffsetT) * 8),
                                  reinterpret_cast<std::int32_t *>(A.col_idx.data()), A.val.data(), &merged, 0,
                                  nullptr));
  A.col_idx.resize(static_cast<std::size_t>(merged));
  A.val.resize(static_cast<std::size_t>(merged));
  return A;
}

}  // namespace sparse
#endif  // LHPC_SPARSE_IO_HPP_
