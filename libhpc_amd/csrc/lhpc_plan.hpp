// lhpc_plan.hpp — host-side plan-time re-encodings of A (built by g++ with
// OpenMP in lhpc_plan.cpp; consumed by the HIP plan in lhpc_spmv.hip).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>

namespace lhpc {

// XSLICE: A split by column into S slices of `width` columns; inside a
// slice, rows are grouped in 64-row chunks (one wave per chunk).  A chunk's
// nonzeros are stored either
//   jagged = true : jagged-diagonal order — all rows' 1st in-slice element,
//                   then all 2nd elements, ... (lane-per-row kernel), or
//   jagged = false: CSR order — row by row (stream kernel: the wave loads the
//                   chunk's elements contiguously, products go through LDS).
// Element j of a row is its j-th in-slice element in the caller's order, so
// each row accumulates in its CSR order either way.
struct XsliceHost {
  int S = 0;
  int64_t width = 0;
  int64_t n_rows = 0, n_chunks = 0, n_rows_pad = 0;  // n_rows_pad = 64·n_chunks
  int64_t nnz = 0;
  int64_t max_chunk = 0;  // largest chunk (nonzeros of one (slice, chunk))
  std::unique_ptr<uint8_t[]> lens;    // [S][n_rows_pad] in-slice row lengths (<= 255)
  std::unique_ptr<int64_t[]> cbase;   // [S·n_chunks + 1] chunk start offsets
  std::unique_ptr<int32_t[]> col;     // [nnz]
  std::unique_ptr<unsigned char[]> val;  // [nnz · tsz]
};

// 0 on success; LHPC_ERR_UNSUPPORTED when some row has > 255 nonzeros in one
// slice (the caller then keeps a non-sliced kernel).
int build_xslice(const void *row_ptr, int rp_bits, const int32_t *col, const void *val,
                 size_t tsz, int64_t n_rows, int64_t n_cols, int S, bool jagged, XsliceHost &out);

}  // namespace lhpc
