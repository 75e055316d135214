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
  int lens_bytes = 1;                 // 1: uint8 lengths, 2: uint16 (some row > 255 in a slice)
  std::unique_ptr<uint8_t[]> lens;    // [S][n_rows_pad] in-slice row lengths, lens_bytes each
  std::unique_ptr<int64_t[]> cbase;   // [S·n_chunks + 1] chunk start offsets
  std::unique_ptr<int32_t[]> col;     // [nnz]
  std::unique_ptr<unsigned char[]> val;  // [nnz · tsz]
};

// 0 on success; LHPC_ERR_UNSUPPORTED when some row has > 65535 nonzeros in
// one slice, or > 255 with allow16 = false (the jagged kernel is uint8-only).
int build_xslice(const void *row_ptr, int rp_bits, const int32_t *col, const void *val,
                 size_t tsz, int64_t n_rows, int64_t n_cols, int S, bool jagged, XsliceHost &out);

// in-slice length of row r in slice s
inline int xs_len(const XsliceHost &o, int s, int64_t r) {
  const size_t i = static_cast<size_t>(s) * o.n_rows_pad + r;
  return o.lens_bytes == 1 ? o.lens[i] : reinterpret_cast<const uint16_t *>(o.lens.get())[i];
}

}  // namespace lhpc
