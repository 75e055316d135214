// lhpc_plan.hpp — host-side plan-time re-encodings of A (built by g++ with
// OpenMP in lhpc_plan.cpp; consumed by the HIP plan in lhpc_spmv.hip).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

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

// XTILE: x tiled by column into S tiles of W columns, each tile small enough
// to sit in one workgroup's LDS (fp32 40960 / fp64 20480 columns = 160 KB).
// Two passes per SpMV:
//   gather : a workgroup loads tile s of x into LDS and streams the tile's
//            nonzeros (col16 = column − s·W), writing xg[g] = x[col] — every
//            x read is an LDS gather, every HBM access is a coalesced stream;
//   reduce : a workgroup owns a chunk of ≤ M consecutive CSR nonzeros, reads
//            the chunk's S segments of xg (one per tile) and scatters them
//            into LDS at perm[g] (the slot xtile_slot(i) of the nonzero's
//            position i in the chunk; cm: i itself), then
//            multiplies by val (CSR order) and sums rows merge-path style.
// The stream is ordered (tile, chunk, CSR position): segment (s, c) is
// [segoff[c·S + s], segoff[(c+1)·S + s]).  Each tile's stream starts at a
// multiple of 8 (padding entries are written by gather, never read).
// Chunks cut the CSR order at row starts where one lies in the back half of
// the M window, else mid-row; a chunk owns the rows that start in it (≤ Rmax)
// and a row cut by a chunk end is finished by a fix-up over `cont`.
//
// cm = true (chunk-major xg, opt-in): gather writes xg in the chunk's
// segment concatenation order — chunk c occupies [ce[c], ce[c+1]) of xg,
// tiles ascending inside it — so reduce reads its chunk as one contiguous run
// and needs no segment table.  Each tile-stream segment is padded to a
// multiple of 8 (padding col16 = 0xFFFF, never stored); gdst[q] is the xg
// position of group q's first entry (a group's entries are contiguous in
// xg), and perm is indexed by xg position.  Pieces are (tile, chunk range)
// pairs ordered so that blocks b with b % 8 == x (one XCD) gather a
// contiguous run of tiles — the xg lines of a chunk are then assembled in
// one L2 — and a whole chunk range before the next (H ranges).
// cm = false: xg is in tile-stream order (tile, chunk, CSR position), perm is
// indexed by stream position, and reduce locates its S segments by segoff.
// pad > 1 (cm = false only): every segment is padded to a multiple of pad
// (pad entries: col16 0, perm = the spare slot M) so that the reduce loads
// pad consecutive positions as one aligned vector; chunks are cut so that
// their padded length stays ≤ M.
struct XtileHost {
  int S = 0;
  int64_t W = 0;
  int M = 0, Rmax = 0;
  bool cm = false;
  int64_t n_chunks = 0;
  int64_t total = 0;                 // padded tile-stream length
  std::vector<int32_t> ce, cr;       // [C+1] chunk first nonzero / first owned row
  std::vector<int32_t> segoff;       // [(C+1)·S] segment starts in the tile stream
  std::vector<int32_t> pieces;       // gather workgroups: (g0, g1, s) triples (g0 == g1: idle)
  std::vector<int32_t> cont;         // chunks whose last owned row runs past the chunk
  std::vector<int64_t> rchunk;       // [n_splits + 2] first chunk of each row range (+ C)
  std::unique_ptr<uint16_t[]> col16;  // [total]
  std::unique_ptr<uint16_t[]> perm;   // [total] (cm: [nnz])
  std::unique_ptr<int32_t[]> gdst;    // cm: [total / 8]
  // iperm mode: [n_chunks·M] — for CSR position i of chunk c, iperm[c·M + i]
  // is its flat position in the chunk's segment concatenation (tiles
  // ascending); perm is then not used by the reduce
  std::unique_ptr<uint16_t[]> iperm;
};

// 0 on success; LHPC_ERR_UNSUPPORTED when the layout does not fit its
// index types (nnz + padding ≥ 2^31, S > 4096, or an oversized segment table).
// piece_nnz: target nonzeros per gather workgroup (multiple of 8 is used;
// cm: the number of chunk ranges H is derived from it).  splits: ascending
// rows in (0, n_rows) at which a chunk must start (row ranges that can be
// reduced separately, lhpc_spmv_range); LHPC_ERR_INVALID_ARG otherwise.
int build_xtile(const void *row_ptr, int rp_bits, const int32_t *col, int64_t n_rows,
                int64_t n_cols, int64_t W, int M, int Rmax, int64_t piece_nnz, bool cm,
                int slot_bytes, const int64_t *splits, int n_splits, XtileHost &out,
                int pad = 1, bool iperm = false);

// LDS slot of chunk position i in the XTILE seg reduce (lhpc_spmv.hip
// xt_slot): run t = i/run holds run = 64/elem_bytes elements (64 B) at
// run·t, its 16-B slot q at q ^ swz(t), swz = (t/4) % 4.
inline int xtile_slot(int i, int elem_bytes) {
  const int vw = 16 / elem_bytes, run = 64 / elem_bytes, t = i / run;
  const int swz = (t >> 2) & 3;
  return (i & ~(run - 1)) | ((((i & (run - 1)) / vw) ^ swz) * vw) | (i & (vw - 1));
}

// in-slice length of row r in slice s
inline int xs_len(const XsliceHost &o, int s, int64_t r) {
  const size_t i = static_cast<size_t>(s) * o.n_rows_pad + r;
  return o.lens_bytes == 1 ? o.lens[i] : reinterpret_cast<const uint16_t *>(o.lens.get())[i];
}

}  // namespace lhpc
