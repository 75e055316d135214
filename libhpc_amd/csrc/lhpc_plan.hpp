// lhpc_plan.hpp — host-side plan-time re-encodings of A (built by g++ with
// OpenMP in lhpc_plan.cpp; consumed by the HIP plans in lhpc_spmv_*.hip).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace lhpc {

// CSR sanity, always run by lhpc_spmv_plan_create before any layout pass
// indexes host arrays by row_ptr or col_idx: row_ptr[0] == 0, row_ptr
// non-decreasing, row_ptr[n_rows] == nnz, every col_idx in [0, n_cols).
// 0 or LHPC_ERR_BAD_CSR.  OpenMP, one pass over row_ptr and col_idx.
int validate_csr(const void *row_ptr, int rp_bits, const int32_t *col, int64_t n_rows, int64_t n_cols,
                 int64_t nnz);

// XTILE column blocks: rows [r0, r1) of A restricted to columns [c0, c1),
// columns rebased to c0, each row's nonzeros in the caller's order.  out_rp
// gets r1 − r0 + 1 offsets; out_col / out_val are resized to the block's
// nonzeros (tsz bytes per value).  OpenMP: count per row, scan, fill.
void csr_column_block(const void *row_ptr, int rp_bits, const int32_t *col, const void *val, size_t tsz,
                      int64_t r0, int64_t r1, int64_t c0, int64_t c1, std::vector<int64_t> &out_rp,
                      std::vector<int32_t> &out_col, std::vector<unsigned char> &out_val);

// XSLICE: A split by column into S slices of `width` columns; inside a
// slice, rows are grouped in 64-row chunks (one wave per chunk), and a
// chunk's in-slice nonzeros are stored in CSR order (row by row; the wave
// loads them contiguously and stages the products in LDS).  Element j of a
// row is its j-th in-slice element in the caller's order, so each row
// accumulates in its CSR order.
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
// one slice.
int build_xslice(const void *row_ptr, int rp_bits, const int32_t *col, const void *val,
                 size_t tsz, int64_t n_rows, int64_t n_cols, int S, XsliceHost &out);

// XTILE: x tiled by column into S tiles of W columns, each tile small enough
// to sit in one workgroup's LDS (fp32 40960 / fp64 20480 columns = 160 KB).
// Two passes per SpMV:
//   gather : a workgroup loads tile s of x into LDS and streams the tile's
//            nonzeros (col16 = column − s·W), writing xg[g] = x[col] — every
//            x read is an LDS gather, every HBM access is a coalesced stream;
//   reduce : a workgroup owns a chunk of ≤ M consecutive CSR nonzeros and
//            reads the chunk's S segments of xg (one per tile).  perm mode
//            scatters them into LDS at perm[g] (the slot xtile_slot(i) of the
//            nonzero's chunk position i); iperm mode keeps them in flat order
//            (the chunk's segment concatenation, tiles ascending) and gathers
//            CSR position i's x from flat slot iperm[e0 + i].  Then it
//            multiplies by val (CSR order) and sums rows merge-path style.
// The stream is ordered (tile, chunk, CSR position): segment (s, c) is
// [segoff[c·S + s], segoff[(c+1)·S + s]).  Each tile's stream starts at a
// multiple of 8 (padding entries are written by gather, never read); with
// unit > 1 every segment's length is also a multiple of `unit`.
// Chunks cut the CSR order at the last row start in the back `cut_window`
// entries of the M window, else mid-row (so every chunk but a range's last
// holds ≥ M − cut_window nonzeros); a chunk owns the rows that start in it
// (≤ Rmax) and a row cut by a chunk end is finished by a fix-up over `cont`.
struct XtileHost {
  int S = 0;
  int64_t W = 0;
  int M = 0, Rmax = 0;
  int unit = 1;                      // every segment padded to a multiple of `unit` entries
  int64_t n_chunks = 0;
  int64_t total = 0;                 // padded tile-stream length
  std::vector<int32_t> ce, cr;       // [C+1] chunk first nonzero / first owned row
  std::vector<int32_t> segoff;       // [(C+1)·S] segment starts in the tile stream
  std::vector<int32_t> pieces;       // gather workgroups: (g0, g1, s) triples
  std::vector<int32_t> cont;         // chunks whose last owned row runs past the chunk
  std::vector<int64_t> rchunk;       // [n_splits + 2] first chunk of each row range (+ C)
  std::unique_ptr<uint16_t[]> col16;  // [total]
  std::unique_ptr<uint16_t[]> perm;   // perm mode: [total]
  // iperm mode: [nnz] in CSR order — for nonzero k of chunk c, iperm[k] is its
  // flat position in the chunk's segment concatenation (tiles ascending)
  std::unique_ptr<uint16_t[]> iperm;
  bool iperm_mode = false;           // which reduce index stream the plan carries
  int slot_bytes = 4;
  // xg ring (xtile_ring_pieces; cache-sized ranges): one range-sized xg buffer
  // reused by every range.  Range k's part of tile s (sub-run (k, s) =
  // [segoff[rchunk[k]][s], segoff[rchunk[k+1]][s]) of the tile-major stream)
  // lives at stream position + rdelta[k·S + s] in the ring (a multiple of 8);
  // ring_len = the longest range's ring.  pext: 2 int32 per piece {delta,
  // flags}: bit 0 also gathers the 8-entry group before the piece, bit 1 the
  // group at its end (the groups two ranges share, unpermuted).  hrow[k]:
  // range k's first segment-table hi row (hi groups restart at each range).
  std::vector<int32_t> rdelta, pext;
  std::vector<int64_t> hrow;
  int64_t ring_len = 0;
};

// Device form of the segment table (the reduce reads one 4-B word per tile
// and chunk instead of two starts): seg[c·S + s] = lo | len << 16 with
// start(c, s) = hi[⌊c / kXtSegHi⌋·S + s] + lo (ring plans: ring starts,
// hi row hrow[k] + ⌊(c − rchunk[k]) / kXtSegHi⌋ for c in range k) and len = start(c+1, s) −
// start(c, s) ≤ M; lo ≤ (kXtSegHi − 1)·M < 2^16 for M ≤ 8192.  Size ≈ 4.6 B
// per (chunk, tile): 21 MB for C2, 1.3 GB at n = 80M (where a dense int32
// table of starts hit the old 2.7e8-entry limit).
#ifndef LHPC_XT_SEGHI
#define LHPC_XT_SEGHI 7  // (kXtSegHi − 1)·M < 2^16: 7 for M = 8192, 4 for M = 16384
#endif
constexpr int kXtSegHi = LHPC_XT_SEGHI;
void xtile_segment_table(const XtileHost &o, std::vector<uint32_t> &seg, std::vector<int32_t> &hi);

// 0 on success; LHPC_ERR_UNSUPPORTED when the layout does not fit its
// index types (nnz + padding ≥ 2^31 or S > 4096).
// piece_nnz: target nonzeros per gather workgroup (a multiple of 8 is used).
// cut_window: see above, in (0, M] (M/2 cuts at any row start in the back half).
// splits: ascending rows in (0, n_rows) at which a chunk must start (row
// ranges that can be reduced separately, lhpc_spmv_range);
// LHPC_ERR_INVALID_ARG otherwise.  iperm selects the reduce's index stream
// (perm for false, iperm for true; only the selected one is built).
// unit > 1 (iperm only; 2 or 4): aligned segments — every (tile, chunk)
// segment is padded at its end to a multiple of `unit` entries, so each
// starts on a 16-B boundary of xg and the reduce loads it in 16-B units
// (padding entries: col16 0, never referenced by iperm); chunks are then cut
// so that their padded length, not their nonzero count, stays ≤ M.
int build_xtile(const void *row_ptr, int rp_bits, const int32_t *col, int64_t n_rows,
                int64_t n_cols, int64_t W, int M, int Rmax, int64_t piece_nnz, int slot_bytes,
                const int64_t *splits, int n_splits, bool iperm, int cut_window, XtileHost &out,
                int unit = 1);

// The phases of build_xtile, so that the O(nnz) passes can also run on the
// GPU from device-resident input (lhpc_xtile_device.hip) while everything that
// decides the layout stays this one host code:
//   xtile_plan_chunks      validation, chunk cuts (ce, cr), ranges, cont; needs
//                          col only for unit > 1; zeroes segoff
//   (counts)               segoff row c+1 = count of chunk c per tile
//   xtile_plan_offsets     tile bases (tbase, each a multiple of 8), total,
//                          segoff = segment starts
//   xtile_plan_scatter_host  col16 + perm / iperm from host col
//   xtile_plan_pieces      the gather workgroups from tbase
int xtile_plan_chunks(const void *rp, int bits, const int32_t *col, int64_t n_rows, int64_t n_cols, int64_t W,
                      int M, int Rmax, int slot_bytes, const int64_t *splits, int n_splits, bool iperm,
                      int cut_window, XtileHost &o, int unit);
int xtile_plan_offsets(XtileHost &o, std::vector<int64_t> &tbase);
void xtile_plan_scatter_host(const int32_t *col, int64_t nnz, XtileHost &o);
void xtile_plan_pieces(XtileHost &o, const std::vector<int64_t> &tbase, int64_t piece_nnz);

// Wave-transposed run layout of the XTILE reduce's per-position streams (val,
// iperm): chunk position i belongs to thread t = i / run (run = 64 B of
// values: fp32 16, fp64 8), element j = i % run.  Thread t sits in wave
// w = t / 64 at lane l = t % 64; the chunk's wave region w holds 64·run
// positions, and inside it the vw-element vector q of lane l (vw = 16 B /
// element size) is stored at (q·64 + l)·vw, so the wave's load instruction q
// reads 64 consecutive 16-B vectors.
inline int64_t xtile_wave_pos(int64_t i, int run, int vw) {
  const int64_t t = i / run, j = i % run, w = t / 64, l = t % 64, q = j / vw, r = j % vw;
  return w * 64 * run + (q * 64 + l) * vw + r;
}

// Per-chunk region bases (vbase[c]: chunk c's positions start there, each
// chunk padded to whole wave regions of 64·run positions; vbase[C] = total)
// and the val (tsz bytes each) and, when o.iperm is set, iperm streams in
// the wave-transposed layout; val padding is 0, iperm padding is M (the
// reduce keeps x = 0 in LDS slot M, so a padded position needs no mask).  Extra `tail` entries
// of zero padding follow vbase[C].  LHPC_ERR_UNSUPPORTED if vbase[C] ≥ 2^31.
int xtile_transpose_runs(const XtileHost &o, const void *val, size_t tsz, int run, int64_t tail,
                         std::vector<int32_t> &vbase, std::unique_ptr<unsigned char[]> &valt,
                         std::unique_ptr<uint16_t[]> &ipt);

// Wave-coalesced gather stores: inside each piece, every full block of 512
// stream entries (64 lanes × 8 entries, from the piece start) has its col16
// permuted so that lane l's 8 entries are stream positions
// (k / vw)·64·vw + vw·l + k % vw, k = 0..7 (vw = 16 B / value size): the
// gather's 16-B store h of every lane then covers one contiguous KB.  A
// partial last block keeps lane l's entries at 8·l .. 8·l + 7.
inline int xtile_gather_pos(int k, int l, int vw) { return (k / vw) * 64 * vw + vw * l + k % vw; }
void xtile_permute_gather_blocks(XtileHost &o, int vw);
// replace o.pieces by per-range pieces: range k's part of tile s is
// [⌈segoff[rchunk[k]][s]⌉₈, ⌈segoff[rchunk[k+1]][s]⌉₈) (the ≤ 7 entries of
// range k before its rounded start were written by range k − 1's gather: a
// gathered entry depends only on its position), cut into ≈ piece_nnz pieces;
// rpc[k] = first piece of range k.
void xtile_range_pieces(XtileHost &o, int64_t piece_nnz, std::vector<int64_t> &rpc);
// The same for an xg ring (round 6): sub-run (k, s) of [a, b) gets pieces
// over the whole groups [⌈a⌉₈, ⌊b⌋₈) and, when a (b) is not a multiple of 8,
// the group around it as a flagged prefix (suffix) of its first (last) piece
// — so each range gathers every entry it reads into its own ring, and no
// col16 group is permuted by two pieces.  Ring layout: sub-runs (k, s) in
// tile order, [⌊a⌋₈, ⌈b⌉₈) at an 8-aligned cursor; rdelta, pext, ring_len.
void xtile_ring_pieces(XtileHost &o, int64_t piece_nnz, std::vector<int64_t> &rpc);
// Phase-A tables of the iperm reduce (round 6, k_xtile_reduce PRE): per chunk
// c, base_ne[c·S + r] = start of its r-th non-empty segment (stream position,
// or ring position when o.rdelta is set) − that segment's flat offset (unused
// entries repeat the last one), and for each of its M/64 batches b of flat
// positions the rank terms bt[(c·M/64 + b)·4 …] = {w >> 1 (low, high word),
// starts before the batch − 1 + (w & 1), 0}, w = the batch's 64 start bits.
void xtile_phase_tables(const XtileHost &o, std::vector<uint32_t> &bt, std::vector<int32_t> &base_ne);

// LDS slot of chunk position i in the XTILE reduce (lhpc_spmv_xtile.hip
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
