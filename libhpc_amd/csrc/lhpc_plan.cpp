// lhpc_plan.cpp — plan-time CSR validation and re-encodings of CSR into the
// XSLICE and XTILE layouts (see lhpc_plan.hpp).  Host only, OpenMP; every
// output is identical for any thread count.
#include "lhpc_plan.hpp"

#include <omp.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/lhpc.h"

namespace lhpc {
namespace {
inline int64_t rp_at(const void *rp, int bits, int64_t i) {
  return bits == 64 ? static_cast<const int64_t *>(rp)[i]
                    : static_cast<const int32_t *>(rp)[i];
}
}  // namespace

int validate_csr(const void *rp, int bits, const int32_t *col, int64_t n_rows, int64_t n_cols, int64_t nnz) {
  if (n_rows < 0 || nnz < 0 || rp_at(rp, bits, 0) != 0 || rp_at(rp, bits, n_rows) != nnz) return LHPC_ERR_BAD_CSR;
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t i = 0; i < n_rows; ++i) bad |= rp_at(rp, bits, i + 1) < rp_at(rp, bits, i) ? 1 : 0;
  if (bad) return LHPC_ERR_BAD_CSR;
  const uint32_t lim = static_cast<uint32_t>(n_cols);  // n_cols ≤ INT32_MAX; a negative col wraps above it
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (int64_t k = 0; k < nnz; ++k) bad |= static_cast<uint32_t>(col[k]) >= lim ? 1 : 0;
  return bad ? LHPC_ERR_BAD_CSR : LHPC_OK;
}

void csr_column_block(const void *rp, int bits, const int32_t *col, const void *val, size_t tsz, int64_t r0,
                      int64_t r1, int64_t c0, int64_t c1, std::vector<int64_t> &orp, std::vector<int32_t> &ocol,
                      std::vector<unsigned char> &oval) {
  const int64_t nr = r1 - r0;
  orp.assign(static_cast<size_t>(nr) + 1, 0);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < nr; ++r) {
    int64_t c = 0;
    for (int64_t k = rp_at(rp, bits, r0 + r); k < rp_at(rp, bits, r0 + r + 1); ++k) c += col[k] >= c0 && col[k] < c1;
    orp[static_cast<size_t>(r) + 1] = c;
  }
  for (int64_t r = 0; r < nr; ++r) orp[static_cast<size_t>(r) + 1] += orp[static_cast<size_t>(r)];
  const int64_t m = orp[static_cast<size_t>(nr)];
  ocol.resize(static_cast<size_t>(m));
  oval.resize(static_cast<size_t>(m) * tsz);
  const auto *vb = static_cast<const unsigned char *>(val);
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < nr; ++r) {
    int64_t o = orp[static_cast<size_t>(r)];
    for (int64_t k = rp_at(rp, bits, r0 + r); k < rp_at(rp, bits, r0 + r + 1); ++k)
      if (col[k] >= c0 && col[k] < c1) {
        ocol[static_cast<size_t>(o)] = static_cast<int32_t>(col[k] - c0);
        std::memcpy(oval.data() + static_cast<size_t>(o) * tsz, vb + static_cast<size_t>(k) * tsz, tsz);
        ++o;
      }
  }
}

int build_xslice(const void *rp, int bits, const int32_t *col, const void *val, size_t tsz,
                 int64_t n_rows, int64_t n_cols, int S, XsliceHost &o) {
  if (S < 1 || S > 256) return LHPC_ERR_INVALID_ARG;
  o.S = S;
  o.n_rows = n_rows;
  o.n_chunks = (n_rows + 63) / 64;
  o.n_rows_pad = o.n_chunks * 64;
  o.width = ((n_cols + S - 1) / S + 63) / 64 * 64;
  if (o.width == 0) o.width = 64;
  const int64_t nnz = rp_at(rp, bits, n_rows) - rp_at(rp, bits, 0);
  o.nnz = nnz;
  o.cbase.reset(new int64_t[static_cast<size_t>(S) * o.n_chunks + 1]);
  o.col.reset(new int32_t[nnz > 0 ? nnz : 1]);
  o.val.reset(new unsigned char[(nnz > 0 ? nnz : 1) * tsz]);
  const int64_t W = o.width;
  const size_t nl = static_cast<size_t>(S) * o.n_rows_pad;
  std::unique_ptr<uint16_t[]> l16(new uint16_t[nl]);
  int bad = 0, maxc = 0;
  // pass 1: in-slice lengths
#pragma omp parallel for schedule(static) reduction(| : bad) reduction(max : maxc)
  for (int64_t r = 0; r < o.n_rows_pad; ++r) {
    int cnt[256];
    std::memset(cnt, 0, sizeof(int) * static_cast<size_t>(S));
    if (r < n_rows) {
      for (int64_t k = rp_at(rp, bits, r); k < rp_at(rp, bits, r + 1); ++k) ++cnt[col[k] / W];
    }
    for (int s = 0; s < S; ++s) {
      if (cnt[s] > 65535) bad = 1;
      maxc = std::max(maxc, cnt[s]);
      l16[static_cast<size_t>(s) * o.n_rows_pad + r] = static_cast<uint16_t>(std::min(cnt[s], 65535));
    }
  }
  if (bad) return LHPC_ERR_UNSUPPORTED;
  o.lens_bytes = maxc > 255 ? 2 : 1;
  o.lens.reset(new uint8_t[nl * o.lens_bytes]);
  if (o.lens_bytes == 2) {
    std::memcpy(o.lens.get(), l16.get(), nl * 2);
  } else {
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < static_cast<int64_t>(nl); ++i) o.lens[i] = static_cast<uint8_t>(l16[i]);
  }
  // chunk sizes → offsets, slice-major
  std::vector<int64_t> csz(static_cast<size_t>(S) * o.n_chunks);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < S * o.n_chunks; ++i) {
    const uint16_t *l = l16.get() + (i / o.n_chunks) * o.n_rows_pad + (i % o.n_chunks) * 64;
    int64_t t = 0;
    for (int r = 0; r < 64; ++r) t += l[r];
    csz[static_cast<size_t>(i)] = t;
  }
  int64_t acc = 0;
  o.max_chunk = 0;
  for (int64_t i = 0; i < S * o.n_chunks; ++i) {
    o.cbase[i] = acc;
    acc += csz[static_cast<size_t>(i)];
    o.max_chunk = std::max(o.max_chunk, csz[static_cast<size_t>(i)]);
  }
  o.cbase[S * o.n_chunks] = acc;
  if (acc != nnz) return LHPC_ERR_INTERNAL;
  // pass 2: fill, one 64-row chunk per iteration (all slices)
#pragma omp parallel
  {
    std::vector<int64_t> order;   // element ids of the chunk, bucketed by (row, slice)
    std::vector<int64_t> start;   // [64][S+1] start of (row, slice) bucket in `order`
#pragma omp for schedule(dynamic, 64)
    for (int64_t c = 0; c < o.n_chunks; ++c) {
      const int64_t r0 = c * 64;
      const int64_t e0 = rp_at(rp, bits, std::min(r0, n_rows));
      const int64_t e1 = rp_at(rp, bits, std::min(r0 + 64, n_rows));
      order.assign(static_cast<size_t>(e1 - e0), 0);
      start.assign(static_cast<size_t>(64) * (S + 1), 0);
      for (int r = 0; r < 64 && r0 + r < n_rows; ++r) {
        const int64_t s0 = rp_at(rp, bits, r0 + r), s1 = rp_at(rp, bits, r0 + r + 1);
        int64_t *st = start.data() + static_cast<size_t>(r) * (S + 1);
        st[0] = s0 - e0;
        for (int s = 0; s < S; ++s) st[s + 1] = st[s] + l16[static_cast<size_t>(s) * o.n_rows_pad + r0 + r];
        int64_t fill[256];  // stable counting sort by slice
        for (int s = 0; s < S; ++s) fill[s] = st[s];
        for (int64_t k = s0; k < s1; ++k) order[static_cast<size_t>(fill[col[k] / W]++)] = k;
      }
      for (int s = 0; s < S; ++s) {
        int64_t pos = o.cbase[s * o.n_chunks + c];
        const uint16_t *l = l16.get() + static_cast<size_t>(s) * o.n_rows_pad + r0;
        auto emit = [&](int64_t e) {
          o.col[pos] = col[e];
          std::memcpy(o.val.get() + pos * tsz, static_cast<const unsigned char *>(val) + e * tsz, tsz);
          ++pos;
        };
        for (int r = 0; r < 64; ++r)
          for (int j = 0; j < l[r]; ++j)
            emit(order[static_cast<size_t>(start[static_cast<size_t>(r) * (S + 1) + s] + j)]);
      }
    }
  }
  return LHPC_OK;
}

int xtile_plan_chunks(const void *rp, int bits, const int32_t *col, int64_t n_rows, int64_t n_cols, int64_t W,
                      int M, int Rmax, int slot_bytes, const int64_t *splits, int n_splits, bool iperm,
                      int cut_window, XtileHost &o, int unit) {
  const int64_t nnz = rp_at(rp, bits, n_rows) - rp_at(rp, bits, 0);
  if (W < 8 || M < 64 || M >= 65536 || M % 16 || Rmax < 1 || (slot_bytes != 4 && slot_bytes != 8) ||
      cut_window < 1 || cut_window > M || (unit != 1 && unit != 2 && unit != 4) || (unit > 1 && !iperm))
    return LHPC_ERR_INVALID_ARG;
  const int64_t S = n_cols > 0 ? (n_cols + W - 1) / W : 1;
  if (S > 4096 || nnz + 8 * S >= INT32_MAX || n_rows >= INT32_MAX) return LHPC_ERR_UNSUPPORTED;
  o.S = static_cast<int>(S);
  o.W = W;
  o.M = M;
  o.Rmax = Rmax;
  o.unit = unit;
  const int64_t U = unit;
  auto RP = [&](int64_t i) { return rp_at(rp, bits, i); };
  // aligned segments: the longest window [e, e + len) whose padded length
  // Σ_s ⌈count_s / U⌉·U stays ≤ M (monotone in len, so any shorter cut fits)
  std::vector<int32_t> wcnt(unit > 1 ? static_cast<size_t>(S) : 0, 0);
  std::vector<int32_t> touched;
  auto window = [&](int64_t e) -> int64_t {
    if (U == 1) return M;
    int64_t k = e, padded = 0;
    for (; k < nnz; ++k) {
      const int64_t s = col[k] / W;
      const int64_t add = wcnt[static_cast<size_t>(s)] % U == 0 ? U : 0;
      if (padded + add > M) break;
      if (wcnt[static_cast<size_t>(s)] == 0) touched.push_back(static_cast<int32_t>(s));
      ++wcnt[static_cast<size_t>(s)];
      padded += add;
    }
    for (const int32_t s : touched) wcnt[static_cast<size_t>(s)] = 0;
    touched.clear();
    return k - e;
  };
  // first row r in [lo, n_rows] with rp[r] >= e
  auto lower_row = [&](int64_t lo, int64_t e) {
    int64_t hi = n_rows;
    while (lo < hi) {
      const int64_t mid = lo + (hi - lo) / 2;
      if (RP(mid) < e) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
  // ---- chunks: (ce, cr) pairs; invariant: cr[c] = first row with rp >= ce[c]
  //      (or a row whose predecessors starting at ce[c] are empty)
  o.ce.assign(1, 0);
  o.cr.assign(1, 0);
  for (int i = 0; i < n_splits; ++i)
    if (splits[i] <= 0 || splits[i] >= n_rows || (i > 0 && splits[i] <= splits[i - 1]))
      return LHPC_ERR_INVALID_ARG;
  {
    int64_t e = 0, r = 0;
    int si = 0;  // next split row after r
    while (!(e == nnz && r == n_rows)) {
      int64_t en, rb;
      const int64_t Mc = window(e);
      // a cut inside the window: row starts in its back cut_window entries
      // (scaled to the window when padding shortens it)
      const int64_t cw = U == 1 ? cut_window : std::max<int64_t>(1, cut_window * Mc / M);
      // a split row is done once a chunk starts at it (e == its start, r == it)
      while (si < n_splits && (RP(splits[si]) < e || (RP(splits[si]) == e && splits[si] <= r))) ++si;
      if (si < n_splits && RP(splits[si]) <= e + Mc) {
        en = RP(splits[si]);  // a range starts at this row: cut there
        rb = splits[si];
      } else if (e + Mc >= nnz) {
        en = nnz;
        rb = n_rows;
      } else {
        const int64_t target = e + Mc;
        // last row q with rp[q] <= target
        const int64_t q = lower_row(r, target + 1) - 1;
        if (q >= r && RP(q) > e + Mc - cw) {
          en = RP(q);  // cut at a row start
        } else {
          en = target;  // cut mid-row
        }
        rb = lower_row(r, en);
      }
      if (rb - r > Rmax) {
        rb = r + Rmax;
        en = RP(rb);
      }
      o.ce.push_back(static_cast<int32_t>(en));
      o.cr.push_back(static_cast<int32_t>(rb));
      e = en;
      r = rb;
    }
  }
  const int64_t C = static_cast<int64_t>(o.ce.size()) - 1;
  o.n_chunks = C;
  // range k = chunks [rchunk[k], rchunk[k+1]): the chunk owning split row k−1 first
  o.rchunk.assign(1, 0);
  for (int i = 0; i < n_splits; ++i) {
    // chunks inside a long row just before the split also have cr == split
    // (they own no row); the range starts at the one beginning at the split row
    int64_t c = std::lower_bound(o.cr.begin(), o.cr.end(), static_cast<int32_t>(splits[i])) - o.cr.begin();
    while (c < C && !(o.cr[c] == splits[i] && o.ce[c] == RP(splits[i]))) ++c;
    if (c >= C) return LHPC_ERR_INTERNAL;
    o.rchunk.push_back(c);
  }
  o.rchunk.push_back(C);
  if (M > 65535 / (kXtSegHi - 1)) return LHPC_ERR_UNSUPPORTED;  // seg lo fits 16 bits
  o.cont.clear();
  for (int64_t c = 0; c < C; ++c) {
    const int64_t r0 = o.cr[c], r1 = o.cr[c + 1];
    if (r1 > r0 && RP(r1) > o.ce[c + 1]) o.cont.push_back(static_cast<int32_t>(c));
  }
  o.iperm_mode = iperm;
  o.slot_bytes = slot_bytes;
  o.segoff.assign(static_cast<size_t>((C + 1) * S), 0);
  return LHPC_OK;
}

int xtile_plan_offsets(XtileHost &o, std::vector<int64_t> &tbase) {
  const int64_t S = o.S, C = o.n_chunks, U = o.unit;
  auto pad = [U](int64_t len) { return (len + U - 1) / U * U; };
  int32_t *cnt = o.segoff.data() + S;  // row c+1 holds count[c] on entry
  if (U > 1)  // aligned segments: padding at each segment's end
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < C; ++c)
      for (int64_t s = 0; s < S; ++s) cnt[c * S + s] = static_cast<int32_t>(pad(cnt[c * S + s]));
  tbase.assign(static_cast<size_t>(S) + 1, 0);
  {
    std::vector<int64_t> tot(static_cast<size_t>(S), 0);
#pragma omp parallel for schedule(static)
    for (int64_t s = 0; s < S; ++s) {
      int64_t t = 0;
      for (int64_t c = 0; c < C; ++c) t += cnt[c * S + s];
      tot[static_cast<size_t>(s)] = t;
    }
    for (int64_t s = 0; s < S; ++s) tbase[s + 1] = tbase[s] + (tot[s] + 7) / 8 * 8;
  }
  if (tbase[S] >= INT32_MAX) return LHPC_ERR_UNSUPPORTED;  // segment padding pushed the stream past int32
  o.total = tbase[S];
  // exclusive prefix down each tile column: segoff[c][s] = tbase[s] + Σ_{c'<c} count[c'][s]
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < S; ++s) {
    int64_t acc = tbase[s];
    for (int64_t c = 0; c <= C; ++c) {
      const int64_t n = c < C ? o.segoff[(c + 1) * S + s] : 0;
      o.segoff[c * S + s] = static_cast<int32_t>(acc);
      acc += n;
    }
  }
  return LHPC_OK;
}

void xtile_plan_scatter_host(const int32_t *col, int64_t nnz, XtileHost &o) {
  const int64_t S = o.S, C = o.n_chunks, W = o.W;
  const bool iperm = o.iperm_mode;
  const int slot_bytes = o.slot_bytes;
  // ---- scatter (stable: CSR order inside each segment)
  o.col16.reset(new uint16_t[o.total > 0 ? o.total : 1]());
  if (iperm)
    o.iperm.reset(new uint16_t[nnz > 0 ? nnz : 1]());
  else
    o.perm.reset(new uint16_t[o.total > 0 ? o.total : 1]());
#pragma omp parallel
  {
    std::vector<int32_t> cur(static_cast<size_t>(S)), flat(iperm ? static_cast<size_t>(S) : 0);
#pragma omp for schedule(dynamic, 64)
    for (int64_t c = 0; c < C; ++c) {
      std::memcpy(cur.data(), o.segoff.data() + c * S, sizeof(int32_t) * static_cast<size_t>(S));
      if (iperm) {  // flat offset of each tile's segment in the chunk's concatenation
        int32_t f = 0;
        for (int64_t s = 0; s < S; ++s) {
          flat[static_cast<size_t>(s)] = f;
          f += o.segoff[(c + 1) * S + s] - o.segoff[c * S + s];
        }
      }
      const int64_t e0 = o.ce[c];
      for (int64_t k = e0; k < o.ce[c + 1]; ++k) {
        const int64_t s = col[k] / W;
        const int32_t g = cur[static_cast<size_t>(s)]++;
        o.col16[g] = static_cast<uint16_t>(col[k] - s * W);
        if (iperm)
          o.iperm[k] = static_cast<uint16_t>(flat[static_cast<size_t>(s)] + (g - o.segoff[c * S + s]));
        else
          o.perm[g] = static_cast<uint16_t>(xtile_slot(static_cast<int>(k - e0), slot_bytes));
      }
    }
  }
}

void xtile_plan_pieces(XtileHost &o, const std::vector<int64_t> &tbase, int64_t piece_nnz) {
  const int64_t S = o.S;
  // ---- gather workgroups: each non-empty tile split into pieces of ≈ piece_nnz.
  //      Order: tiles in runs of 8, and inside a run piece k of the 8 tiles
  //      before piece k + 1, so the pieces of one tile are 8 workgroups
  //      apart — the same XCD under round-robin dispatch — and the x tile
  //      the second one loads is an L2 hit.  (Placement only; any order is
  //      correct.)
  o.pieces.clear();
  const int64_t pn = std::max<int64_t>(8, (piece_nnz + 7) / 8 * 8);
  for (int64_t s0 = 0; s0 < S; s0 += 8) {
    std::vector<int64_t> step(8, 0), np(8, 0);
    int64_t kmax = 0;
    for (int64_t s = s0; s < std::min<int64_t>(S, s0 + 8); ++s) {
      const int64_t len = tbase[s + 1] - tbase[s];
      if (len == 0) continue;
      const int64_t P = (len + pn - 1) / pn;
      step[s - s0] = ((len + P - 1) / P + 7) / 8 * 8;
      np[s - s0] = (len + step[s - s0] - 1) / step[s - s0];
      kmax = std::max(kmax, np[s - s0]);
    }
    for (int64_t k = 0; k < kmax; ++k)
      for (int64_t s = s0; s < std::min<int64_t>(S, s0 + 8); ++s) {
        if (k >= np[s - s0]) continue;
        const int64_t g = tbase[s] + k * step[s - s0];
        o.pieces.push_back(static_cast<int32_t>(g));
        o.pieces.push_back(static_cast<int32_t>(std::min(g + step[s - s0], tbase[s + 1])));
        o.pieces.push_back(static_cast<int32_t>(s));
      }
  }
}

int build_xtile(const void *rp, int bits, const int32_t *col, int64_t n_rows, int64_t n_cols,
                int64_t W, int M, int Rmax, int64_t piece_nnz, int slot_bytes,
                const int64_t *splits, int n_splits, bool iperm, int cut_window, XtileHost &o, int unit) {
  int st = xtile_plan_chunks(rp, bits, col, n_rows, n_cols, W, M, Rmax, slot_bytes, splits, n_splits, iperm,
                             cut_window, o, unit);
  if (st != LHPC_OK) return st;
  const int64_t S = o.S, C = o.n_chunks;
  // ---- per (chunk, tile) counts → segment offsets in (tile, chunk) order
  int32_t *cnt = o.segoff.data() + S;  // row c+1 temporarily holds count[c]
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t c = 0; c < C; ++c) {
    int32_t *cc = cnt + c * S;
    for (int64_t k = o.ce[c]; k < o.ce[c + 1]; ++k) ++cc[col[k] / W];
  }
  std::vector<int64_t> tbase;
  if ((st = xtile_plan_offsets(o, tbase)) != LHPC_OK) return st;
  xtile_plan_scatter_host(col, rp_at(rp, bits, n_rows) - rp_at(rp, bits, 0), o);
  xtile_plan_pieces(o, tbase, piece_nnz);
  return LHPC_OK;
}

int xtile_transpose_runs(const XtileHost &o, const void *val, size_t tsz, int run, int64_t tail,
                         std::vector<int32_t> &vbase, std::unique_ptr<unsigned char[]> &valt,
                         std::unique_ptr<uint16_t[]> &ipt) {
  const int64_t C = o.n_chunks, reg = 64 * static_cast<int64_t>(run);
  std::vector<int64_t> vb(static_cast<size_t>(C) + 1, 0);
  for (int64_t c = 0; c < C; ++c) vb[c + 1] = vb[c] + (o.ce[c + 1] - o.ce[c] + reg - 1) / reg * reg;
  if (vb[C] + tail >= INT32_MAX) return LHPC_ERR_UNSUPPORTED;
  vbase.assign(vb.begin(), vb.end());
  const size_t total = static_cast<size_t>(vb[C] + tail);
  valt.reset(new unsigned char[total * tsz]());
  if (o.iperm) {  // padding points at the reduce's zero slot M (x = 0 there)
    ipt.reset(new uint16_t[total]);
    std::fill(ipt.get(), ipt.get() + total, static_cast<uint16_t>(o.M));
  }
  const int vw = static_cast<int>(16 / tsz);
  const unsigned char *vs = static_cast<const unsigned char *>(val);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t c = 0; c < C; ++c) {
    const int64_t e0 = o.ce[c], m = o.ce[c + 1] - e0;
    for (int64_t i = 0; i < m; ++i) {
      std::memcpy(valt.get() + (vb[c] + xtile_wave_pos(i, run, vw)) * tsz, vs + (e0 + i) * tsz, tsz);
      if (o.iperm) ipt[static_cast<size_t>(vb[c] + xtile_wave_pos(i, run, 8))] = o.iperm[static_cast<size_t>(e0 + i)];
    }
  }
  return LHPC_OK;
}

void xtile_segment_table(const XtileHost &o, std::vector<uint32_t> &seg, std::vector<int32_t> &hi) {
  const int64_t S = o.S, C = o.n_chunks;
  if (o.rdelta.empty()) {
    const int64_t H = (C + kXtSegHi - 1) / kXtSegHi;
    seg.assign(static_cast<size_t>(std::max<int64_t>(C, 1) * S), 0u);
    hi.assign(static_cast<size_t>(std::max<int64_t>(H, 1) * S), 0);
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < C; ++c) {
      const int32_t *a = o.segoff.data() + c * S, *b = a + S, *h = o.segoff.data() + (c / kXtSegHi) * kXtSegHi * S;
      if (c % kXtSegHi == 0) std::memcpy(hi.data() + (c / kXtSegHi) * S, a, sizeof(int32_t) * static_cast<size_t>(S));
      for (int64_t s = 0; s < S; ++s)
        seg[static_cast<size_t>(c * S + s)] =
            static_cast<uint32_t>(a[s] - h[s]) | (static_cast<uint32_t>(b[s] - a[s]) << 16);
    }
    return;
  }
  // ring plans: starts in ring positions (stream position + rdelta of the
  // chunk's range), hi groups of kXtSegHi chunks restarting at every range
  // (a group straddling two ranges would mix two rings' positions)
  const int64_t K = static_cast<int64_t>(o.rchunk.size()) - 1;
  std::vector<int64_t> g0;  // first chunk of each hi group, then C (group g of range k: row hrow[k] + …)
  std::vector<int32_t> gk;  // its range
  for (int64_t k = 0; k < K; ++k) {
    for (int64_t c = o.rchunk[k]; c < o.rchunk[k + 1]; c += kXtSegHi) {
      g0.push_back(c);
      gk.push_back(static_cast<int32_t>(k));
    }
  }
  g0.push_back(C);
  const int64_t H = static_cast<int64_t>(g0.size()) - 1;
  seg.assign(static_cast<size_t>(std::max<int64_t>(C, 1) * S), 0u);
  hi.assign(static_cast<size_t>(std::max<int64_t>(H, 1) * S), 0);
#pragma omp parallel for schedule(static)
  for (int64_t g = 0; g < H; ++g) {
    const int32_t *d = o.rdelta.data() + static_cast<int64_t>(gk[g]) * S;
    const int32_t *h = o.segoff.data() + g0[g] * S;
    for (int64_t s = 0; s < S; ++s) hi[static_cast<size_t>(g * S + s)] = h[s] + d[s];
    const int64_t c1 = std::min(g0[g] + kXtSegHi, o.rchunk[gk[g] + 1]);
    for (int64_t c = g0[g]; c < c1; ++c) {
      const int32_t *a = o.segoff.data() + c * S, *b = a + S;
      for (int64_t s = 0; s < S; ++s)
        seg[static_cast<size_t>(c * S + s)] =
            static_cast<uint32_t>(a[s] - h[s]) | (static_cast<uint32_t>(b[s] - a[s]) << 16);
    }
  }
}

void xtile_phase_tables(const XtileHost &o, std::vector<uint32_t> &bt, std::vector<int32_t> &base_ne) {
  const int64_t S = o.S, C = o.n_chunks, M = o.M, NBT = M / 64;
  bt.assign(static_cast<size_t>(std::max<int64_t>(C, 1) * NBT * 4), 0u);
  base_ne.assign(static_cast<size_t>(std::max<int64_t>(C, 1) * S), 0);
  const int64_t K = static_cast<int64_t>(o.rchunk.size()) - 1;
#pragma omp parallel
  {
    std::vector<uint64_t> starts(static_cast<size_t>(NBT));
#pragma omp for schedule(dynamic, 64)
    for (int64_t c = 0; c < C; ++c) {
      int64_t k = 0;  // c's range (for the ring deltas)
      if (!o.rdelta.empty())
        while (k + 1 < K && o.rchunk[k + 1] <= c) ++k;
      std::fill(starts.begin(), starts.end(), uint64_t{0});
      int32_t *bn = base_ne.data() + c * S;
      int64_t flat = 0, nne = 0;
      for (int64_t s = 0; s < S; ++s) {
        const int64_t a = o.segoff[c * S + s], len = o.segoff[(c + 1) * S + s] - a;
        if (len <= 0) continue;
        const int64_t start = a + (o.rdelta.empty() ? 0 : o.rdelta[static_cast<size_t>(k * S + s)]);
        bn[nne++] = static_cast<int32_t>(start - flat);
        starts[static_cast<size_t>(flat / 64)] |= uint64_t{1} << (flat % 64);
        flat += len;
      }
      for (int64_t r = nne; r < S; ++r) bn[r] = nne > 0 ? bn[nne - 1] : 0;
      int64_t before = 0;
      uint32_t *b4 = bt.data() + c * NBT * 4;
      for (int64_t b = 0; b < NBT; ++b) {
        const uint64_t w = starts[static_cast<size_t>(b)], w1 = w >> 1;
        b4[4 * b] = static_cast<uint32_t>(w1);
        b4[4 * b + 1] = static_cast<uint32_t>(w1 >> 32);
        b4[4 * b + 2] = static_cast<uint32_t>(before - 1 + static_cast<int64_t>(w & 1u));
        before += __builtin_popcountll(w);
      }
    }
  }
}

void xtile_ring_pieces(XtileHost &o, int64_t piece_nnz, std::vector<int64_t> &rpc) {
  const int64_t S = o.S, K = static_cast<int64_t>(o.rchunk.size()) - 1;
  const int64_t pn = std::max<int64_t>(8, (piece_nnz + 7) / 8 * 8);
  auto up8 = [](int64_t v) { return (v + 7) / 8 * 8; };
  auto dn8 = [](int64_t v) { return v / 8 * 8; };
  o.pieces.clear();
  o.pext.clear();
  o.rdelta.assign(static_cast<size_t>(K * S), 0);
  o.ring_len = 0;
  o.hrow.assign(1, 0);  // hi groups of kXtSegHi chunks per range (xtile_segment_table)
  for (int64_t k = 0; k + 1 < K; ++k)
    o.hrow.push_back(o.hrow.back() + (o.rchunk[k + 1] - o.rchunk[k] + kXtSegHi - 1) / kXtSegHi);
  rpc.assign(1, 0);
  for (int64_t k = 0; k < K; ++k) {
    int64_t cur = 0;  // ring cursor (a multiple of 8)
    for (int64_t s = 0; s < S; ++s) {
      const int64_t a = o.segoff[o.rchunk[k] * S + s], b = o.segoff[o.rchunk[k + 1] * S + s];
      if (b <= a) continue;
      const int64_t d = cur - dn8(a);  // ring position of stream position g: g + d
      o.rdelta[static_cast<size_t>(k * S + s)] = static_cast<int32_t>(d);
      cur += up8(b) - dn8(a);
      // whole groups [ia, ib) in ≈ piece_nnz pieces; the partial groups at a
      // and b ride on the first / last piece as flagged extra groups
      const int64_t ia = up8(a), ib = dn8(b);
      const bool pre = a % 8 != 0, suf = b % 8 != 0 && ib >= ia;
      if (ib <= ia) {  // no whole group: one piece holding the group(s) around a (and b)
        o.pieces.insert(o.pieces.end(), {static_cast<int32_t>(ia), static_cast<int32_t>(ia), static_cast<int32_t>(s)});
        o.pext.insert(o.pext.end(), {static_cast<int32_t>(d), (pre ? 1 : 0) | (suf ? 2 : 0)});
        continue;
      }
      const int64_t P = (ib - ia + pn - 1) / pn, step = up8((ib - ia + P - 1) / P);
      for (int64_t g = ia; g < ib; g += step) {
        const int64_t e = std::min(ib, g + step);
        o.pieces.insert(o.pieces.end(), {static_cast<int32_t>(g), static_cast<int32_t>(e), static_cast<int32_t>(s)});
        o.pext.insert(o.pext.end(), {static_cast<int32_t>(d), (g == ia && pre ? 1 : 0) | (e == ib && suf ? 2 : 0)});
      }
    }
    o.ring_len = std::max(o.ring_len, cur);
    rpc.push_back(static_cast<int64_t>(o.pieces.size() / 3));
  }
}

void xtile_range_pieces(XtileHost &o, int64_t piece_nnz, std::vector<int64_t> &rpc) {
  const int64_t S = o.S, K = static_cast<int64_t>(o.rchunk.size()) - 1;
  const int64_t pn = std::max<int64_t>(8, (piece_nnz + 7) / 8 * 8);
  auto up8 = [](int64_t v) { return (v + 7) / 8 * 8; };
  o.pieces.clear();
  rpc.assign(1, 0);
  for (int64_t k = 0; k < K; ++k) {
    for (int64_t s = 0; s < S; ++s) {
      const int64_t a = up8(o.segoff[o.rchunk[k] * S + s]), b = up8(o.segoff[o.rchunk[k + 1] * S + s]);
      if (b <= a) continue;
      const int64_t P = (b - a + pn - 1) / pn, step = up8((b - a + P - 1) / P);
      for (int64_t g = a; g < b; g += step) {
        o.pieces.push_back(static_cast<int32_t>(g));
        o.pieces.push_back(static_cast<int32_t>(std::min(b, g + step)));
        o.pieces.push_back(static_cast<int32_t>(s));
      }
    }
    rpc.push_back(static_cast<int64_t>(o.pieces.size() / 3));
  }
}

void xtile_permute_gather_blocks(XtileHost &o, int vw) {
  const int64_t np = static_cast<int64_t>(o.pieces.size() / 3);
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t b = 0; b < np; ++b) {
    const int64_t g0 = o.pieces[3 * b], g1 = o.pieces[3 * b + 1];
    uint16_t tmp[512];
    for (int64_t g = g0; g + 512 <= g1; g += 512) {
      uint16_t *c = o.col16.get() + g;
      for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 8; ++k) tmp[8 * l + k] = c[xtile_gather_pos(k, l, vw)];
      std::memcpy(c, tmp, sizeof(tmp));
    }
  }
}

}  // namespace lhpc
