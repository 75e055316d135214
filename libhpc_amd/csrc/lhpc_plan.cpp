// lhpc_plan.cpp — plan-time re-encoding of CSR into the XSLICE layout
// (see lhpc_plan.hpp).  Host only, OpenMP over 64-row chunks; the output is
// identical for any thread count.
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

int build_xslice(const void *rp, int bits, const int32_t *col, const void *val, size_t tsz,
                 int64_t n_rows, int64_t n_cols, int S, bool jagged, XsliceHost &o) {
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
  if (bad || (jagged && maxc > 255)) return LHPC_ERR_UNSUPPORTED;
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
  // pass 2: jagged-diagonal fill, one 64-row chunk per iteration (all slices)
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
        if (!jagged) {
          for (int r = 0; r < 64; ++r)
            for (int j = 0; j < l[r]; ++j)
              emit(order[static_cast<size_t>(start[static_cast<size_t>(r) * (S + 1) + s] + j)]);
          continue;
        }
        int maxl = 0;
        for (int r = 0; r < 64; ++r) maxl = std::max(maxl, static_cast<int>(l[r]));
        for (int j = 0; j < maxl; ++j)
          for (int r = 0; r < 64; ++r)
            if (l[r] > j) emit(order[static_cast<size_t>(start[static_cast<size_t>(r) * (S + 1) + s] + j)]);
      }
    }
  }
  return LHPC_OK;
}

}  // namespace lhpc
