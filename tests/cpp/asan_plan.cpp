// asan_plan.cpp — host-only driver for the plan-time and I/O code of
// liblhpc.so (lhpc_plan.cpp, lhpc_gen.cpp, lhpc_io.cpp compiled into this
// binary with -fsanitize=address,undefined; no HIP).  Mirrors the reference's
// policy of running every Linux test under ASan
// (/root/reference/tests/CMakeLists.txt:6-9) for the code a GPU box cannot
// sanitize: the CSR validation and the XSLICE / XTILE re-encodings that index
// host arrays by caller-supplied row_ptr / col_idx, and the file readers.
// Built and run by tests/test_asan.py (`make -C tests/cpp asan`).
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/lhpc.h"
#include "../../libhpc_amd/csrc/lhpc_plan.hpp"

static int failures = 0;
#define CHECK(c)                                                             \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++failures;                                                            \
    }                                                                        \
  } while (0)

namespace {

struct Csr {
  int64_t n = 0, m = 0;
  std::vector<int64_t> rp;
  std::vector<int32_t> col;
  std::vector<float> val;
};

Csr uniform(int64_t n, int64_t m, int per_row, uint64_t seed) {
  Csr a;
  a.n = n;
  a.m = m;
  a.rp.resize(static_cast<size_t>(n + 1));
  CHECK(lhpc_gen_uniform_row_ptr(n, per_row, a.rp.data()) == 0);
  a.col.resize(static_cast<size_t>(a.rp[n]));
  CHECK(lhpc_gen_fill_cols(n, m, a.rp.data(), seed, a.col.data()) == 0);
  a.val.resize(a.col.size());
  CHECK(lhpc_gen_fill_values(LHPC_F32, 0, static_cast<int64_t>(a.val.size()), seed + 1, a.val.data()) == 0);
  return a;
}

Csr powerlaw(int64_t n, int64_t m, int64_t lmax, uint64_t seed) {
  Csr a;
  a.n = n;
  a.m = m;
  a.rp.resize(static_cast<size_t>(n + 1));
  int64_t nnz = 0;
  CHECK(lhpc_gen_powerlaw_row_ptr(n, m, 1.792, 1, lmax, seed, a.rp.data(), &nnz) == 0);
  a.col.resize(static_cast<size_t>(nnz));
  CHECK(lhpc_gen_fill_cols(n, m, a.rp.data(), seed, a.col.data()) == 0);
  a.val.resize(a.col.size());
  CHECK(lhpc_gen_fill_values(LHPC_F32, 0, nnz, seed + 1, a.val.data()) == 0);
  return a;
}

// XTILE invariants: every CSR nonzero appears once in its chunk's segment
// concatenation, with the column it had; chunks tile the CSR order.
// unit > 1 (aligned segments): every segment starts and ends on a multiple
// of unit, the padded concatenation stays ≤ M, iperm skips the padding.
void check_xtile(const Csr &a, bool iperm, const std::vector<int64_t> &splits, int cut = 512, int unit = 1) {
  const int64_t W = 4096;
  const int M = 1024, Rmax = 128;
  lhpc::XtileHost xt;
  const int rc = lhpc::build_xtile(a.rp.data(), 64, a.col.data(), a.n, a.m, W, M, Rmax, 3000, 4,
                                   splits.empty() ? nullptr : splits.data(), static_cast<int>(splits.size()), iperm,
                                   cut, xt, unit);
  CHECK(rc == 0);
  if (rc) return;
  const int64_t C = xt.n_chunks, S = xt.S;
  CHECK(xt.ce.front() == 0 && xt.ce[static_cast<size_t>(C)] == a.rp[a.n]);
  for (int64_t c = 0; c < C; ++c) {
    const int64_t e0 = xt.ce[c], e1 = xt.ce[c + 1];
    CHECK(e1 >= e0 && e1 - e0 <= M);
    std::vector<int> seen(static_cast<size_t>(M), 0);
    int64_t flat = 0;
    for (int64_t s = 0; s < S; ++s) {
      const int64_t g0 = xt.segoff[c * S + s], g1 = xt.segoff[(c + 1) * S + s];
      CHECK(g0 <= g1 && g1 <= xt.total);
      CHECK(g0 % unit == 0 && (g1 - g0) % unit == 0);
      for (int64_t g = g0; g < g1; ++g, ++flat) {
        if (iperm) continue;
        (void)xt.perm[g];  // perm mode: every stream entry has a slot
      }
    }
    CHECK(unit == 1 ? flat == e1 - e0 : (flat >= e1 - e0 && flat <= M));
    if (iperm) {
      for (int64_t k = e0; k < e1; ++k) {
        const int f = xt.iperm[k];
        CHECK(f >= 0 && f < flat);
        if (f >= 0 && f < flat) ++seen[static_cast<size_t>(f)];
      }
      int64_t hits = 0;
      for (int v : seen) {
        CHECK(v <= 1);
        hits += v;
      }
      CHECK(hits == e1 - e0);
    }
  }
  // cache-sized ranges: range pieces cover the stream once, and every entry
  // of range k is gathered by range k's pieces or an earlier range's
  {
    std::vector<int64_t> rpc;
    lhpc::xtile_range_pieces(xt, 700, rpc);
    const int64_t K = static_cast<int64_t>(xt.rchunk.size()) - 1;
    CHECK(static_cast<int64_t>(rpc.size()) == K + 1 && static_cast<size_t>(rpc[K]) == xt.pieces.size() / 3);
    std::vector<int> by(static_cast<size_t>(xt.total), -1);
    for (int64_t k = 0; k < K; ++k)
      for (int64_t q = rpc[k]; q < rpc[k + 1]; ++q) {
        const int64_t g0 = xt.pieces[3 * q], g1 = xt.pieces[3 * q + 1], s = xt.pieces[3 * q + 2];
        CHECK(g0 % 8 == 0 && g0 < g1 && g1 <= xt.total && s >= 0 && s < S);
        for (int64_t g = g0; g < g1 && g < xt.total; ++g) {
          CHECK(by[static_cast<size_t>(g)] < 0);
          by[static_cast<size_t>(g)] = static_cast<int>(k);
        }
      }
    for (int64_t k = 0; k < K; ++k)
      for (int64_t s = 0; s < S; ++s)
        for (int64_t g = xt.segoff[xt.rchunk[k] * S + s]; g < xt.segoff[xt.rchunk[k + 1] * S + s]; ++g)
          CHECK(by[static_cast<size_t>(g)] >= 0 && by[static_cast<size_t>(g)] <= k);
  }
  // phase-A tables (xtile_phase_tables): position f of chunk c's segment
  // concatenation lies in non-empty segment rank = term + popcount(w1 &
  // lanes below f % 64) of its 64-position batch, and its xg entry is at
  // base_ne[rank] + f — the stream (or, after xtile_ring_pieces, the ring)
  // position of that entry
  auto check_phase_tables = [&]() {
    std::vector<uint32_t> bt;
    std::vector<int32_t> bne;
    lhpc::xtile_phase_tables(xt, bt, bne);
    const int64_t NBT = xt.M / 64, K = static_cast<int64_t>(xt.rchunk.size()) - 1;
    CHECK(static_cast<int64_t>(bt.size()) == std::max<int64_t>(C, 1) * NBT * 4);
    for (int64_t c = 0; c < C; ++c) {
      int64_t k = 0;
      while (k + 1 < K && xt.rchunk[k + 1] <= c) ++k;
      int64_t flat = 0;
      for (int64_t s = 0; s < S; ++s) {
        const int64_t a = xt.segoff[c * S + s], len = xt.segoff[(c + 1) * S + s] - a;
        const int64_t d = xt.rdelta.empty() ? 0 : xt.rdelta[static_cast<size_t>(k * S + s)];
        for (int64_t j = 0; j < len; ++j, ++flat) {
          const int64_t b = flat / 64, l = flat % 64;
          const uint32_t *t4 = bt.data() + (c * NBT + b) * 4;
          const uint64_t w1 = (static_cast<uint64_t>(t4[1]) << 32) | t4[0];
          const int64_t rank = static_cast<int32_t>(t4[2]) + __builtin_popcountll(w1 & ((uint64_t{1} << l) - 1));
          CHECK(rank >= 0 && rank < S);
          if (rank >= 0 && rank < S) CHECK(bne[static_cast<size_t>(c * S + rank)] + flat == a + j + d);
        }
      }
    }
  };
  if (iperm && unit == 1) check_phase_tables();
  // the xg ring (xtile_ring_pieces): per range, emulate the gather (every
  // piece writes stream entry g at ring position g + delta, plus its flagged
  // shared groups) on a ring wiped before the range, then the reduce's reads
  // through the segment table (hi row hrow[k] + ⌊(c − rchunk[k]) / 7⌋):
  // every segment must read back exactly its own stream entries
  if (iperm && unit == 1 && xt.rchunk.size() > 2) {
    std::vector<int64_t> rpc;
    lhpc::xtile_ring_pieces(xt, 700, rpc);
    std::vector<uint32_t> seg;
    std::vector<int32_t> hi;
    lhpc::xtile_segment_table(xt, seg, hi);
    const int64_t K = static_cast<int64_t>(xt.rchunk.size()) - 1, L = xt.ring_len;
    CHECK(L > 0 && L <= xt.total + 16 * S && static_cast<int64_t>(xt.hrow.size()) == K);
    CHECK(xt.pext.size() == xt.pieces.size() / 3 * 2);
    std::vector<int64_t> ring(static_cast<size_t>(L));
    for (int64_t k = 0; k < K; ++k) {
      std::fill(ring.begin(), ring.end(), -1);
      for (int64_t q = rpc[k]; q < rpc[k + 1]; ++q) {
        const int64_t g0 = xt.pieces[3 * q], g1 = xt.pieces[3 * q + 1], d = xt.pext[2 * q], fl = xt.pext[2 * q + 1];
        CHECK(g0 % 8 == 0 && g1 % 8 == 0 && g0 <= g1 && d % 8 == 0);
        auto put = [&](int64_t g) {
          CHECK(g >= 0 && g < xt.total && g + d >= 0 && g + d < L);
          if (g + d >= 0 && g + d < L) {
            CHECK(ring[static_cast<size_t>(g + d)] < 0);  // no two writers in one range
            ring[static_cast<size_t>(g + d)] = g;
          }
        };
        for (int64_t g = g0; g < g1; ++g) put(g);
        if (fl & 1)
          for (int64_t g = g0 - 8; g < g0; ++g) put(g);
        if (fl & 2)
          for (int64_t g = g1; g < g1 + 8; ++g) put(g);
      }
      for (int64_t c = xt.rchunk[k]; c < xt.rchunk[k + 1]; ++c)
        for (int64_t s = 0; s < S; ++s) {
          const uint32_t w = seg[static_cast<size_t>(c * S + s)];
          const int64_t h = xt.hrow[k] + (c - xt.rchunk[k]) / lhpc::kXtSegHi;
          const int64_t start = hi[static_cast<size_t>(h * S + s)] + static_cast<int64_t>(w & 0xFFFFu), len = w >> 16;
          CHECK(len == xt.segoff[(c + 1) * S + s] - xt.segoff[c * S + s]);
          for (int64_t j = 0; j < len; ++j)
            CHECK(start + j >= 0 && start + j < L && ring[static_cast<size_t>(start + j)] == xt.segoff[c * S + s] + j);
        }
    }
    check_phase_tables();  // with the ring deltas
  }
  // the transposed val/iperm streams and the gather-block permutation
  std::vector<int32_t> vbase;
  std::unique_ptr<unsigned char[]> valt;
  std::unique_ptr<uint16_t[]> ipt;
  CHECK(lhpc::xtile_transpose_runs(xt, a.val.data(), 4, 16, 64 * 16, vbase, valt, ipt) == 0);
  CHECK(static_cast<int64_t>(vbase.size()) == C + 1);
  lhpc::xtile_permute_gather_blocks(xt, 4);
}

void check_bad_csr() {
  // every builder pass indexes host arrays by col / row_ptr, so validation
  // must reject these before any of them runs (lhpc_spmv_plan_create)
  const int64_t rp[] = {0, 2, 3};
  const int32_t good[] = {0, 4, 2}, big[] = {0, 5, 2}, neg[] = {0, -1, 2};
  CHECK(lhpc::validate_csr(rp, 64, good, 2, 5, 3) == 0);
  CHECK(lhpc::validate_csr(rp, 64, big, 2, 5, 3) == LHPC_ERR_BAD_CSR);
  CHECK(lhpc::validate_csr(rp, 64, neg, 2, 5, 3) == LHPC_ERR_BAD_CSR);
  const int64_t down[] = {0, 3, 2};
  CHECK(lhpc::validate_csr(down, 64, good, 2, 5, 2) == LHPC_ERR_BAD_CSR);
  const int32_t rp32[] = {1, 2, 3};
  CHECK(lhpc::validate_csr(rp32, 32, good, 2, 5, 3) == LHPC_ERR_BAD_CSR);  // row_ptr[0] != 0
  CHECK(lhpc::validate_csr(rp, 64, good, 2, 5, 4) == LHPC_ERR_BAD_CSR);     // row_ptr[n] != nnz
}

void check_io(const Csr &a) {
  char tmpl[] = "/tmp/lhpc_asan_XXXXXX";
  const int fd = mkstemp(tmpl);
  CHECK(fd >= 0);
  close(fd);
  const int64_t nnz = a.rp[a.n];
  CHECK(lhpc_csr_save(tmpl, LHPC_F32, a.n, a.m, nnz, a.rp.data(), 64, a.col.data(), a.val.data()) == 0);
  int dt = -1, bits = 0;
  int64_t n = 0, m = 0, z = 0;
  CHECK(lhpc_csr_load_header(tmpl, &dt, &n, &m, &z, &bits) == 0);
  CHECK(dt == LHPC_F32 && n == a.n && m == a.m && z == nnz && bits == 64);
  std::vector<int64_t> rp(static_cast<size_t>(n + 1));
  std::vector<int32_t> col(static_cast<size_t>(z));
  std::vector<float> val(static_cast<size_t>(z));
  CHECK(lhpc_csr_load(tmpl, rp.data(), col.data(), val.data()) == 0);
  CHECK(rp == a.rp && col == a.col && val == a.val);
  // truncated file: the loader must refuse, not read past the mapping
  CHECK(truncate(tmpl, 100) == 0);
  CHECK(lhpc_csr_load_header(tmpl, &dt, &n, &m, &z, &bits) != 0 || lhpc_csr_load(tmpl, rp.data(), col.data(), val.data()) != 0);
  std::remove(tmpl);
  // Matrix Market: symmetric expansion, comments, a bad entry
  const std::string mtx = std::string(tmpl) + ".mtx";
  FILE *f = std::fopen(mtx.c_str(), "w");
  std::fprintf(f, "%%%%MatrixMarket matrix coordinate real symmetric\n%% c\n3 3 3\n1 1 2.0\n2 1 -1.5\n3 3 4e0\n");
  std::fclose(f);
  int64_t zmax = 0, cnt = 0;
  int sym = -1, fld = -1;
  CHECK(lhpc_mm_read_header(mtx.c_str(), &n, &m, &zmax, &sym, &fld) == 0 && zmax == 6);
  std::vector<int32_t> r(static_cast<size_t>(zmax)), c(static_cast<size_t>(zmax));
  std::vector<double> v(static_cast<size_t>(zmax));
  CHECK(lhpc_mm_read_coo(mtx.c_str(), r.data(), c.data(), v.data(), &cnt) == 0 && cnt == 4);
  f = std::fopen(mtx.c_str(), "w");
  std::fprintf(f, "%%%%MatrixMarket matrix coordinate real general\n3 3 2\n1 1 1.0\n4 1 1.0\n");
  std::fclose(f);
  CHECK(lhpc_mm_read_header(mtx.c_str(), &n, &m, &zmax, &sym, &fld) == 0);
  CHECK(lhpc_mm_read_coo(mtx.c_str(), r.data(), c.data(), v.data(), &cnt) != 0);  // row 4 of 3
  std::remove(mtx.c_str());
}

}  // namespace

int main() {
  check_bad_csr();
  const Csr u = uniform(20000, 30000, 15, 0x5EED0001);
  const Csr p = powerlaw(20000, 20000, 3000, 0x5EED0004);
  const Csr e = uniform(777, 100, 0, 7);  // all rows empty
  for (bool ip : {false, true}) {
    check_xtile(u, ip, {});
    check_xtile(p, ip, {});
    check_xtile(p, ip, {1, 5000, 19999});
    check_xtile(u, ip, {5000, 10000, 15000});
    check_xtile(p, ip, {}, 32);
    check_xtile(p, ip, {77}, 1024);
    check_xtile(e, ip, {});
  }
  for (int unit : {2, 4}) {  // aligned segments (iperm only)
    check_xtile(u, true, {}, 512, unit);
    check_xtile(p, true, {1, 5000, 19999}, 512, unit);
    check_xtile(p, true, {}, 32, unit);
    check_xtile(e, true, {}, 512, unit);
  }
  for (int S : {1, 8, 64}) {
    lhpc::XsliceHost xs;
    const int rc = lhpc::build_xslice(p.rp.data(), 64, p.col.data(), p.val.data(), 4, p.n, p.m, S, xs);
    CHECK(rc == 0 || rc == LHPC_ERR_UNSUPPORTED);
    if (rc == 0) CHECK(xs.nnz == p.rp[p.n]);
  }
  int64_t cuts[9];
  CHECK(lhpc_csr_partition_rows(p.rp.data(), 64, p.n, 8, cuts) == 0);
  for (int k = 0; k < 8; ++k) CHECK(cuts[k] <= cuts[k + 1]);
  check_io(u);
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::printf("ALL OK (asan plan/io)\n");
  return 0;
}
