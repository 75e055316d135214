// test_sparse_grid.cpp — the sparse-grid drop-in (include/sparse: RootGrid,
// HashBlock, PointerBlock, DenseBlock) used exactly like the reference
// benchmarks use lib/sparse (test_hpc_benchmark.cpp:859-925), and the
// RootGrid → CSR assembly.
//   test_sparse_grid grid  — no GPU: round trips, foreach coordinates on the
//                            reference's three layouts (incl. the SURVEY
//                            §2c-5 cells (-5,7), (1000,-2000)), PointerBlock
//                            wrap, concurrent OpenMP writes, copies
//   test_sparse_grid gpu   — sparse::to_csr (GPU COO→CSR) vs a std::map build,
//                            then SpMV on the assembled matrix; sparse::save_csr /
//                            load_csr / read_matrix_market (include/sparse/IO.hpp)
#include <sparse/IO.hpp>
#include <sparse/SparseDS.hpp>
#include <sparse/SpMV.hpp>
#include <unistd.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <stdexcept>
#include <utility>
#include <vector>

namespace {

int failures = 0;
#define CHECK(c)                                                         \
  do {                                                                   \
    if (!(c)) {                                                          \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

using Cell = std::pair<std::intptr_t, std::intptr_t>;

template <typename Grid, typename T>
void check_roundtrip(Grid &g, const std::map<Cell, T> &want) {
  for (const auto &[c, v] : want) {
    auto got = g.read(c.first, c.second);
    CHECK(got.has_value() && *got == v);
  }
  std::map<Cell, T> seen;
  g.foreach ([&](std::intptr_t x, std::intptr_t y, const T &v) {
    if (v != T{}) seen[{x, y}] = v;
  });
  CHECK(seen == want);
  if (seen != want) {
    for (const auto &[c, v] : seen)
      if (!want.count(c)) std::fprintf(stderr, "  foreach reported unexpected (%td,%td)\n", c.first, c.second);
  }
}

template <typename Grid>
void layout_case(const char *name, const std::vector<Cell> &cells) {
  Grid g;
  std::map<Cell, double> want;
  double v = 1.0;
  for (const auto &c : cells) {
    g.write(c.first, c.second, v);
    want[c] = v;
    v += 1.0;
  }
  check_roundtrip(g, want);
  CHECK(!g.read(123457, -98765).has_value() || *g.read(123457, -98765) == 0.0);
  // copies are deep
  Grid h = g;
  h.write(cells[0].first, cells[0].second, -1.0);
  CHECK(*g.read(cells[0].first, cells[0].second) == want[cells[0]]);
  std::printf("grid %s: %zu cells ok\n", name, cells.size());
}

int grid_tests() {
  using namespace sparse;
  // §2c-5 regression cells plus a spread of signs / magnitudes / tile edges
  const std::vector<Cell> cells = {{-5, 7},    {1000, -2000}, {0, 0},     {15, 15},   {16, 16},     {-1, -1},
                                   {-16, -17}, {17, -33},     {4095, 1},  {65536, 3}, {-70000, 12}, {3, 1 << 20}};
  layout_case<RootGrid<double, HashBlock<DenseBlock<16, double>>>>("hash/dense16", cells);
  layout_case<RootGrid<double, HashBlock<PointerBlock<64, DenseBlock<16, double>>>>>("hash/pointer64/dense16", cells);
  layout_case<RootGrid<double, HashBlock<PointerBlock<4, PointerBlock<8, DenseBlock<4, double>>>>>>(
      "hash/pointer4/pointer8/dense4", cells);
  // pointer root: covers [0, 2^(6+4)) per axis; in-range cells exact
  const std::vector<Cell> in_range = {{0, 0}, {5, 7}, {1023, 1023}, {16, 1000}, {511, 512}};
  layout_case<RootGrid<double, PointerBlock<64, DenseBlock<16, double>>>>("pointer64/dense16", in_range);
  layout_case<RootGrid<double, PointerBlock<8, PointerBlock<8, DenseBlock<16, double>>>>>("pointer8/pointer8/dense16",
                                                                                          in_range);
  {  // out-of-range coordinates wrap (reference PointerBlock.hpp:157-160) and alias their canonical cell
    RootGrid<double, PointerBlock<8, PointerBlock<8, DenseBlock<16, double>>>> g;  // span 2^10
    g.write(-5, 7, 3.0);
    CHECK(*g.read(-5, 7) == 3.0 && *g.read(1024 - 5, 7) == 3.0);
    std::vector<Cell> seen;
    g.foreach ([&](std::intptr_t x, std::intptr_t y, const double &v) {
      if (v != 0.0) seen.push_back({x, y});
    });
    CHECK(seen.size() == 1 && seen[0] == Cell(1019, 7));
  }
  {  // the reference benchmark's own trajectory and layouts (test_hpc_benchmark.cpp:859-925), written from
     // OpenMP threads; foreach must report each distinct cell once, at its coordinates
    constexpr long N = 200000;
    std::set<Cell> want;
    for (long t = 0; t < N; ++t)
      want.insert({static_cast<std::intptr_t>(std::floor(-100.f + 0.2f * t)),
                   static_cast<std::intptr_t>(std::floor(100.f + -0.6f * t))});
    auto run = [&](auto &grid, const char *name) {
#pragma omp parallel for
      for (long t = 0; t < N; ++t)
        grid.write(static_cast<std::intptr_t>(std::floor(-100.f + 0.2f * t)),
                   static_cast<std::intptr_t>(std::floor(100.f + -0.6f * t)), true);
      std::set<Cell> seen;
      grid.foreach ([&](std::intptr_t x, std::intptr_t y, const bool &v) {
        if (v) seen.insert({x, y});
      });
      CHECK(seen == want);
      std::printf("grid %s: benchmark trajectory %zu cells ok\n", name, seen.size());
    };
    auto hd = std::make_unique<RootGrid<bool, HashBlock<DenseBlock<16, bool>>>>();
    run(*hd, "BM_RootHashDense");
    auto hpd = std::make_unique<RootGrid<bool, HashBlock<PointerBlock<1 << 10, DenseBlock<16, bool>>>>>();
    run(*hpd, "BM_RootHashPointerDense");
  }
  {  // PointerBlock::WriteAccessor caches children, global coordinates
    PointerBlock<16, DenseBlock<8, int>> pb;
    auto acc = pb.access();
    DenseBlock<8, int> tile;
    tile.write(1, 2, 42);
    acc.write(70, 9, tile);  // slot (70>>3 & 15, 9>>3) = (8, 1)
    CHECK(pb.has(70, 9) && pb.has(64, 8) && !pb.has(0, 0));
    CHECK((*pb.read(71, 10)).get().read(1, 2)->get() == 42);
  }
  return failures;
}

int gpu_tests() {
  using namespace sparse;
  std::mt19937_64 rng(0xC5A);
  std::uniform_int_distribution<int> cx(-3000, 3000), cy(-500, 4000);
  std::uniform_real_distribution<double> uv(-1.0, 1.0);
  RootGrid<double, HashBlock<PointerBlock<32, DenseBlock<16, double>>>> g;
  std::map<Cell, double> want;
  for (int i = 0; i < 200000; ++i) {
    const Cell c{cx(rng), cy(rng)};
    const double v = uv(rng);
    g.write(c.first, c.second, v);  // later writes overwrite: the grid is a map
    want[c] = v;
  }
  const GridBounds b = bounds(g);
  CHECK(b.count == static_cast<std::int64_t>(want.size()));
  CHECK(b.row_min == want.begin()->first.first && b.row_max == want.rbegin()->first.first);
  auto A = to_csr<double, std::int32_t, std::int64_t>(g, b);
  A.validate();
  CHECK(A.n_rows == b.n_rows() && A.n_cols == b.n_cols() && A.nnz() == static_cast<std::int64_t>(want.size()));
  {  // CSR equals the std::map (row-major, column-ascending) order exactly
    std::size_t k = 0;
    bool same = true;
    for (const auto &[c, v] : want) {
      const std::int64_t r = c.first - b.row_min;
      same &= A.col_idx[k] == c.second - b.col_min && A.val[k] == v && A.row_ptr[r] <= static_cast<std::int64_t>(k) &&
              static_cast<std::int64_t>(k) < A.row_ptr[r + 1];
      ++k;
    }
    CHECK(same);
  }
  // window bigger than the bounding box, float values, int32 row_ptr
  auto F = to_csr<float>(g, b.row_min - 3, b.col_min - 2, b.n_rows() + 10, b.n_cols() + 5);
  F.validate();
  CHECK(F.nnz() == A.nnz() && F.row_ptr[3] == 0);
  // a kept cell outside the window throws
  bool threw = false;
  try {
    (void)to_csr<float>(g, b.row_min + 1, b.col_min, b.n_rows(), b.n_cols());
  } catch (const std::out_of_range &) {
    threw = true;
  }
  CHECK(threw);
  // empty grid → empty matrix
  RootGrid<double, HashBlock<DenseBlock<16, double>>> e;
  auto E = to_csr<double>(e, bounds(e));
  CHECK(E.n_rows == 0 && E.nnz() == 0);
  // SpMV on the assembled matrix vs a plain loop over the map
  SpMVPlan<double> plan(A);
  hpc::HPCHighDimensionFlatArray<1, double> x(A.n_cols), y(A.n_rows);
  for (std::int64_t j = 0; j < A.n_cols; ++j) x(j) = std::ldexp(static_cast<double>((j * 7) % 17) - 8.0, -3);
  spmv(plan, x, y);
  std::vector<double> ref(static_cast<std::size_t>(A.n_rows), 0.0);
  for (const auto &[c, v] : want) ref[c.first - b.row_min] += v * x(c.second - b.col_min);
  double err = 0.0, mag = 0.0;
  for (std::int64_t i = 0; i < A.n_rows; ++i) {
    err = std::max(err, std::fabs(y(i) - ref[static_cast<std::size_t>(i)]));
    mag = std::max(mag, std::fabs(ref[static_cast<std::size_t>(i)]));
  }
  CHECK(err <= 1e-12 * (1.0 + mag));
  std::printf("to_csr: %lld x %lld, nnz %lld ok; spmv max err %.3g\n", static_cast<long long>(A.n_rows),
              static_cast<long long>(A.n_cols), static_cast<long long>(A.nnz()), err);
  {  // file round trips
    char tmpl[] = "/tmp/lhpc_io_XXXXXX";
    const int fd = mkstemp(tmpl);
    CHECK(fd >= 0);
    close(fd);
    save_csr(tmpl, A);
    auto B = load_csr<double, std::int64_t>(tmpl);
    CHECK(B.n_rows == A.n_rows && B.n_cols == A.n_cols && B.row_ptr == A.row_ptr && B.col_idx == A.col_idx &&
          B.val == A.val);
    bool threw_type = false;
    try {
      (void)load_csr<float, std::int64_t>(tmpl);
    } catch (const std::invalid_argument &) {
      threw_type = true;
    }
    CHECK(threw_type);
    const std::string mtx = std::string(tmpl) + ".mtx";
    FILE *f = std::fopen(mtx.c_str(), "w");
    std::fprintf(f, "%%%%MatrixMarket matrix coordinate real symmetric\n%% comment\n3 3 3\n1 1 2.0\n2 1 -1.5\n3 3 4e0\n");
    std::fclose(f);
    auto M = read_matrix_market<double>(mtx);
    CHECK(M.n_rows == 3 && M.n_cols == 3 && M.nnz() == 4);
    if (!(M.n_rows == 3 && M.n_cols == 3 && M.nnz() == 4)) {
      std::fprintf(stderr, "mm: %lld x %lld nnz %lld rp", static_cast<long long>(M.n_rows),
                   static_cast<long long>(M.n_cols), static_cast<long long>(M.nnz()));
      for (auto v : M.row_ptr) std::fprintf(stderr, " %lld", static_cast<long long>(v));
      for (std::size_t i = 0; i < M.col_idx.size(); ++i)
        std::fprintf(stderr, " (%d %g)", static_cast<int>(M.col_idx[i]), static_cast<double>(M.val[i]));
      std::fprintf(stderr, "\n");
    }
    const std::int32_t rp_want[] = {0, 2, 3, 4};
    const std::int32_t col_want[] = {0, 1, 0, 2};
    const double val_want[] = {2.0, -1.5, -1.5, 4.0};
    for (int i = 0; i < 4; ++i) CHECK(M.row_ptr[i] == rp_want[i]);
    for (int i = 0; i < 4; ++i) CHECK(M.col_idx[i] == col_want[i] && M.val[i] == val_want[i]);
    std::remove(tmpl);
    std::remove(mtx.c_str());
    std::printf("io: lcsr round trip + matrix market ok\n");
  }
  return failures;
}

}  // namespace

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "grid";
  int rc = 0;
  try {
    if (!std::strcmp(mode, "grid")) rc = grid_tests();
    else if (!std::strcmp(mode, "gpu")) rc = gpu_tests();
    else {
      std::fprintf(stderr, "usage: %s grid|gpu\n", argv[0]);
      return 2;
    }
  } catch (const std::exception &e) {
    std::fprintf(stderr, "FAIL: exception %s\n", e.what());
    return 1;
  }
  if (rc) std::fprintf(stderr, "%d check(s) failed\n", rc);
  else std::printf("ALL OK (%s)\n", mode);
  return rc ? 1 : 0;
}
