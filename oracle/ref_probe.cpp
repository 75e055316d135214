// ref_probe.cpp — TEST INFRASTRUCTURE ONLY.  A driver compiled (by
// oracle/Makefile) against the reference's own, unmodified
// lib/hpc/include/HPCHighDimensionFlatArray.hpp + AlignedAlloc.hpp where they
// lie under /root/reference; output binary goes to oracle/_ref/ (git-ignored).
// It pins, with the reference container itself:
//   layout2/layout3  flat offsets of hpc::HPCHighDimensionFlatArray<D,float,g>
//                    (HPCHighDimensionFlatArray.hpp:161-187 via at(), :107-109)
//   blur x|y         the BM_x_blur / BM_y_blur loop semantics
//                    (tests/test_hpc_benchmark/test_hpc_benchmark.cpp:354-368,
//                    :444-457) evaluated through the reference operator()
//                    (:123-125) on a ghost-8 array, writing a.data() and
//                    b.data() so golden fixtures carry the reference bytes.
// Single translation unit on purpose: the reference header defines
// non-inline functions (AlignedAlloc.hpp:13,20).
#include <HPCHighDimensionFlatArray.hpp>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

namespace {
uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
float unit(uint64_t seed, uint64_t i) {  // U[-1,1), exact in fp32
  const uint64_t d = mix64(seed ^ mix64(i + 1) ^ 0x9E3779B97F4A7C15ull);
  return static_cast<float>(static_cast<double>(d >> 40) * 0x1.0p-23 - 1.0);
}

constexpr int kNblur = 8;  // test_hpc_benchmark.cpp:29

int blur(char dir, long ny, long nx, uint64_t seed, int zero_ghost, const char *prefix) {
  hpc::HPCHighDimensionFlatArray<2, float, kNblur> a(ny, nx);
  hpc::HPCHighDimensionFlatArray<2, float> b(ny, nx);
  for (long y = -kNblur; y < ny + kNblur; ++y)
    for (long x = -kNblur; x < nx + kNblur; ++x) {
      const bool ghost = y < 0 || x < 0 || y >= ny || x >= nx;
      const uint64_t id = static_cast<uint64_t>((y + kNblur) * (nx + 2 * kNblur) + (x + kNblur));
      a.at({y, x}) = (ghost && zero_ghost) ? 0.f : unit(seed, id);
    }
  for (long y = 0; y < ny; ++y)
    for (long x = 0; x < nx; ++x) {
      float res = {0.f};
      if (dir == 'x')
        for (int k = -kNblur; k <= kNblur; ++k) res += a(y, x + k);
      else
        for (int k = -kNblur; k <= kNblur; ++k) res += a(y + k, x);
      b(y, x) = res;
    }
  char path[4096];
  std::snprintf(path, sizeof path, "%s_a.f32", prefix);
  FILE *f = std::fopen(path, "wb");
  if (!f) return 2;
  std::fwrite(a.data(), sizeof(float), static_cast<size_t>((ny + 2 * kNblur) * (nx + 2 * kNblur)), f);
  std::fclose(f);
  std::snprintf(path, sizeof path, "%s_b.f32", prefix);
  f = std::fopen(path, "wb");
  if (!f) return 2;
  std::fwrite(b.data(), sizeof(float), static_cast<size_t>(ny * nx), f);
  std::fclose(f);
  return 0;
}

template <std::size_t G>
int layout2(long ny, long nx) {
  hpc::HPCHighDimensionFlatArray<2, float, G> a(ny, nx);
  const long g = static_cast<long>(G);
  const long pts[][2] = {{-g, -g}, {0, 0}, {0, 1}, {1, 0}, {ny - 1, nx - 1}, {ny + g - 1, nx + g - 1}};
  std::printf("{\"dims\":[%ld,%ld],\"ghost\":%ld,\"offsets\":[", ny, nx, g);
  for (size_t i = 0; i < sizeof pts / sizeof pts[0]; ++i)
    std::printf("%s[%ld,%ld,%td]", i ? "," : "", pts[i][0], pts[i][1],
                &a.at({pts[i][0], pts[i][1]}) - a.data());
  bool threw = false;
  try {
    a.at({ny + g, 0});
  } catch (const std::out_of_range &) {
    threw = true;
  }
  std::printf("],\"at_out_of_range_throws\":%s}\n", threw ? "true" : "false");
  return 0;
}

int layout3(long nz, long ny, long nx) {
  hpc::HPCHighDimensionFlatArray<3, float, 1> a(nz, ny, nx);
  const long pts[][3] = {{-1, -1, -1}, {0, 0, 0}, {0, 0, 1}, {0, 1, 0}, {1, 0, 0},
                         {nz - 1, ny - 1, nx - 1}, {nz, ny, nx}};
  std::printf("{\"dims\":[%ld,%ld,%ld],\"ghost\":1,\"offsets\":[", nz, ny, nx);
  for (size_t i = 0; i < sizeof pts / sizeof pts[0]; ++i)
    std::printf("%s[%ld,%ld,%ld,%td]", i ? "," : "", pts[i][0], pts[i][1], pts[i][2],
                &a.at({pts[i][0], pts[i][1], pts[i][2]}) - a.data());
  std::printf("]}\n");
  return 0;
}
}  // namespace

int main(int argc, char **argv) {
  if (argc >= 7 && !std::strcmp(argv[1], "blur"))
    return blur(argv[2][0], std::atol(argv[3]), std::atol(argv[4]), std::strtoull(argv[5], nullptr, 0),
                std::atoi(argv[6]), argc >= 8 ? argv[7] : "blur");
  if (argc == 5 && !std::strcmp(argv[1], "layout2")) {
    const long g = std::atol(argv[4]);
    if (g == 0) return layout2<0>(std::atol(argv[2]), std::atol(argv[3]));
    if (g == 1) return layout2<1>(std::atol(argv[2]), std::atol(argv[3]));
    if (g == 8) return layout2<8>(std::atol(argv[2]), std::atol(argv[3]));
    return 1;
  }
  if (argc == 5 && !std::strcmp(argv[1], "layout3"))
    return layout3(std::atol(argv[2]), std::atol(argv[3]), std::atol(argv[4]));
  std::fprintf(stderr,
               "usage: ref_probe blur <x|y> ny nx seed zero_ghost [prefix]\n"
               "       ref_probe layout2 ny nx ghost{0,1,8}\n"
               "       ref_probe layout3 nz ny nx\n");
  return 1;
}
