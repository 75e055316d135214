// test_cpp_api.cpp — exercises the C++ drop-in surface exactly as a reference
// user would: hpc::HPCHighDimensionFlatArray / hpc::AlignedAllocator (same
// names and layout as lib/hpc/include), sparse::CSRMatrix + sparse::spmv, and
// hpc::blur_x / blur_y / stencil7, all forwarding to liblhpc.so.
//   test_cpp_api layout   — no GPU: layout offsets (JSON) + at() bounds
//   test_cpp_api gpu      — SpMV / blur / stencil7 on the device vs plain loops
// Linked with second_tu.cpp, which includes the same headers: the reference's
// AlignedAlloc.hpp fails to link this way; ours must not.
#include <HPCHighDimensionFlatArray.hpp>
#include <Stencil.hpp>
#include <sparse/DeviceCSR.hpp>
#include <sparse/Dist.hpp>
#include <sparse/SparseDS.hpp>
#include <sparse/SpMV.hpp>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <system_error>
#include <vector>

int second_tu_sum(int n);  // second_tu.cpp

namespace {

int fail(const char *what) {
  std::fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

template <std::size_t G>
void print_layout2(long ny, long nx, bool first) {
  hpc::HPCHighDimensionFlatArray<2, float, G> a(ny, nx);
  const long g = static_cast<long>(G);
  const long pts[][2] = {{-g, -g}, {0, 0}, {0, 1}, {1, 0}, {ny - 1, nx - 1}, {ny + g - 1, nx + g - 1}};
  std::printf("%s{\"dims\":[%ld,%ld],\"ghost\":%ld,\"offsets\":[", first ? "" : ",", ny, nx, g);
  for (size_t i = 0; i < 6; ++i)
    std::printf("%s[%ld,%ld,%td]", i ? "," : "", pts[i][0], pts[i][1], &a.at({pts[i][0], pts[i][1]}) - a.data());
  bool threw = false;
  try {
    a.at({ny + g, 0});
  } catch (const std::out_of_range &) {
    threw = true;
  }
  std::printf("],\"at_out_of_range_throws\":%s}", threw ? "true" : "false");
}

void print_layout3(long nz, long ny, long nx) {
  hpc::HPCHighDimensionFlatArray<3, float, 1> a(nz, ny, nx);
  const long pts[][3] = {{-1, -1, -1}, {0, 0, 0}, {0, 0, 1}, {0, 1, 0}, {1, 0, 0}, {nz - 1, ny - 1, nx - 1}, {nz, ny, nx}};
  std::printf(",{\"dims\":[%ld,%ld,%ld],\"ghost\":1,\"offsets\":[", nz, ny, nx);
  for (size_t i = 0; i < 7; ++i)
    std::printf("%s[%ld,%ld,%ld,%td]", i ? "," : "", pts[i][0], pts[i][1], pts[i][2],
                &a.at({pts[i][0], pts[i][1], pts[i][2]}) - a.data());
  std::printf("]}");
}

int layout_mode() {
  std::printf("[");
  print_layout2<8>(5, 7, true);
  print_layout2<0>(3, 4, false);
  print_layout2<1>(9, 2, false);
  print_layout3(4, 5, 6);
  print_layout3(1, 1, 1);
  std::printf("]\n");
  // zero-initialised, aligned, usable from a second TU
  hpc::HPCHighDimensionFlatArray<2, double, 2, 2, 64> z(3, 3);
  for (std::size_t i = 0; i < z.size(); ++i)
    if (z.data()[i] != 0.0) return fail("not zero-initialised");
  if (reinterpret_cast<std::uintptr_t>(z.data()) % 64) return fail("alignment");
  if (second_tu_sum(10) != 45) return fail("second TU");
  return 0;
}

float dyadic(unsigned i) { return static_cast<float>(static_cast<int>((i * 2654435761u) >> 28) % 17 - 8) * 0.125f; }

int gpu_mode() {
  // ---- SpMV through sparse::SpMVPlan / sparse::spmv with flat-array vectors
  const std::int64_t n = 5000, m = 4001;
  sparse::CSRMatrix<float> A(n, m);
  for (std::int64_t i = 0; i < n; ++i) {
    const int len = static_cast<int>(i % 23);
    for (int j = 0; j < len; ++j) {
      A.col_idx.push_back(static_cast<std::int32_t>((i * 37 + j * 151) % m));
      A.val.push_back(dyadic(static_cast<unsigned>(i * 31 + j)));
    }
    std::sort(A.col_idx.end() - len, A.col_idx.end());
    // distinct columns: (i*37 + j*151) % m is injective in j for len < 23
    A.row_ptr[static_cast<std::size_t>(i + 1)] = static_cast<std::int32_t>(A.col_idx.size());
  }
  A.validate();
  hpc::HPCHighDimensionFlatArray<1, float> x(m), y(n);
  for (std::int64_t c = 0; c < m; ++c) x(c) = dyadic(static_cast<unsigned>(c + 7));
  sparse::SpMVPlan<float> plan(A);
  sparse::spmv(plan, x, y);
  for (std::int64_t i = 0; i < n; ++i) {
    double s = 0;
    for (auto k = A.row_ptr[i]; k < A.row_ptr[i + 1]; ++k) s += double(A.val[k]) * double(x(A.col_idx[k]));
    if (static_cast<float>(s) != y(i)) return fail("spmv mismatch (dyadic inputs must be exact)");
  }
  // wrong-size vector → std::system_error in the lhpc category
  try {
    hpc::HPCHighDimensionFlatArray<1, float> shortx(10);
    sparse::spmv(plan, shortx, y);
    return fail("expected std::system_error");
  } catch (const std::system_error &e) {
    if (std::strcmp(e.code().category().name(), "lhpc") != 0) return fail("error category");
  }
  // ---- blur_x / blur_y on the reference container types
  const long ny = 37, nx = 70;
  hpc::HPCHighDimensionFlatArray<2, float, 8> a(ny, nx);
  hpc::HPCHighDimensionFlatArray<2, float> b(ny, nx);
  for (long yy = -8; yy < ny + 8; ++yy)
    for (long xx = -8; xx < nx + 8; ++xx) a.at({yy, xx}) = std::sin(0.37f * yy + 0.11f * xx);
  for (int dir = 0; dir < 2; ++dir) {
    if (dir == 0) hpc::blur_x<8>(a, b); else hpc::blur_y<8>(a, b);
    for (long yy = 0; yy < ny; ++yy)
      for (long xx = 0; xx < nx; ++xx) {
        float res = 0.f;
        for (int k = -8; k <= 8; ++k) res += dir == 0 ? a(yy, xx + k) : a(yy + k, xx);
        if (res != b(yy, xx)) return fail(dir == 0 ? "blur_x mismatch" : "blur_y mismatch");
      }
  }
  // ---- stencil7
  hpc::HPCHighDimensionFlatArray<3, float, 1> u(9, 10, 11), o(9, 10, 11);
  for (long z = 0; z < 9; ++z)
    for (long yy = 0; yy < 10; ++yy)
      for (long xx = 0; xx < 11; ++xx) u(z, yy, xx) = std::cos(0.3f * z + 0.7f * yy - 0.2f * xx);
  hpc::stencil7(u, o, -6.f, 1.f);
  for (long z = 0; z < 9; ++z)
    for (long yy = 0; yy < 10; ++yy)
      for (long xx = 0; xx < 11; ++xx) {
        float s = u(z - 1, yy, xx) + u(z + 1, yy, xx);
        s = s + u(z, yy - 1, xx);
        s = s + u(z, yy + 1, xx);
        s = s + u(z, yy, xx - 1);
        s = s + u(z, yy, xx + 1);
        const float t0 = -6.f * u(z, yy, xx), t1 = 1.f * s;
        if (t0 + t1 != o(z, yy, xx)) return fail("stencil7 mismatch");
      }
  // ---- multi-GPU layer at world 1 (sparse/Dist.hpp): K = 2 interleaved
  //      chunks through lhpc_dist_spmv equal the single-plan y bit for bit
  {
    sparse::DistComm comm(sparse::DistComm::unique_id(), 1, 0, 0);
    const int K = 2;
    const auto cuts = sparse::interleaved_cuts(A, 1, K);
    const auto L = sparse::interleaved_local(A, cuts, 1, K, 0);
    sparse::DistSpMVPlan<float> dplan(comm, n, m, K, cuts, L);
    float *dx = nullptr, *dy = nullptr;
    double *dd = nullptr;
    auto hip_ok = [](hipError_t e) { return e == hipSuccess; };
    if (!hip_ok(hipMalloc(&dx, sizeof(float) * m)) || !hip_ok(hipMalloc(&dy, sizeof(float) * n)) ||
        !hip_ok(hipMalloc(&dd, sizeof(double) * 4)))
      return fail("hipMalloc");
    if (!hip_ok(hipMemcpy(dx, x.data(), sizeof(float) * m, hipMemcpyHostToDevice))) return fail("hipMemcpy");
    sparse::spmv(dplan, dx, dy);
    std::vector<float> yd(static_cast<std::size_t>(n));
    if (!hip_ok(hipMemcpy(yd.data(), dy, sizeof(float) * n, hipMemcpyDeviceToHost))) return fail("hipMemcpy");
    for (std::int64_t i = 0; i < n; ++i)
      if (yd[std::size_t(i)] != y(i)) return fail("dist spmv mismatch");
    const double h4[4] = {1.5, -2.0, 3.25, 0.0};
    double b4[4];
    if (!hip_ok(hipMemcpy(dd, h4, sizeof(h4), hipMemcpyHostToDevice))) return fail("hipMemcpy");
    comm.allreduce_sum(dd, 4);
    if (!hip_ok(hipMemcpy(b4, dd, sizeof(b4), hipMemcpyDeviceToHost))) return fail("hipMemcpy");
    for (int i = 0; i < 4; ++i)
      if (b4[i] != h4[i]) return fail("allreduce world 1");
    // RCCL-free local communicator with a registered y window (world 1:
    // no peers; the P2P calls and the dist plan must still work through it)
    {
      auto lc = sparse::DistComm::local(1, 0, 0);
      const auto blob = lc.p2p_export(dy, static_cast<std::int64_t>(sizeof(float) * n));
      lc.p2p_import({blob});
      sparse::DistSpMVPlan<float> lplan(lc, n, m, K, cuts, L);
      if (!hip_ok(hipMemset(dy, 0xFF, sizeof(float) * n))) return fail("hipMemset");
      sparse::spmv(lplan, dx, dy);
      if (!hip_ok(hipMemcpy(yd.data(), dy, sizeof(float) * n, hipMemcpyDeviceToHost))) return fail("hipMemcpy");
      for (std::int64_t i = 0; i < n; ++i)
        if (yd[std::size_t(i)] != y(i)) return fail("local-comm dist spmv mismatch");
      // the P2P scalar all-reduce of a local communicator (world 1: unchanged)
      lc.allreduce_sum(dd, 4);
      if (!hip_ok(hipMemcpy(b4, dd, sizeof(b4), hipMemcpyDeviceToHost))) return fail("hipMemcpy");
      for (int i = 0; i < 4; ++i)
        if (b4[i] != h4[i]) return fail("local-comm allreduce world 1");
    }
    // chained calls (cross-step overlap API) at world 1: x → y → x
    {
      float *dz = nullptr;
      if (!hip_ok(hipMalloc(&dz, sizeof(float) * m))) return fail("hipMalloc");
      sparse::spmv_begin(dplan, dx, dy);
      sparse::spmv_end(dplan);
      std::vector<float> y1(static_cast<std::size_t>(n));
      if (!hip_ok(hipMemcpy(y1.data(), dy, sizeof(float) * n, hipMemcpyDeviceToHost))) return fail("hipMemcpy");
      for (std::int64_t i = 0; i < n; ++i)
        if (y1[std::size_t(i)] != y(i)) return fail("spmv_begin/end mismatch");
      (void)hipFree(dz);
    }
    // explicit variant options: the RCCL exchange driven at world 1 (an
    // in-place no-op), then the exchange alone; the schedule as data
    {
      auto o = sparse::default_options();
      o.dist_exchange = LHPC_DIST_EXCHANGE_RCCL;
      o.dist_world1 = 1;
      o.dist_broadcast = 1;
      sparse::DistSpMVPlan<float> oplan(comm, n, m, K, cuts, L, LHPC_PLAN_DEFAULT, &o);
      sparse::spmv(oplan, dx, dy);
      sparse::exchange(oplan, dy);
      if (!hip_ok(hipMemcpy(yd.data(), dy, sizeof(float) * n, hipMemcpyDeviceToHost))) return fail("hipMemcpy");
      for (std::int64_t i = 0; i < n; ++i)
        if (yd[std::size_t(i)] != y(i)) return fail("options dist spmv mismatch");
      const auto sched = sparse::exchange_schedule(cuts, 1, K, 0, LHPC_DIST_EXCHANGE_RCCL, true);
      std::int64_t rows = 0;
      for (const auto &t : sched) rows += t.kind == LHPC_XFER_BROADCAST ? t.count : 0;
      if (rows != n) return fail("broadcast schedule covers every row once");
    }
    if (!hip_ok(hipFree(dx)) || !hip_ok(hipFree(dy)) || !hip_ok(hipFree(dd))) return fail("hipFree");
  }
  // ---- single-process multi-device plan: the device listed
  //      twice (the box has one GPU) — host vectors, then full replicas
  {
    sparse::SpMVPlan<float> mplan(A, std::vector<int>{0, 0});
    if (mplan.devices() != 2) return fail("multi plan devices");
    hpc::HPCHighDimensionFlatArray<1, float> ym(n);
    sparse::spmv(mplan, x, ym);
    for (std::int64_t i = 0; i < n; ++i)
      if (ym(i) != y(i)) return fail("multi-device spmv mismatch");
    float *dx = nullptr, *dy0 = nullptr, *dy1 = nullptr;
    if (hipMalloc(&dx, sizeof(float) * m) != hipSuccess || hipMalloc(&dy0, sizeof(float) * n) != hipSuccess ||
        hipMalloc(&dy1, sizeof(float) * n) != hipSuccess)
      return fail("hipMalloc");
    if (hipMemcpy(dx, x.data(), sizeof(float) * m, hipMemcpyHostToDevice) != hipSuccess) return fail("hipMemcpy");
    sparse::spmv_multi(mplan, {dx, dx}, {dy0, dy1});
    if (hipDeviceSynchronize() != hipSuccess) return fail("sync");
    std::vector<float> h0(static_cast<std::size_t>(n)), h1(static_cast<std::size_t>(n));
    if (hipMemcpy(h0.data(), dy0, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(h1.data(), dy1, sizeof(float) * n, hipMemcpyDeviceToHost) != hipSuccess)
      return fail("hipMemcpy");
    for (std::int64_t i = 0; i < n; ++i)
      if (h0[std::size_t(i)] != y(i) || h1[std::size_t(i)] != y(i)) return fail("multi-device replicas mismatch");
    (void)hipFree(dx);
    (void)hipFree(dy0);
    (void)hipFree(dy1);
  }
  // ---- RootGrid → device CSR (GPU COO → CSR) → plan from device arrays
  {
    sparse::RootGrid<float, sparse::HashBlock<sparse::DenseBlock<16, float>>> grid;
    for (std::int64_t i = 0; i < n; ++i)
      for (auto k = A.row_ptr[i]; k < A.row_ptr[i + 1]; ++k) grid.write(i, A.col_idx[k], A.val[k] == 0.f ? 0.5f : A.val[k]);
    auto dA = sparse::to_csr_device<float>(grid, 0, 0, n, m, 0);
    sparse::SpMVPlan<float> dplan2(dA.view());
    hpc::HPCHighDimensionFlatArray<1, float> yg(n);
    sparse::spmv(dplan2, x, yg);
    for (std::int64_t i = 0; i < n; ++i) {
      double s = 0;
      for (auto k = A.row_ptr[i]; k < A.row_ptr[i + 1]; ++k)
        s += double(A.val[k] == 0.f ? 0.5f : A.val[k]) * double(x(A.col_idx[k]));
      if (static_cast<float>(s) != yg(i)) return fail("grid → device CSR → spmv mismatch");
    }
  }
  // ---- explicit XTILE column blocks through the options (more launches);
  //      both plans within the 1e-6·Σ|a·x| bound of the fp64 row sums
  {
    auto o = sparse::default_options();
    o.xtile_col_blocks = 3;
    sparse::SpMVPlan<float> cb(A, -1, LHPC_PLAN_FORCE_XTILE, &o);
    sparse::SpMVPlan<float> one(A, -1, LHPC_PLAN_FORCE_XTILE);
    if (cb.info().launches <= one.info().launches) return fail("column blocks: more launches expected");
    hpc::HPCHighDimensionFlatArray<1, float> y1(n), y3(n);
    sparse::spmv(one, x, y1);
    sparse::spmv(cb, x, y3);
    for (std::int64_t i = 0; i < n; ++i) {
      double s = 0, a = 0;
      for (auto k = A.row_ptr[i]; k < A.row_ptr[i + 1]; ++k) {
        s += double(A.val[k]) * double(x(A.col_idx[k]));
        a += std::fabs(double(A.val[k]) * double(x(A.col_idx[k])));
      }
      if (std::fabs(double(y3(i)) - s) > 1e-6 * a + 1e-30 || std::fabs(double(y1(i)) - s) > 1e-6 * a + 1e-30)
        return fail("column blocks spmv outside the bound");
    }
  }
  std::printf("cpp api gpu: ok (spmv kernel %d)\n", plan.info().kernel);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc > 1 && !std::strcmp(argv[1], "gpu")) return gpu_mode();
  return layout_mode();
}
