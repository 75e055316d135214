// lhpc_solver.hip — conjugate gradient on the SpMV plan (SURVEY §8f rank 3:
// "iterative consumer (CG/Jacobi) loop using SpMV + allgather + dot-product
// allreduce — makes 'y becomes the next x' real").  No reference
// counterpart.
//
// Per iteration (HBM-bound vector work around one SpMV):
//   q = A·p, pq = p·q               lhpc_spmv_dot (fused into the ADAPTIVE epilogue;
//                                   SpMV + k_dot_partial/k_dot_finish for other plans)
//   α = rr/pq; r -= α·q; rr' = r·r  k_cg_r (reads r q, writes r, block partials) + k_dot_finish
//   β = rr'/rr; x += α·p;           k_cg_xp (reads x p r, writes x p)
//   p = r + β·p
// (k_cg_xr / k_cg_p, the x update beside the r update, stay as building
// blocks of the C ABI.)  On SELL plans k_cg_xp is fused into the next
// iteration's SpMV (lhpc_spmv_csr.hip k_spmv_sell_cg): two passes per
// iteration, x bit-identical to the three-pass loop.
// α and β are read on the device from fp64 scalars, so no host round trip is
// needed between kernels; the host reads rr' only every `check_every`
// iterations to test convergence.  Dots accumulate in fp64 with a fixed
// two-stage order (per-block strided sums, then one block in index order):
// results are deterministic run to run.  The building blocks are exported so
// the multi-GPU solver (libhpc_amd/dist.py) can put an RCCL all-reduce
// between the dot and its use, and an all-gather of p after k_cg_p.
#include <hip/hip_runtime.h>

#include <atomic>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "lhpc_common.hpp"
#include "lhpc_spmv_impl.hpp"

namespace lhpc {
namespace {

constexpr int kVecThreads = 256;
constexpr int kDotBlocks = 1024;

__device__ __forceinline__ double block_sum(double v, double *sh) {
  for (int o = kWave / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  const int w = threadIdx.x / kWave, lane = threadIdx.x & (kWave - 1);
  if (lane == 0) sh[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kVecThreads / kWave; ++i) s += sh[i];
  return s;  // valid in thread 0
}

template <typename T>
__global__ __launch_bounds__(kVecThreads) void k_dot_partial(const T *__restrict__ a, const T *__restrict__ b,
                                                             int64_t n, double *__restrict__ part) {
  __shared__ double sh[kVecThreads / kWave];
  double s = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kVecThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kVecThreads)
    s += static_cast<double>(a[i]) * static_cast<double>(b[i]);
  const double t = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// out = Σ part[0..nb) in a fixed order (one block)
__global__ __launch_bounds__(kVecThreads) void k_dot_finish(const double *__restrict__ part, int nb,
                                                            double *__restrict__ out) {
  __shared__ double sh[kVecThreads / kWave];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += kVecThreads) s += part[i];
  const double t = block_sum(s, sh);
  if (threadIdx.x == 0) *out = t;
}

template <typename T>
__global__ __launch_bounds__(kVecThreads) void k_cg_xr(T *__restrict__ x, const T *__restrict__ p,
                                                       T *__restrict__ r, const T *__restrict__ q, int64_t n,
                                                       const double *__restrict__ num,
                                                       const double *__restrict__ den, double *__restrict__ part) {
  __shared__ double sh[kVecThreads / kWave];
  const double alpha = *num / *den;
  const T a = static_cast<T>(alpha);
  double s = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kVecThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kVecThreads) {
    x[i] = x[i] + a * p[i];
    const T ri = r[i] - a * q[i];
    r[i] = ri;
    s += static_cast<double>(ri) * static_cast<double>(ri);
  }
  const double t = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <typename T>
__global__ __launch_bounds__(kVecThreads) void k_cg_p(const T *__restrict__ r, T *__restrict__ p, int64_t n,
                                                      const double *__restrict__ num,
                                                      const double *__restrict__ den) {
  const T beta = static_cast<T>(*num / *den);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kVecThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kVecThreads)
    p[i] = r[i] + beta * p[i];
}

// The x update moved next to the p update (k_cg_r + k_cg_xp replace
// k_cg_xr + k_cg_p): r -= α·q with rr' = r·r reads r, q and writes r; then
// x += α·p, p = r + β·p reads x, p, r and writes x, p — eight vector passes
// per iteration instead of nine, the same operations on the same values
// (bit-identical x, r, p).  β = null: x += α·p only (the last iteration).
template <typename T>
__global__ __launch_bounds__(kVecThreads) void k_cg_r(T *__restrict__ r, const T *__restrict__ q, int64_t n,
                                                      const double *__restrict__ num,
                                                      const double *__restrict__ den, double *__restrict__ part) {
  __shared__ double sh[kVecThreads / kWave];
  const T a = static_cast<T>(*num / *den);
  double s = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kVecThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kVecThreads) {
    const T ri = r[i] - a * q[i];
    r[i] = ri;
    s += static_cast<double>(ri) * static_cast<double>(ri);
  }
  const double t = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

template <typename T, bool P>
__global__ __launch_bounds__(kVecThreads) void k_cg_xp(T *__restrict__ x, T *__restrict__ p,
                                                       const T *__restrict__ r, int64_t n,
                                                       const double *__restrict__ anum,
                                                       const double *__restrict__ aden,
                                                       const double *__restrict__ bnum,
                                                       const double *__restrict__ bden) {
  const T a = static_cast<T>(*anum / *aden);
  const T beta = P ? static_cast<T>(*bnum / *bden) : T(0);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kVecThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kVecThreads) {
    const T pi = p[i];
    x[i] = x[i] + a * pi;
    if constexpr (P) p[i] = r[i] + beta * pi;
  }
}

// the fused loop's start: rr[1] = pq = 1 (any finite pair: they scale p_old = 0)
__global__ void k_cg_scalar_ones(double *a, double *b) {
  *a = 1.0;
  *b = 1.0;
}

// r = b - q, p = r, part = block partials of r·r
template <typename T>
__global__ __launch_bounds__(kVecThreads) void k_cg_init(const T *__restrict__ b, const T *__restrict__ q,
                                                         T *__restrict__ r, T *__restrict__ p, int64_t n,
                                                         double *__restrict__ part) {
  __shared__ double sh[kVecThreads / kWave];
  double s = 0.0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kVecThreads + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * kVecThreads) {
    const T ri = b[i] - q[i];
    r[i] = ri;
    p[i] = ri;
    s += static_cast<double>(ri) * static_cast<double>(ri);
  }
  const double t = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

int vec_grid(int64_t n) {
  return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(kDotBlocks, (n + kVecThreads - 1) / kVecThreads)));
}

struct Scratch {
  double *d = nullptr;
  hipStream_t s = nullptr;
  ~Scratch() {
    if (d) (void)hipFreeAsync(d, s);
  }
};

template <typename T>
int dot_dev(const T *a, const T *b, int64_t n, double *out, double *part, hipStream_t s) {
  const int g = vec_grid(n);
  hipLaunchKernelGGL((k_dot_partial<T>), dim3(g), dim3(kVecThreads), 0, s, a, b, n, part);
  hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(kVecThreads), 0, s, part, g, out);
  return check_launch(s);
}

// r -= α·q, rr_out = r·r with the caller's partials buffer (no allocation:
// the solver's iterations are captured into a graph)
int cg_r_launch(int dtype, int64_t n, const double *num, const double *den, void *r, const void *q, double *rr_out,
                double *part, hipStream_t s) {
  const int g = vec_grid(n);
  if (dtype == LHPC_F32)
    hipLaunchKernelGGL((k_cg_r<float>), dim3(g), dim3(kVecThreads), 0, s, static_cast<float *>(r),
                       static_cast<const float *>(q), n, num, den, part);
  else
    hipLaunchKernelGGL((k_cg_r<double>), dim3(g), dim3(kVecThreads), 0, s, static_cast<double *>(r),
                       static_cast<const double *>(q), n, num, den, part);
  hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(kVecThreads), 0, s, part, g, rr_out);
  return check_launch(s);
}

}  // namespace
}  // namespace lhpc

using namespace lhpc;

namespace {
int dtype_ok(int dtype) { return dtype == LHPC_F32 || dtype == LHPC_F64; }
}  // namespace

extern "C" int lhpc_vec_dot(int dtype, int64_t n, const void *a, const void *b, double *out, void *stream) {
  try {
    if (!dtype_ok(dtype) || n < 0 || !out || (n > 0 && (!a || !b))) return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Scratch part;
    part.s = s;
    LHPC_HIP_TRY(scratch_alloc(reinterpret_cast<void **>(&part.d), kDotBlocks * sizeof(double), s));
    if (dtype == LHPC_F32)
      return dot_dev(static_cast<const float *>(a), static_cast<const float *>(b), n, out, part.d, s);
    return dot_dev(static_cast<const double *>(a), static_cast<const double *>(b), n, out, part.d, s);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_cg_step_xr(int dtype, int64_t n, const double *alpha_num, const double *alpha_den, void *x,
                               const void *p, void *r, const void *q, double *rr_out, void *stream) {
  try {
    if (!dtype_ok(dtype) || n < 0 || !alpha_num || !alpha_den || !rr_out || (n > 0 && (!x || !p || !r || !q)))
      return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Scratch part;
    part.s = s;
    LHPC_HIP_TRY(scratch_alloc(reinterpret_cast<void **>(&part.d), kDotBlocks * sizeof(double), s));
    const int g = vec_grid(n);
    if (dtype == LHPC_F32)
      hipLaunchKernelGGL((k_cg_xr<float>), dim3(g), dim3(kVecThreads), 0, s, static_cast<float *>(x),
                         static_cast<const float *>(p), static_cast<float *>(r), static_cast<const float *>(q), n,
                         alpha_num, alpha_den, part.d);
    else
      hipLaunchKernelGGL((k_cg_xr<double>), dim3(g), dim3(kVecThreads), 0, s, static_cast<double *>(x),
                         static_cast<const double *>(p), static_cast<double *>(r), static_cast<const double *>(q), n,
                         alpha_num, alpha_den, part.d);
    hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(kVecThreads), 0, s, part.d, g, rr_out);
    return check_launch(s);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_cg_step_p(int dtype, int64_t n, const double *beta_num, const double *beta_den, const void *r,
                              void *p, void *stream) {
  try {
    if (!dtype_ok(dtype) || n < 0 || !beta_num || !beta_den || (n > 0 && (!r || !p))) return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int g = vec_grid(n);
    if (dtype == LHPC_F32)
      hipLaunchKernelGGL((k_cg_p<float>), dim3(g), dim3(kVecThreads), 0, s, static_cast<const float *>(r),
                         static_cast<float *>(p), n, beta_num, beta_den);
    else
      hipLaunchKernelGGL((k_cg_p<double>), dim3(g), dim3(kVecThreads), 0, s, static_cast<const double *>(r),
                         static_cast<double *>(p), n, beta_num, beta_den);
    return check_launch(s);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_cg_step_r(int dtype, int64_t n, const double *alpha_num, const double *alpha_den, void *r,
                              const void *q, double *rr_out, void *stream) {
  try {
    if (!dtype_ok(dtype) || n < 0 || !alpha_num || !alpha_den || !rr_out || (n > 0 && (!r || !q)))
      return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    Scratch part;
    part.s = s;
    LHPC_HIP_TRY(scratch_alloc(reinterpret_cast<void **>(&part.d), kDotBlocks * sizeof(double), s));
    const int g = vec_grid(n);
    if (dtype == LHPC_F32)
      hipLaunchKernelGGL((k_cg_r<float>), dim3(g), dim3(kVecThreads), 0, s, static_cast<float *>(r),
                         static_cast<const float *>(q), n, alpha_num, alpha_den, part.d);
    else
      hipLaunchKernelGGL((k_cg_r<double>), dim3(g), dim3(kVecThreads), 0, s, static_cast<double *>(r),
                         static_cast<const double *>(q), n, alpha_num, alpha_den, part.d);
    hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(kVecThreads), 0, s, part.d, g, rr_out);
    return check_launch(s);
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_cg_step_xp(int dtype, int64_t n, const double *alpha_num, const double *alpha_den,
                               const double *beta_num, const double *beta_den, void *x, void *p, const void *r,
                               void *stream) {
  try {
    const bool up = beta_num != nullptr;
    if (!dtype_ok(dtype) || n < 0 || !alpha_num || !alpha_den || (up && !beta_den) ||
        (n > 0 && (!x || !p || (up && !r))))
      return LHPC_ERR_INVALID_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int g = vec_grid(n);
    if (dtype == LHPC_F32) {
      float *xf = static_cast<float *>(x), *pf = static_cast<float *>(p);
      const float *rf = static_cast<const float *>(r);
      if (up)
        hipLaunchKernelGGL((k_cg_xp<float, true>), dim3(g), dim3(kVecThreads), 0, s, xf, pf, rf, n, alpha_num,
                           alpha_den, beta_num, beta_den);
      else
        hipLaunchKernelGGL((k_cg_xp<float, false>), dim3(g), dim3(kVecThreads), 0, s, xf, pf, rf, n, alpha_num,
                           alpha_den, beta_num, beta_den);
    } else {
      double *xd = static_cast<double *>(x), *pd = static_cast<double *>(p);
      const double *rd = static_cast<const double *>(r);
      if (up)
        hipLaunchKernelGGL((k_cg_xp<double, true>), dim3(g), dim3(kVecThreads), 0, s, xd, pd, rd, n, alpha_num,
                           alpha_den, beta_num, beta_den);
      else
        hipLaunchKernelGGL((k_cg_xp<double, false>), dim3(g), dim3(kVecThreads), 0, s, xd, pd, rd, n, alpha_num,
                           alpha_den, beta_num, beta_den);
    }
    return check_launch(s);
  } LHPC_ABI_CATCH
}

namespace {
int cg_solve_owned(lhpc_spmv_plan *plan, const void *b, void *x, double tol, int max_iter, int check_every,
                   int *iters_out, double *resid_out, void *stream);
}

#ifdef LHPC_DEBUG_BOUNDS
// Debug build only (tests/debug_build_check.py): iteration body number k
// (0-based, counted over the next solves) returns LHPC_ERR_INTERNAL after
// enqueueing its work — lhpc_cg_solve's error path with work on the stream.
namespace {
std::atomic<int> g_cg_fail_at{-1};
bool cg_fault_now() {
  const int v = g_cg_fail_at.load();
  if (v < 0) return false;
  g_cg_fail_at.store(v - 1);
  return v == 0;
}
}  // namespace
extern "C" int lhpc_debug_cg_fail_at(int k) {
  g_cg_fail_at.store(k);
  return LHPC_OK;
}
#endif

// One solve per plan at a time: the work vectors, scalars and captured
// graphs belong to the plan, so a second concurrent solve is
// refused instead of racing on them.  The flag is released only once the
// solve's stream has drained: an error return after the first enqueue
//  leaves kernels in flight that still use the plan's work, and
// the next solve (on any stream) may reuse it as soon as the flag is free.
extern "C" int lhpc_cg_solve(lhpc_spmv_plan *plan, const void *b, void *x, double tol, int max_iter,
                             int check_every, int *iters_out, double *resid_out, void *stream) {
  try {
    if (!plan || !b || !x || max_iter < 0 || !(tol >= 0.0)) return LHPC_ERR_INVALID_ARG;
    int idle = 0;
    if (!plan->cg_busy.compare_exchange_strong(idle, 1)) return LHPC_ERR_BUSY;
    struct Release {  // on every exit, the exception path included
      lhpc_spmv_plan *p;
      hipStream_t s;
      ~Release() {
        (void)hipStreamSynchronize(s);  // a no-op wait on the success path (already drained)
        p->cg_busy.store(0);
      }
    } release{plan, static_cast<hipStream_t>(stream)};
    return cg_solve_owned(plan, b, x, tol, max_iter, check_every, iters_out, resid_out, stream);
  } LHPC_ABI_CATCH
}

namespace {
int cg_solve_owned(lhpc_spmv_plan *plan, const void *b, void *x, double tol, int max_iter, int check_every,
                   int *iters_out, double *resid_out, void *stream) {
  lhpc_spmv_plan_info info{};
  LHPC_TRY(lhpc_spmv_plan_info_get(plan, &info));
  if (info.n_rows != info.n_cols) return LHPC_ERR_INVALID_ARG;  // CG needs a square (SPD) matrix
  RocTxRange rx("lhpc_cg_solve");
  const int64_t n = info.n_rows;
  const int dtype = info.dtype;
  const size_t ts = dtype == LHPC_F32 ? 4 : 8;
  if (check_every < 1) check_every = 1;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // work (kept with the plan, so a captured iteration block can be replayed
  // by later solves): r, p, q, x vectors + scalars [rr0, rr1, pq, bb] + dot
  // partials; the caller's x is copied in and out
  if (!plan->cg_vecs) {  // on the plan's device, whatever the caller's current device
    int cur = 0;
    LHPC_HIP_TRY(hipGetDevice(&cur));
    LHPC_HIP_TRY(hipSetDevice(plan->device));
    hipError_t e = hipMalloc(&plan->cg_vecs, static_cast<size_t>(std::max<int64_t>(n, 1)) * ts * 5);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&plan->cg_scal), (8 + kDotBlocks) * sizeof(double));
    (void)hipSetDevice(cur);
    LHPC_HIP_TRY(e);
  }
  char *vb = static_cast<char *>(plan->cg_vecs);
  void *r = vb, *p = vb + static_cast<size_t>(n) * ts, *q = vb + 2 * static_cast<size_t>(n) * ts;
  void *x_user = x;
  x = vb + 3 * static_cast<size_t>(n) * ts;
  // SELL plans fuse each iteration's x += α·p, p = r + β·p into the next
  // iteration's SpMV (sell_cg_step), which reads p from one buffer and writes
  // the other: the p of an iteration of parity c lives in pb[c]
  const bool fused = plan->kernel == LHPC_KERNEL_SELL && !plan->multi && plan->parts.empty() && n > 0 &&
                     plan->n_blocks <= int64_t{2048} * 2048;  // sell_cg_step's two-stage dot (≤ 2^30 rows)
  void *pb[2] = {p, vb + 4 * static_cast<size_t>(n) * ts};
  LHPC_HIP_TRY(hipMemcpyAsync(x, x_user, static_cast<size_t>(n) * ts, hipMemcpyDeviceToDevice, s));
  double *rr[2] = {plan->cg_scal, plan->cg_scal + 1}, *pq = plan->cg_scal + 2, *bb = plan->cg_scal + 3,
         *part = plan->cg_scal + 8;
  const int g = vec_grid(n);
  int it = 0;
  // the two scalars the host loop reads come back into pinned memory: no
  // asynchronous copy touches pageable host memory.  The
  // buffer belongs to the plan (allocated on the first solve, freed with the
  // plan): hipHostFree synchronises the whole device, so it is not paid per
  // solve
  if (!plan->h_scalars)
    LHPC_HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&plan->h_scalars), 2 * sizeof(double), hipHostMallocDefault));
  double *hs = plan->h_scalars;
  double &h_rr = hs[0], &h_bb = hs[1];
  h_rr = 0.0;
  h_bb = 0.0;
  // bb = b·b; q = A·x; r = b - q; p = r; rr = r·r
  if (dtype == LHPC_F32) LHPC_TRY(dot_dev(static_cast<const float *>(b), static_cast<const float *>(b), n, bb, part, s));
  else LHPC_TRY(dot_dev(static_cast<const double *>(b), static_cast<const double *>(b), n, bb, part, s));
  LHPC_TRY(lhpc_spmv(plan, x, q, 1, s));
  if (dtype == LHPC_F32)
    hipLaunchKernelGGL((k_cg_init<float>), dim3(g), dim3(kVecThreads), 0, s, static_cast<const float *>(b),
                       static_cast<const float *>(q), static_cast<float *>(r), static_cast<float *>(p), n, part);
  else
    hipLaunchKernelGGL((k_cg_init<double>), dim3(g), dim3(kVecThreads), 0, s, static_cast<const double *>(b),
                       static_cast<const double *>(q), static_cast<double *>(r), static_cast<double *>(p), n, part);
  hipLaunchKernelGGL(k_dot_finish, dim3(1), dim3(kVecThreads), 0, s, part, g, rr[0]);
  LHPC_TRY(check_launch(s));
  LHPC_HIP_TRY(hipMemcpyAsync(&h_bb, bb, 8, hipMemcpyDeviceToHost, s));  // pinned
  LHPC_HIP_TRY(hipMemcpyAsync(&h_rr, rr[0], 8, hipMemcpyDeviceToHost, s));
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  const double stop = tol * tol * (h_bb > 0.0 ? h_bb : 1.0);
  int cur = 0;
  int status = LHPC_OK;
  // one iteration's device work: q = A·p and p·q in one pass (ADAPTIVE), r -=
  // α·q with rr' = r·r, and (full) x += α·p, p = r + β·p in one pass.  Fused
  // (SELL): the previous iteration's x / p update, q = A·p and p·q in one
  // pass, then r -= α·q with rr' = r·r; nothing is left for after the block
  // but the pending x += α·p, which the next iteration's first pass does
  auto body = [&](int c, bool full) -> int {
    if (fused) {
      LHPC_TRY(sell_cg_step(plan, r, pb[c ^ 1], pb[c], x, q, rr[c ^ 1], pq, rr[c], rr[c ^ 1], pq, s));
      LHPC_TRY(cg_r_launch(dtype, n, rr[c], pq, r, q, rr[c ^ 1], part, s));
    } else {
      LHPC_TRY(lhpc_spmv_dot(plan, p, q, p, pq, s));
      LHPC_TRY(cg_r_launch(dtype, n, rr[c], pq, r, q, rr[c ^ 1], part, s));
      if (full) LHPC_TRY(lhpc_cg_step_xp(dtype, n, rr[c], pq, rr[c ^ 1], rr[c], x, p, r, s));
    }
#ifdef LHPC_DEBUG_BOUNDS
    if (cg_fault_now()) return LHPC_ERR_INTERNAL;
#endif
    return LHPC_OK;
  };
  // the pending x += α·p of the last iteration (parity c), when the loop ends
  auto finish_x = [&](int c) -> int {
    return lhpc_cg_step_xp(dtype, n, rr[c], pq, nullptr, nullptr, x, fused ? pb[c] : p, nullptr, s);
  };
  // Graph blocks: the C = check_every iterations between two convergence
  // checks — C − 1 full iterations and the C-th up to rr' — captured once per
  // starting parity of the rr pair and replayed (one launch instead of ≈ 5C;
  // the same kernels in the same order, so x is bit-identical to the loop's).
  // ADAPTIVE / SELL plans only (their fused dot allocates nothing after the
  // first call, which the x·x warm-up below makes); not on the null stream, not
  // for multi-device plans, not in the synchronous-check debug build.
#ifdef LHPC_DEBUG_SYNC
  bool graphs = false;
#else
  bool graphs = s != nullptr && check_every >= 4 &&
                (plan->kernel == LHPC_KERNEL_ADAPTIVE || plan->kernel == LHPC_KERNEL_SELL) && !plan->multi &&
                plan->parts.empty() && plan->n_blocks > 0;
#endif
  // kept with the plan: every pointer in them (the plan's arrays and work)
  // outlives the solve, so later solves with the same check_every replay them
  hipGraphExec_t *ge = plan->cg_graph;
  for (int c = 0; c < 2; ++c)
    if (ge[c] && plan->cg_graph_iters[c] != check_every) {
      (void)hipGraphExecDestroy(ge[c]);
      ge[c] = nullptr;
    }
  auto capture = [&](int c) -> bool {
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) return false;
    int st = LHPC_OK, cc = c;
    for (int i = 0; i < check_every - 1 && st == LHPC_OK; ++i, cc ^= 1) st = body(cc, true);
    if (st == LHPC_OK) st = body(cc, false);
    const hipError_t e = hipStreamEndCapture(s, &g);
    (void)hipGetLastError();
    bool ok = st == LHPC_OK && e == hipSuccess && g &&
              hipGraphInstantiate(&ge[c], g, nullptr, nullptr, 0) == hipSuccess;
    plan->cg_graph_iters[c] = ok ? check_every : 0;
    if (g) (void)hipGraphDestroy(g);
    if (!ok && ge[c]) {
      (void)hipGraphExecDestroy(ge[c]);
      ge[c] = nullptr;
    }
    return ok;
  };
  if (graphs && !plan->d_dpart) {  // the fused dot's partials exist before any capture
    LHPC_TRY(lhpc_spmv_dot(plan, x, q, x, pq, s));
  }
  int last = -1;  // parity of the last iteration whose x update is pending (fused)
  if (fused && h_rr > stop) {
    // the first iteration's "previous" step is x += 1·0, p = r + β·0 with
    // p_old = pb[1] = 0 and rr[1] = pq = 1: x unchanged and p = r exactly, so
    // every iteration (and every captured block) has the same form (after
    // the warm-up above, which writes pq)
    LHPC_HIP_TRY(hipMemsetAsync(pb[1], 0, static_cast<size_t>(n) * ts, s));
    hipLaunchKernelGGL(k_cg_scalar_ones, dim3(1), dim3(1), 0, s, rr[1], pq);
    LHPC_TRY(check_launch(s));
  }
  if (h_rr > stop) {
    for (it = 0; it < max_iter;) {
      if (graphs && it % check_every == 0 && it + check_every <= max_iter) {
        if (!ge[cur] && !capture(cur)) {
          graphs = false;  // capture refused: the plain loop below
          continue;
        }
        LHPC_HIP_TRY(hipGraphLaunch(ge[cur], s));
        it += check_every;
        const int c = cur ^ ((check_every - 1) & 1);  // parity of the block's last iteration
        LHPC_HIP_TRY(hipMemcpyAsync(&h_rr, rr[c ^ 1], 8, hipMemcpyDeviceToHost, s));
        LHPC_HIP_TRY(hipStreamSynchronize(s));
        if (!std::isfinite(h_rr)) {
          status = LHPC_ERR_INTERNAL;
          break;
        }
        if (h_rr <= stop) {
          LHPC_TRY(finish_x(c));  // x += α·p
          last = -1;
          break;
        }
        if (!fused) LHPC_TRY(lhpc_cg_step_xp(dtype, n, rr[c], pq, rr[c ^ 1], rr[c], x, p, r, s));
        last = c;
        cur = c ^ 1;
        continue;
      }
      ++it;
      LHPC_TRY(body(cur, false));
      if (it % check_every == 0 || it == max_iter) {
        LHPC_HIP_TRY(hipMemcpyAsync(&h_rr, rr[cur ^ 1], 8, hipMemcpyDeviceToHost, s));
        LHPC_HIP_TRY(hipStreamSynchronize(s));
        if (!std::isfinite(h_rr)) {
          status = LHPC_ERR_INTERNAL;  // breakdown (p·Ap = 0 or overflow): matrix not SPD?
          break;
        }
        if (h_rr <= stop) {
          LHPC_TRY(finish_x(cur));  // x += α·p
          last = -1;
          break;
        }
      }
      // x += α·p, then p = r + β·p (same pass; fused: in the next iteration's SpMV)
      if (!fused) LHPC_TRY(lhpc_cg_step_xp(dtype, n, rr[cur], pq, rr[cur ^ 1], rr[cur], x, p, r, s));
      last = cur;
      cur ^= 1;
    }
    if (it > max_iter) it = max_iter;
    if (fused && last >= 0 && status == LHPC_OK) LHPC_TRY(finish_x(last));  // max_iter reached
  }
  LHPC_HIP_TRY(hipMemcpyAsync(x_user, x, static_cast<size_t>(n) * ts, hipMemcpyDeviceToDevice, s));
  LHPC_HIP_TRY(hipStreamSynchronize(s));
  if (iters_out) *iters_out = it;
  if (resid_out) *resid_out = std::sqrt(std::max(h_rr, 0.0)) / std::sqrt(h_bb > 0.0 ? h_bb : 1.0);
  return status;
}
}  // namespace
