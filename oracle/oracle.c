/*
 * oracle.c — CPU restatement of the libHPC hot path.  TEST INFRASTRUCTURE
 * ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg, as the checker / reported baseline.  Never linked into
 * or called by the product (libhpc_amd/_lib/liblhpc.so).
 *
 * Parity anchors
 *  - blur_x / blur_y: tests/test_hpc_benchmark/test_hpc_benchmark.cpp:354-368
 *    (BM_x_blur) and :444-457 (BM_y_blur): res = 0.f; for blur in
 *    [-nblur, nblur] ascending: res += a(...); b(y,x) = res.  The SSE twins
 *    (:425-441 BM_x_blur_tiling_simd_prefetch, :575-601
 *    BM_YXx_blur_tiling_prefetch_streamed_IPL) add lane-wise in the same
 *    order and are bit-identical (verified during the survey).
 *    Layout: HPCHighDimensionFlatArray<2,float,ghost>
 *    (lib/hpc/include/HPCHighDimensionFlatArray.hpp:161-187), pinned by
 *    oracle/ref_probe.cpp compiled against the reference header itself.
 *  - spmv: ABSENT from the reference — parity unpinned by the
 *    reference.  Restated from the standard CSR definition with sequential
 *    ascending-k accumulation in fp64; pinned instead to
 *    exact arithmetic (tests/test_oracle.py: Fractions on dyadic inputs,
 *    math.fsum on random inputs) and cross-checked against scipy.sparse.
 *  - stencil7: build-defined (BASELINE config C5) on the same ghost layout,
 *    evaluated in the order SURVEY §8d fixes, compiled -ffp-contract=off.
 *
 * The *_simd functions are the CPU baseline ("port" kind): the reference has
 * no CPU SpMV, so they are written in its idiom — OpenMP parallel for,
 * _mm_prefetch of the next line (test_hpc_benchmark.cpp:184), SSE/AVX2
 * loads — and the blur baselines restate the reference's SSE loops.
 */
#include <immintrin.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORACLE_API __attribute__((visibility("default")))

static inline int64_t rp_at(const void *rp, int bits, int64_t i) {
  return bits == 64 ? ((const int64_t *)rp)[i] : (int64_t)((const int32_t *)rp)[i];
}

/* ------------------------------------------------------------ SpMV oracle */
/* y64[i] = Σ_k val[k]·x[col[k]] accumulated sequentially, ascending k, fp64. */
ORACLE_API void oracle_spmv_f32(int64_t n_rows, const void *row_ptr, int rp_bits,
                                const int32_t *col, const float *val, const float *x,
                                double *y64, float *y32, double *abs_sum) {
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t i = 0; i < n_rows; ++i) {
    double acc = 0.0, aacc = 0.0;
    const int64_t e = rp_at(row_ptr, rp_bits, i + 1);
    for (int64_t k = rp_at(row_ptr, rp_bits, i); k < e; ++k) {
      const double p = (double)val[k] * (double)x[col[k]]; /* exact in fp64 */
      acc += p;
      aacc += fabs(p);
    }
    if (y64) y64[i] = acc;
    if (y32) y32[i] = (float)acc;
    if (abs_sum) abs_sum[i] = aacc;
  }
}

ORACLE_API void oracle_spmv_f64(int64_t n_rows, const void *row_ptr, int rp_bits,
                                const int32_t *col, const double *val, const double *x,
                                double *y64, double *abs_sum) {
#pragma omp parallel for schedule(dynamic, 1024)
  for (int64_t i = 0; i < n_rows; ++i) {
    double acc = 0.0, aacc = 0.0;
    const int64_t e = rp_at(row_ptr, rp_bits, i + 1);
    for (int64_t k = rp_at(row_ptr, rp_bits, i); k < e; ++k) {
      const double p = val[k] * x[col[k]];
      acc += p;
      aacc += fabs(p);
    }
    y64[i] = acc;
    if (abs_sum) abs_sum[i] = aacc;
  }
}

/* ------------------------------------------------- SpMV CPU SIMD baseline */
/* OpenMP over rows (static chunks), AVX2 8-wide gathers of x, products
 * accumulated in fp64 (matching the GPU numerics), _mm_prefetch of the
 * val/col stream one cache line ahead as the reference does for its blur
 * (test_hpc_benchmark.cpp:184).  Returns the thread count used. */
__attribute__((target("avx2,fma"))) static void spmv_rows_avx2_f32(
    int64_t r0, int64_t r1, const void *row_ptr, int rp_bits, const int32_t *col,
    const float *val, const float *x, float *y) {
  for (int64_t i = r0; i < r1; ++i) {
    const int64_t s = rp_at(row_ptr, rp_bits, i), e = rp_at(row_ptr, rp_bits, i + 1);
    _mm_prefetch((const char *)(val + e + 16), _MM_HINT_T0);
    _mm_prefetch((const char *)(col + e + 16), _MM_HINT_T0);
    __m256d acc0 = _mm256_setzero_pd(), acc1 = _mm256_setzero_pd();
    int64_t k = s;
    for (; k + 8 <= e; k += 8) {
      const __m256i ci = _mm256_loadu_si256((const __m256i *)(col + k));
      const __m256 xv = _mm256_i32gather_ps(x, ci, 4);
      const __m256 vv = _mm256_loadu_ps(val + k);
      /* fp64 products: widen both operands, then multiply (exact) */
      const __m256d vlo = _mm256_cvtps_pd(_mm256_castps256_ps128(vv));
      const __m256d vhi = _mm256_cvtps_pd(_mm256_extractf128_ps(vv, 1));
      const __m256d xlo = _mm256_cvtps_pd(_mm256_castps256_ps128(xv));
      const __m256d xhi = _mm256_cvtps_pd(_mm256_extractf128_ps(xv, 1));
      acc0 = _mm256_add_pd(acc0, _mm256_mul_pd(vlo, xlo));
      acc1 = _mm256_add_pd(acc1, _mm256_mul_pd(vhi, xhi));
    }
    __m256d acc = _mm256_add_pd(acc0, acc1);
    double t[4];
    _mm256_storeu_pd(t, acc);
    double sum = (t[0] + t[1]) + (t[2] + t[3]);
    for (; k < e; ++k) sum += (double)val[k] * (double)x[col[k]];
    y[i] = (float)sum;
  }
}

__attribute__((target("avx2,fma"))) static void spmv_rows_avx2_f64(
    int64_t r0, int64_t r1, const void *row_ptr, int rp_bits, const int32_t *col,
    const double *val, const double *x, double *y) {
  for (int64_t i = r0; i < r1; ++i) {
    const int64_t s = rp_at(row_ptr, rp_bits, i), e = rp_at(row_ptr, rp_bits, i + 1);
    _mm_prefetch((const char *)(val + e + 8), _MM_HINT_T0);
    _mm_prefetch((const char *)(col + e + 16), _MM_HINT_T0);
    __m256d acc = _mm256_setzero_pd();
    int64_t k = s;
    for (; k + 4 <= e; k += 4) {
      const __m128i ci = _mm_loadu_si128((const __m128i *)(col + k));
      const __m256d xv = _mm256_i32gather_pd(x, ci, 8);
      acc = _mm256_add_pd(acc, _mm256_mul_pd(_mm256_loadu_pd(val + k), xv));
    }
    double t[4];
    _mm256_storeu_pd(t, acc);
    double sum = (t[0] + t[1]) + (t[2] + t[3]);
    for (; k < e; ++k) sum += val[k] * x[col[k]];
    y[i] = sum;
  }
}

ORACLE_API int cpu_spmv_simd(int dtype, int64_t n_rows, const void *row_ptr, int rp_bits,
                             const int32_t *col, const void *val, const void *x, void *y,
                             int threads) {
  if (threads <= 0) threads = omp_get_max_threads();
  const int64_t chunk = 4096;
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t r0 = 0; r0 < n_rows; r0 += chunk) {
    const int64_t r1 = r0 + chunk < n_rows ? r0 + chunk : n_rows;
    if (dtype == 0)
      spmv_rows_avx2_f32(r0, r1, row_ptr, rp_bits, col, (const float *)val,
                         (const float *)x, (float *)y);
    else
      spmv_rows_avx2_f64(r0, r1, row_ptr, rp_bits, col, (const double *)val,
                         (const double *)x, (double *)y);
  }
  return threads;
}

/* ------------------------------------------------------------- blur oracle */
/* a: HPCHighDimensionFlatArray<2,float,ghost> with logical (ny, nx);
 * b: HPCHighDimensionFlatArray<2,float,0> (ny, nx). */
ORACLE_API void oracle_blur_x(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                              int nblur) {
  const int64_t P = nx + 2 * ghost;
#pragma omp parallel for schedule(static)
  for (int64_t y = 0; y < ny; ++y) {
    const float *row = a + (y + ghost) * P + ghost;
    for (int64_t x = 0; x < nx; ++x) {
      float res = 0.f;
      for (int k = -nblur; k <= nblur; ++k) res += row[x + k];
      b[y * nx + x] = res;
    }
  }
}

ORACLE_API void oracle_blur_y(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                              int nblur) {
  const int64_t P = nx + 2 * ghost;
#pragma omp parallel for schedule(static)
  for (int64_t y = 0; y < ny; ++y) {
    for (int64_t x = 0; x < nx; ++x) {
      float res = 0.f;
      for (int k = -nblur; k <= nblur; ++k) res += a[(y + k + ghost) * P + ghost + x];
      b[y * nx + x] = res;
    }
  }
}

/* CPU baselines: the reference's SSE blurs restated (lane-wise ascending
 * adds, streaming stores).  nblur = 8, nx % 16 == 0, ghost % 4 == 0. */
ORACLE_API int cpu_blur_x_sse(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                              int threads) {
  const int nb = 8;
  const int64_t P = nx + 2 * ghost;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t y = 0; y < ny; ++y) {
    const float *row = a + (y + ghost) * P + ghost;
    for (int64_t xb = 0; xb < nx; xb += 2 * nb) {
      _mm_prefetch((const char *)(row + xb + 2 * nb), _MM_HINT_T0);
      for (int64_t x = xb; x < xb + 2 * nb && x < nx; x += 4) {
        __m128 r = _mm_setzero_ps();
        for (int k = -nb; k <= nb; ++k) r = _mm_add_ps(_mm_loadu_ps(row + x + k), r);
        _mm_stream_ps(b + y * nx + x, r);
      }
    }
  }
  _mm_sfence();
  return threads;
}

ORACLE_API int cpu_blur_y_sse(const float *a, float *b, int64_t ny, int64_t nx, int64_t ghost,
                              int threads) {
  const int nb = 8, bs = 64;
  const int64_t P = nx + 2 * ghost;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(threads)
  for (int64_t y = 0; y < ny; ++y) {
    for (int64_t xb = 0; xb < nx; xb += bs) {
      _mm_prefetch((const char *)(a + (y + nb + ghost) * P + ghost + xb), _MM_HINT_T0);
      for (int64_t x = xb; x < xb + bs && x < nx; x += 16) {
        __m128 r[4];
        for (int o = 0; o < 4; ++o) r[o] = _mm_setzero_ps();
        for (int k = -nb; k <= nb; ++k)
          for (int o = 0; o < 4; ++o)
            r[o] = _mm_add_ps(r[o], _mm_loadu_ps(a + (y + k + ghost) * P + ghost + x + 4 * o));
        for (int o = 0; o < 4; ++o) _mm_stream_ps(b + y * nx + x + 4 * o, r[o]);
      }
    }
  }
  _mm_sfence();
  return threads;
}

/* --------------------------------------------------------- stencil7 oracle */
ORACLE_API void oracle_stencil7(const float *u, float *out, int64_t nz, int64_t ny, int64_t nx,
                                int64_t g, float c0, float c1, int threads) {
  const int64_t Px = nx + 2 * g, Pyx = (ny + 2 * g) * Px;
  if (threads <= 0) threads = omp_get_max_threads();
#pragma omp parallel for collapse(2) schedule(static) num_threads(threads)
  for (int64_t z = 0; z < nz; ++z)
    for (int64_t y = 0; y < ny; ++y) {
      const int64_t b = (z + g) * Pyx + (y + g) * Px + g;
      for (int64_t x = 0; x < nx; ++x) {
        const float *p = u + b + x;
        float s = p[-Pyx] + p[Pyx];
        s = s + p[-Px];
        s = s + p[Px];
        s = s + p[-1];
        s = s + p[1];
        const float t0 = c0 * p[0];
        const float t1 = c1 * s;
        out[b + x] = t0 + t1;
      }
    }
}

/* ------------------------------------------------------------ radix sort
 * LSD counting sort, 8-bit digits, ascending, stable — the algorithm of the
 * reference's sort::radix::details::radix_sort_v4 / _cache_v1
 * (lib/sort/radix_cpu/include/radix_sort_cpu.hpp:125-166, :168-203): per
 * pass, histogram the digit, exclusive-scan the 256 counts, scatter in input
 * order into the other buffer, swap.  Restricted to bits [begin, end) (the
 * GPU ABI's contract); the last digit is masked to the remaining bits.
 * Pinned by tests/test_oracle.py against numpy's stable sort and against the
 * reference's own CPU sort compiled from its sources (oracle/_ref).        */
#define ORACLE_SORT_BODY(KT)                                                         \
  KT *tk = (KT *)malloc((size_t)(n > 0 ? n : 1) * sizeof(KT));                      \
  uint32_t *tv = vals ? (uint32_t *)malloc((size_t)(n > 0 ? n : 1) * 4) : NULL;     \
  KT *ka = keys, *kb = tk;                                                           \
  uint32_t *va = vals, *vb = tv;                                                     \
  int passes = 0;                                                                    \
  for (int shift = begin; shift < end; shift += 8, ++passes) {                       \
    const int bits = end - shift < 8 ? end - shift : 8;                              \
    const uint64_t mask = (1ull << bits) - 1;                                        \
    int64_t cnt[256] = {0};                                                          \
    for (int64_t i = 0; i < n; ++i) cnt[(ka[i] >> shift) & mask]++;                 \
    int64_t sum = 0;                                                                 \
    for (int d = 0; d < 256; ++d) {                                                  \
      const int64_t c = cnt[d];                                                      \
      cnt[d] = sum;                                                                  \
      sum += c;                                                                      \
    }                                                                                \
    for (int64_t i = 0; i < n; ++i) {                                                \
      const int64_t p = cnt[(ka[i] >> shift) & mask]++;                              \
      kb[p] = ka[i];                                                                 \
      if (va) vb[p] = va[i];                                                         \
    }                                                                                \
    KT *tt = ka; ka = kb; kb = tt;                                                   \
    uint32_t *vt = va; va = vb; vb = vt;                                             \
  }                                                                                  \
  if (passes & 1) {                                                                  \
    memcpy(keys, ka, (size_t)n * sizeof(KT));                                        \
    if (vals) memcpy(vals, va, (size_t)n * 4);                                       \
  }                                                                                  \
  free(tk);                                                                          \
  free(tv);

ORACLE_API void oracle_radix_sort_u32(uint32_t *keys, uint32_t *vals, int64_t n, int begin, int end) {
  ORACLE_SORT_BODY(uint32_t)
}

ORACLE_API void oracle_radix_sort_u64(uint64_t *keys, uint32_t *vals, int64_t n, int begin, int end) {
  ORACLE_SORT_BODY(uint64_t)
}

/* COO → CSR: order by (row, col) with the stable sort
 * above on key = row << col_bits | col, then merge equal coordinates by
 * summing their values left to right in input order (the ABI's contract).
 * Returns the merged nnz, or -1 for an out-of-range coordinate.            */
#define ORACLE_COO(NAME, VT)                                                                          \
ORACLE_API int64_t NAME(int64_t n_rows, int64_t n_cols, int64_t nnz, const int32_t *rows,               \
                        const int32_t *cols, const VT *vals, int64_t *row_ptr, int32_t *col_out,        \
                        VT *val_out) {                                                                  \
  int cb = 1, rb = 1;                                                                               \
  while ((1ll << cb) < n_cols) ++cb;                                                                \
  while ((1ll << rb) < n_rows) ++rb;                                                                \
  uint64_t *k = (uint64_t *)malloc((size_t)(nnz > 0 ? nnz : 1) * 8);                                \
  uint32_t *ix = (uint32_t *)malloc((size_t)(nnz > 0 ? nnz : 1) * 4);                               \
  for (int64_t i = 0; i < nnz; ++i) {                                                               \
    if (rows[i] < 0 || rows[i] >= n_rows || cols[i] < 0 || cols[i] >= n_cols) {                     \
      free(k);                                                                                      \
      free(ix);                                                                                     \
      return -1;                                                                                    \
    }                                                                                               \
    k[i] = ((uint64_t)rows[i] << cb) | (uint64_t)cols[i];                                           \
    ix[i] = (uint32_t)i;                                                                            \
  }                                                                                                 \
  oracle_radix_sort_u64(k, ix, nnz, 0, cb + rb);                                                    \
  int64_t u = 0;                                                                                    \
  for (int64_t r = 0; r <= n_rows; ++r) row_ptr[r] = 0;                                             \
  for (int64_t i = 0; i < nnz;) {                                                                   \
    VT s = vals[ix[i]];                                                                             \
    int64_t j = i + 1;                                                                              \
    while (j < nnz && k[j] == k[i]) s = s + vals[ix[j++]];                                          \
    col_out[u] = (int32_t)(k[i] & ((1ull << cb) - 1));                                              \
    val_out[u] = s;                                                                                 \
    row_ptr[(int64_t)(k[i] >> cb) + 1]++;                                                           \
    ++u;                                                                                            \
    i = j;                                                                                          \
  }                                                                                                 \
  for (int64_t r = 0; r < n_rows; ++r) row_ptr[r + 1] += row_ptr[r];                                \
  free(k);                                                                                          \
  free(ix);                                                                                         \
  return u;                                                                                         \
}
ORACLE_COO(oracle_coo_to_csr_f64, double)
ORACLE_COO(oracle_coo_to_csr_f32, float)

/* ------------------------------------------------------------------ CG
 * Conjugate gradient in fp64 (no reference counterpart):
 * the textbook recurrence the GPU solver (lhpc_solver.hip) runs —
 *   r = b - A·x; p = r; rr = r·r
 *   loop: q = A·p; α = rr / p·q; x += α·p; r -= α·q; rr' = r·r;
 *         stop if rr' ≤ tol²·b·b; β = rr'/rr; p = r + β·p
 * with sequential ascending-index sums.  Returns the iterations run;
 * *resid = ‖r‖/‖b‖ of the recursive residual.  x is the initial guess in.  */
ORACLE_API int oracle_cg_f64(int64_t n, const void *rp, int bits, const int32_t *col, const double *val,
                             const double *b, double *x, double tol, int max_iter, double *resid) {
  double *r = (double *)malloc((size_t)(n > 0 ? n : 1) * 8), *p = (double *)malloc((size_t)(n > 0 ? n : 1) * 8),
         *q = (double *)malloc((size_t)(n > 0 ? n : 1) * 8);
  double bb = 0.0, rr = 0.0;
  for (int64_t i = 0; i < n; ++i) bb += b[i] * b[i];
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0;
    for (int64_t k = rp_at(rp, bits, i); k < rp_at(rp, bits, i + 1); ++k) s += val[k] * x[col[k]];
    r[i] = b[i] - s;
    p[i] = r[i];
    rr += r[i] * r[i];
  }
  const double stop = tol * tol * (bb > 0.0 ? bb : 1.0);
  int it = 0;
  if (rr > stop) {
    for (it = 1; it <= max_iter; ++it) {
      double pq = 0.0;
      for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t k = rp_at(rp, bits, i); k < rp_at(rp, bits, i + 1); ++k) s += val[k] * p[col[k]];
        q[i] = s;
      }
      for (int64_t i = 0; i < n; ++i) pq += p[i] * q[i];
      const double alpha = rr / pq;
      double rn = 0.0;
      for (int64_t i = 0; i < n; ++i) {
        x[i] += alpha * p[i];
        r[i] -= alpha * q[i];
        rn += r[i] * r[i];
      }
      if (rn <= stop) {
        rr = rn;
        break;
      }
      const double beta = rn / rr;
      for (int64_t i = 0; i < n; ++i) p[i] = r[i] + beta * p[i];
      rr = rn;
    }
    if (it > max_iter) it = max_iter;
  }
  *resid = sqrt(rr) / sqrt(bb > 0.0 ? bb : 1.0);
  free(r);
  free(p);
  free(q);
  return it;
}
