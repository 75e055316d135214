/*
 * asan_oracle.c — TEST INFRASTRUCTURE: drives every entry point of oracle.c
 * on small inputs in a binary built with -fsanitize=address,undefined
 * (`make -C oracle asan`, run by tests/test_asan.py), as the reference runs
 * all its Linux tests under ASan (/root/reference/tests/CMakeLists.txt:6-9).
 * Cross-checks are light (the oracle's numerics are pinned by
 * tests/test_oracle*.py); the point is memory safety of the checker itself,
 * including empty and ragged shapes.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_spmv_f32(int64_t, const void *, int, const int32_t *, const float *, const float *, double *, float *,
                     double *);
void oracle_spmv_f64(int64_t, const void *, int, const int32_t *, const double *, const double *, double *, double *);
int cpu_spmv_simd(int, int64_t, const void *, int, const int32_t *, const void *, const void *, void *, int);
void oracle_blur_x(const float *, float *, int64_t, int64_t, int64_t, int);
void oracle_blur_y(const float *, float *, int64_t, int64_t, int64_t, int);
int cpu_blur_x_sse(const float *, float *, int64_t, int64_t, int64_t, int);
int cpu_blur_y_sse(const float *, float *, int64_t, int64_t, int64_t, int);
void oracle_stencil7(const float *, float *, int64_t, int64_t, int64_t, int64_t, float, float, int);
void oracle_radix_sort_u32(uint32_t *, uint32_t *, int64_t, int, int);
void oracle_radix_sort_u64(uint64_t *, uint32_t *, int64_t, int, int);
int64_t oracle_coo_to_csr_f64(int64_t, int64_t, int64_t, const int32_t *, const int32_t *, const double *, int64_t *,
                              int32_t *, double *);
int oracle_cg_f64(int64_t, const void *, int, const int32_t *, const double *, const double *, double *, double, int,
                  double *);

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);      \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static uint64_t rng = 0x5EED0A5A;
static uint32_t next_u32(void) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (uint32_t)(rng >> 11);
}

static void spmv_case(int64_t n, int64_t m, int maxlen) {
  int64_t *rp = malloc((size_t)(n + 1) * 8);
  rp[0] = 0;
  for (int64_t i = 0; i < n; ++i) rp[i + 1] = rp[i] + (maxlen ? (int64_t)(next_u32() % (uint32_t)(maxlen + 1)) : 0);
  const int64_t nnz = rp[n];
  int32_t *col = malloc((size_t)(nnz ? nnz : 1) * 4);
  float *v32 = malloc((size_t)(nnz ? nnz : 1) * 4), *x32 = malloc((size_t)(m ? m : 1) * 4);
  double *v64 = malloc((size_t)(nnz ? nnz : 1) * 8), *x64 = malloc((size_t)(m ? m : 1) * 8);
  for (int64_t k = 0; k < nnz; ++k) {
    col[k] = (int32_t)(next_u32() % (uint32_t)m);
    v32[k] = (float)((int)(next_u32() % 17) - 8) / 8.0f;
    v64[k] = v32[k];
  }
  for (int64_t j = 0; j < m; ++j) x64[j] = x32[j] = (float)((int)(next_u32() % 17) - 8) / 8.0f;
  double *y64 = malloc((size_t)(n ? n : 1) * 8), *a = malloc((size_t)(n ? n : 1) * 8),
         *z64 = malloc((size_t)(n ? n : 1) * 8);
  float *y32 = malloc((size_t)(n ? n : 1) * 4), *s32 = malloc((size_t)(n ? n : 1) * 4);
  oracle_spmv_f32(n, rp, 64, col, v32, x32, y64, y32, a);
  oracle_spmv_f64(n, rp, 64, col, v64, x64, z64, a);
  CHECK(cpu_spmv_simd(0, n, rp, 64, col, v32, x32, s32, 2) == 2);
  for (int64_t i = 0; i < n; ++i) {  /* dyadic: every order is exact */
    CHECK(y64[i] == z64[i]);
    CHECK(s32[i] == y32[i]);
  }
  free(rp), free(col), free(v32), free(x32), free(v64), free(x64), free(y64), free(a), free(z64), free(y32), free(s32);
}

static void blur_case(int64_t ny, int64_t nx) {
  const int64_t g = 8, P = nx + 2 * g, N = (ny + 2 * g) * P;
  float *a = malloc((size_t)N * 4), *b1 = malloc((size_t)(ny * nx ? ny * nx : 1) * 4),
        *b2 = malloc((size_t)(ny * nx ? ny * nx : 1) * 4);
  for (int64_t i = 0; i < N; ++i) a[i] = (float)((int)(next_u32() % 17) - 8) / 8.0f;
  oracle_blur_x(a, b1, ny, nx, g, 8);
  if (nx % 16 == 0) { /* the SSE baselines' contract: nx % 16 == 0 */
    CHECK(cpu_blur_x_sse(a, b2, ny, nx, g, 2) == 2);
    CHECK(memcmp(b1, b2, (size_t)(ny * nx) * 4) == 0);
  }
  oracle_blur_y(a, b1, ny, nx, g, 8);
  if (nx % 16 == 0) {
    CHECK(cpu_blur_y_sse(a, b2, ny, nx, g, 2) == 2);
    CHECK(memcmp(b1, b2, (size_t)(ny * nx) * 4) == 0);
  }
  free(a), free(b1), free(b2);
}

int main(void) {
  spmv_case(0, 1, 3);
  spmv_case(1, 1, 3);
  spmv_case(65, 33, 0);
  spmv_case(1000, 4099, 40);
  blur_case(1, 1);
  blur_case(64, 64);
  blur_case(131, 257);
  blur_case(33, 128);
  {
    const int64_t nz = 5, ny = 7, nx = 9, g = 1, N = (nz + 2) * (ny + 2) * (nx + 2);
    float *u = calloc((size_t)N, 4), *o = calloc((size_t)N, 4);
    for (int64_t i = 0; i < N; ++i) u[i] = (float)(next_u32() % 5);
    oracle_stencil7(u, o, nz, ny, nx, g, -6.0f, 1.0f, 2);
    free(u), free(o);
  }
  {
    const int64_t n = 4097;
    uint32_t *k = malloc(n * 4), *v = malloc(n * 4);
    uint64_t *k64 = malloc(n * 8);
    for (int64_t i = 0; i < n; ++i) k[i] = next_u32(), v[i] = (uint32_t)i, k64[i] = ((uint64_t)next_u32() << 20) ^ i;
    oracle_radix_sort_u32(k, v, n, 0, 32);
    for (int64_t i = 1; i < n; ++i) CHECK(k[i - 1] <= k[i]);
    oracle_radix_sort_u64(k64, v, n, 0, 64);
    for (int64_t i = 1; i < n; ++i) CHECK(k64[i - 1] <= k64[i]);
    oracle_radix_sort_u32(k, NULL, 0, 0, 32);
    free(k), free(v), free(k64);
  }
  {
    const int32_t r[] = {2, 0, 2, 1, 0}, c[] = {1, 0, 1, 3, 2}, bad[] = {2, 0, 5, 1, 0};
    const double v[] = {1, 2, 3, 4, 5};
    int64_t rp[4];
    int32_t co[5];
    double vo[5];
    CHECK(oracle_coo_to_csr_f64(3, 4, 5, r, c, v, rp, co, vo) == 4);
    CHECK(rp[0] == 0 && rp[1] == 2 && rp[2] == 3 && rp[3] == 4 && vo[3] == 4.0);
    CHECK(oracle_coo_to_csr_f64(3, 4, 5, r, bad, v, rp, co, vo) == -1);
    CHECK(oracle_coo_to_csr_f64(3, 4, 0, r, c, v, rp, co, vo) == 0);
  }
  {  /* 1-D Laplacian, n = 50 */
    const int64_t n = 50;
    int64_t *rp = malloc((n + 1) * 8);
    int32_t *col = malloc(3 * n * 4);
    double *val = malloc(3 * n * 8), *b = malloc(n * 8), *x = calloc(n, 8), res = 0;
    int64_t k = 0;
    rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
      if (i > 0) col[k] = (int32_t)(i - 1), val[k++] = -1;
      col[k] = (int32_t)i, val[k++] = 2;
      if (i < n - 1) col[k] = (int32_t)(i + 1), val[k++] = -1;
      rp[i + 1] = k;
      b[i] = 1.0;
    }
    const int it = oracle_cg_f64(n, rp, 64, col, val, b, x, 1e-10, 200, &res);
    CHECK(it > 0 && it <= 200 && res <= 1e-10);
    free(rp), free(col), free(val), free(b), free(x);
  }
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("ALL OK (asan oracle)\n");
  return 0;
}
