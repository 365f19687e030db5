/*
 * st_oracle.c — CPU restatement of the reference's similarity-transform
 * max-eigenvalue iteration.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker (or the timed CPU baseline).
 * The product path (eigen_value_amd/, libsimilarity_transform.so) never
 * links or calls it.
 *
 * What it restates (citations are /root/reference/<file>:<line>):
 *   - sum_across_rows      similarity_transform.cpp:77-152, main.py:19-22
 *   - find_max (init 0.f)  similarity_transform.cpp:154-227 (line 185)
 *   - compute_eigen_vector similarity_transform.cpp:229-265 (line 260),
 *                          main.py:38-39
 *   - stop (cyclic)        similarity_transform.cpp:332-460 (lines 413-421)
 *   - stop (non-cyclic)    main.py:25-27
 *   - compute_next_matrix  similarity_transform.cpp:286-330 (lines 324-325):
 *                          A[r][c] *= (1/s[r]) * s[c]
 *   - compute_next         main.py:13-16: diag(1/s) @ A @ diag(s), i.e.
 *                          ((1/s[r]) * A[r][c]) * s[c] element-wise (the
 *                          zero terms of the diagonal products are exact)
 *   - round loop           similarity_transform.cpp:34-66, main.py:30-47
 *   - generate_hilbert     utils.cpp:137-154 (1/(r+c+1), line 150)
 *   - EPS, MAX_ITR         include/similarity_transform.hpp:4-5, main.py:6
 *
 * Row sums use numpy's summation order (0 + pairwise(buffer) for each
 * 8192-element buffer, 8-way unrolled leaves of <= 128 elements), so that in SEM_MAINPY mode the
 * fp64 solve is bit-identical to the reference's main.py (pinned by
 * tests/golden/).  The SYCL path sums with non-deterministic float atomics
 * (similarity_transform.cpp:124-147), so its bits cannot be pinned; the
 * SYCL-semantics mode is pinned by the reference's own known answers
 * (tests/test.cpp:99-102, README.md:70-76 round counts).
 *
 * Rows are processed in parallel with OpenMP when nthreads > 1; the
 * per-row summation order does not depend on the thread count.
 *
 * Build: see oracle/Makefile (gcc -O3 -fopenmp -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_PW_BLOCK 128
/* numpy's reduction visits a contiguous row in buffers of NPY_BUFSIZE
 * elements and adds each buffer's pairwise sum to the running result */
#define ORC_NPY_BUFSIZE 8192

enum
{
  ORC_SEM_SYCL = 0,   /* cyclic stop, A*((1/s_r)*s_c), count = break index */
  ORC_SEM_MAINPY = 1  /* non-cyclic stop, ((1/s_r)*A)*s_c, count = itr + 1  */
};

/* ----------------------------------------------------------------------- */
/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src)       */
/* ----------------------------------------------------------------------- */
#define DEFINE_PAIRWISE(T, NAME)                                              \
  static T NAME##_rec(const T* a, int64_t n)                                  \
  {                                                                           \
    if (n < 8) {                                                              \
      T res = (T)0;                                                           \
      for (int64_t i = 0; i < n; i++)                                         \
        res += a[i];                                                          \
      return res;                                                             \
    } else if (n <= ORC_PW_BLOCK) {                                           \
      T r[8];                                                                 \
      for (int j = 0; j < 8; j++)                                             \
        r[j] = a[j];                                                          \
      int64_t i;                                                              \
      for (i = 8; i < n - (n % 8); i += 8)                                    \
        for (int j = 0; j < 8; j++)                                           \
          r[j] += a[i + j];                                                   \
      T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7])); \
      for (; i < n; i++)                                                      \
        res += a[i];                                                          \
      return res;                                                             \
    } else {                                                                  \
      int64_t n2 = n / 2;                                                     \
      n2 -= n2 % 8;                                                           \
      return NAME##_rec(a, n2) + NAME##_rec(a + n2, n - n2);                  \
    }                                                                         \
  }                                                                           \
  T NAME(const T* a, int64_t n)                                               \
  {                                                                           \
    T res = (T)0;                                                             \
    for (int64_t i = 0; i < n; i += ORC_NPY_BUFSIZE)                          \
      res += NAME##_rec(a + i, n - i < ORC_NPY_BUFSIZE ? n - i : ORC_NPY_BUFSIZE); \
    return res;                                                               \
  }

DEFINE_PAIRWISE(double, orc_pairwise_sum_f64)
DEFINE_PAIRWISE(float, orc_pairwise_sum_f32)

/* ----------------------------------------------------------------------- */
/* input generators                                                        */
/* ----------------------------------------------------------------------- */

/* utils.cpp:150 — A[r][c] = 1/(r+c+1), rows [row0, row0+nrows) */
void
orc_hilbert_f64(double* m, uint32_t nrows, uint32_t ncols, uint32_t row0)
{
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < (int64_t)nrows; r++)
    for (uint32_t c = 0; c < ncols; c++)
      m[r * (int64_t)ncols + c] = 1.0 / (double)((uint64_t)row0 + r + c + 1);
}

void
orc_hilbert_f32(float* m, uint32_t nrows, uint32_t ncols, uint32_t row0)
{
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < (int64_t)nrows; r++)
    for (uint32_t c = 0; c < ncols; c++)
      m[r * (int64_t)ncols + c] = 1.f / (float)((uint64_t)row0 + r + c + 1);
}

/* Seeded counter hash replacing utils.cpp:125-134 (std::random_device,
 * non-reproducible).  splitmix64 of (seed, global element index); the same
 * bits are produced by the HIP generator and by oracle.py's numpy form. */
static inline uint64_t
orc_splitmix(uint64_t seed, uint64_t idx)
{
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

/* U(0,1] fp64: ((z >> 11) + 1) * 2^-53 */
void
orc_random_f64(double* m, uint32_t nrows, uint32_t ncols, uint32_t row0,
               uint64_t seed)
{
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < (int64_t)nrows; r++)
    for (uint32_t c = 0; c < ncols; c++) {
      uint64_t idx = ((uint64_t)row0 + r) * ncols + c;
      m[r * (int64_t)ncols + c] =
        (double)((orc_splitmix(seed, idx) >> 11) + 1) * 0x1.0p-53;
    }
}

/* U(0,1] fp32: ((z >> 40) + 1) * 2^-24 */
void
orc_random_f32(float* m, uint32_t nrows, uint32_t ncols, uint32_t row0,
               uint64_t seed)
{
#pragma omp parallel for schedule(static)
  for (int64_t r = 0; r < (int64_t)nrows; r++)
    for (uint32_t c = 0; c < ncols; c++) {
      uint64_t idx = ((uint64_t)row0 + r) * ncols + c;
      m[r * (int64_t)ncols + c] =
        (float)((orc_splitmix(seed, idx) >> 40) + 1) * 0x1.0p-24f;
    }
}

/* ----------------------------------------------------------------------- */
/* per-kernel restatements (templated by macro over the element type)       */
/* ----------------------------------------------------------------------- */
#define DEFINE_KERNELS(T, SFX)                                                \
  /* similarity_transform.cpp:77-152 / main.py:19-22 */                        \
  void orc_rowsum_##SFX(const T* m, T* s, uint32_t nrows, uint32_t ncols)     \
  {                                                                           \
    _Pragma("omp parallel for schedule(static)")                              \
    for (int64_t r = 0; r < (int64_t)nrows; r++)                              \
      s[r] = orc_pairwise_sum_##SFX(m + r * (int64_t)ncols, ncols);           \
  }                                                                           \
  /* similarity_transform.cpp:154-227: running max initialised to 0 (185) */  \
  T orc_find_max_##SFX(const T* s, uint32_t n)                                \
  {                                                                           \
    T mx = (T)0;                                                              \
    for (uint32_t i = 0; i < n; i++)                                          \
      mx = s[i] > mx ? s[i] : mx;                                             \
    return mx;                                                                \
  }                                                                           \
  /* similarity_transform.cpp:260, main.py:38-39: v[r] *= s[r] / m */         \
  void orc_compute_eigen_vector_##SFX(const T* s, T m, T* v, uint32_t n)      \
  {                                                                           \
    for (uint32_t i = 0; i < n; i++)                                          \
      v[i] = v[i] * (s[i] / m);                                               \
  }                                                                           \
  /* cyclic: similarity_transform.cpp:413-421; non-cyclic: main.py:25-27 */   \
  int orc_stop_##SFX(const T* s, uint32_t n, T eps, int cyclic)               \
  {                                                                           \
    uint32_t last = cyclic ? n : (n ? n - 1 : 0);                             \
    for (uint32_t i = 0; i < last; i++) {                                     \
      T d = s[i] - s[(i + 1) % n];                                            \
      if (!(fabs((double)d) < (double)eps))                                   \
        return 0;                                                             \
    }                                                                         \
    return 1;                                                                 \
  }                                                                           \
  /* order 0 (SYCL, similarity_transform.cpp:324-325): A *= (1/s_r)*s_c      \
   * order 1 (main.py:13-16):                       A = ((1/s_r)*A)*s_c      \
   * s_full is indexed by GLOBAL row/column; rows [row0, row0+nrows). */      \
  void orc_compute_next_##SFX(T* m, const T* s_full, uint32_t nrows,          \
                              uint32_t ncols, uint32_t row0, int order)       \
  {                                                                           \
    _Pragma("omp parallel for schedule(static)")                              \
    for (int64_t r = 0; r < (int64_t)nrows; r++) {                            \
      const T inv = (T)1 / s_full[row0 + r];                                  \
      T* row = m + r * (int64_t)ncols;                                        \
      if (order == 0) {                                                       \
        for (uint32_t c = 0; c < ncols; c++)                                  \
          row[c] = row[c] * (inv * s_full[c]);                                \
      } else {                                                                \
        for (uint32_t c = 0; c < ncols; c++)                                  \
          row[c] = (inv * row[c]) * s_full[c];                                \
      }                                                                       \
    }                                                                         \
  }

DEFINE_KERNELS(double, f64)
DEFINE_KERNELS(float, f32)

/* ----------------------------------------------------------------------- */
/* whole solve — similarity_transform.cpp:5-75 / main.py:30-47              */
/* ----------------------------------------------------------------------- */
static double
orc_now_ms(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e3 + (double)ts.tv_nsec * 1e-6;
}

/*
 * Returns 0 on success, -1 on bad arguments / allocation failure.
 * semantics: ORC_SEM_SYCL or ORC_SEM_MAINPY.
 * nthreads  : OpenMP threads (<= 0: leave the runtime default).
 * max_dsum  : optional [max_itr] array, per evaluated round max|s_i - s_i+1|
 *             over the pairs the stop test inspects (NULL to skip).
 * loop_ms   : optional; wall time of the round loop (the reference's `ts`
 *             region, similarity_transform.cpp:36-58).
 * rounds_evaluated: optional; number of row-sum evaluations performed.
 */
#define DEFINE_SOLVE(T, SFX)                                                  \
  static int orc_solve_##SFX(const T* mat, uint32_t n, T eps,                 \
                             uint32_t max_itr, int semantics, int nthreads,   \
                             T* eigen_val, T* eigen_vec,                      \
                             uint32_t* iter_count, double* max_dsum,          \
                             double* loop_ms, uint32_t* rounds_evaluated,     \
                             T* s_trace)                                      \
  {                                                                           \
    if (n == 0 || !mat || !eigen_val || !eigen_vec || !iter_count)            \
      return -1;                                                              \
    if (nthreads > 0)                                                         \
      omp_set_num_threads(nthreads);                                          \
    const size_t nn = (size_t)n * n;                                          \
    T* a = (T*)malloc(sizeof(T) * nn); /* private copy: cpp:14,19 */          \
    T* s = (T*)malloc(sizeof(T) * n);                                         \
    if (!a || !s) {                                                           \
      free(a);                                                                \
      free(s);                                                                \
      return -1;                                                              \
    }                                                                         \
    memcpy(a, mat, sizeof(T) * nn);                                           \
    const int cyclic = semantics == ORC_SEM_SYCL;                             \
    const int order = semantics == ORC_SEM_SYCL ? 0 : 1;                      \
    for (uint32_t i = 0; i < n; i++)                                          \
      eigen_vec[i] = (T)1; /* initialise_eigen_vector, cpp:34 */              \
    double t0 = orc_now_ms();                                                 \
    uint32_t i = 0, evals = 0;                                                \
    for (; i < max_itr; i++) {                                                \
      orc_rowsum_##SFX(a, s, n, n);                                           \
      evals++;                                                                \
      if (s_trace)                                                            \
        memcpy(s_trace + (size_t)i * n, s, sizeof(T) * n);                    \
      T mx = orc_find_max_##SFX(s, n);                                        \
      orc_compute_eigen_vector_##SFX(s, mx, eigen_vec, n);                    \
      if (max_dsum) {                                                         \
        double d = 0.0;                                                       \
        uint32_t last = cyclic ? n : n - 1;                                   \
        for (uint32_t k = 0; k < last; k++) {                                 \
          double e = fabs((double)(s[k] - s[(k + 1) % n]));                   \
          d = e > d ? e : d;                                                  \
        }                                                                     \
        max_dsum[i] = d;                                                      \
      }                                                                       \
      *eigen_val = s[0];                                                      \
      if (orc_stop_##SFX(s, n, eps, cyclic))                                  \
        break;                                                                \
      orc_compute_next_##SFX(a, s, n, n, 0, order);                           \
    }                                                                         \
    double t1 = orc_now_ms();                                                 \
    /* SYCL: iter_count = break index (cpp:54); main.py returns itr + 1 */    \
    *iter_count = semantics == ORC_SEM_SYCL ? i : (i < max_itr ? i + 1 : i);  \
    if (loop_ms)                                                              \
      *loop_ms = t1 - t0;                                                     \
    if (rounds_evaluated)                                                     \
      *rounds_evaluated = evals;                                              \
    free(a);                                                                  \
    free(s);                                                                  \
    return 0;                                                                 \
  }                                                                           \
  int orc_similarity_transform_##SFX(const T* mat, uint32_t n, T eps,         \
                                     uint32_t max_itr, int semantics,         \
                                     int nthreads, T* eigen_val,              \
                                     T* eigen_vec, uint32_t* iter_count,      \
                                     double* max_dsum, double* loop_ms,       \
                                     uint32_t* rounds_evaluated)              \
  {                                                                           \
    return orc_solve_##SFX(mat, n, eps, max_itr, semantics, nthreads,         \
                           eigen_val, eigen_vec, iter_count, max_dsum,        \
                           loop_ms, rounds_evaluated, NULL);                  \
  }                                                                           \
  /* the same solve, also writing s_k of every evaluated round k into         \
   * s_trace[k * n .. (k + 1) * n) ([max_itr * n]): the vectors the stop test  \
   * compared, for checking a device solve's per-round decisions */           \
  int orc_similarity_transform_trace_##SFX(                                   \
    const T* mat, uint32_t n, T eps, uint32_t max_itr, int semantics,         \
    int nthreads, T* eigen_val, T* eigen_vec, uint32_t* iter_count,           \
    double* max_dsum, double* loop_ms, uint32_t* rounds_evaluated,            \
    T* s_trace)                                                               \
  {                                                                           \
    return orc_solve_##SFX(mat, n, eps, max_itr, semantics, nthreads,         \
                           eigen_val, eigen_vec, iter_count, max_dsum,        \
                           loop_ms, rounds_evaluated, s_trace);               \
  }

/*
 * Streaming form of the same loop for a GENERATED input too large to keep
 * twice on the host (configs[3]: 65536^2 fp64 = 32 GiB): A_0 is never
 * stored; round k regenerates it in blocks of chunk_rows rows, re-applies the
 * k recorded transforms row by row with exactly orc_compute_next's
 * operations, (1/s_i[r]) then x*(inv*s_i[c]) (or (inv*x)*s_i[c]), oldest
 * first, and sums each row with orc_pairwise_sum.  Every element sees the
 * same operations in the same order as in orc_similarity_transform and a
 * row's sum depends on that row only, so the results are bit-identical to
 * it (checked in tests/test_oracle.py); the cost is O(k) passes in round k,
 * fine for the few rounds random inputs take.  kind 1 = Hilbert, 2 =
 * seeded random.  max_itr bounds the s history (max_itr * n elements).
 */
#define DEFINE_SOLVE_GEN(T, SFX)                                              \
  int orc_similarity_transform_gen_##SFX(                                     \
    int kind, uint64_t seed, uint32_t n, T eps, uint32_t max_itr,             \
    int semantics, int nthreads, uint32_t chunk_rows, T* eigen_val,           \
    T* eigen_vec, uint32_t* iter_count, double* loop_ms,                      \
    uint32_t* rounds_evaluated)                                               \
  {                                                                           \
    if (n == 0 || max_itr == 0 || (kind != 1 && kind != 2) || !eigen_val ||   \
        !eigen_vec || !iter_count)                                            \
      return -1;                                                              \
    if (nthreads > 0)                                                         \
      omp_set_num_threads(nthreads);                                          \
    if (chunk_rows == 0 || chunk_rows > n)                                    \
      chunk_rows = n;                                                         \
    T* hist = (T*)malloc(sizeof(T) * (size_t)max_itr * n); /* s_0..s_k */     \
    T* blk = (T*)malloc(sizeof(T) * (size_t)chunk_rows * n);                  \
    if (!hist || !blk) {                                                      \
      free(hist);                                                             \
      free(blk);                                                              \
      return -1;                                                              \
    }                                                                         \
    const int cyclic = semantics == ORC_SEM_SYCL;                             \
    const int order = semantics == ORC_SEM_SYCL ? 0 : 1;                      \
    for (uint32_t i = 0; i < n; i++)                                          \
      eigen_vec[i] = (T)1;                                                    \
    double t0 = orc_now_ms();                                                 \
    uint32_t i = 0, evals = 0;                                                \
    for (; i < max_itr; i++) {                                                \
      T* s = hist + (size_t)i * n;                                            \
      for (uint32_t r0 = 0; r0 < n; r0 += chunk_rows) {                       \
        const uint32_t nr = n - r0 < chunk_rows ? n - r0 : chunk_rows;        \
        if (kind == 1)                                                        \
          orc_hilbert_##SFX(blk, nr, n, r0);                                  \
        else                                                                  \
          orc_random_##SFX(blk, nr, n, r0, seed);                             \
        for (uint32_t j = 0; j < i; j++)                                      \
          orc_compute_next_##SFX(blk, hist + (size_t)j * n, nr, n, r0,        \
                                 order);                                      \
        orc_rowsum_##SFX(blk, s + r0, nr, n);                                 \
      }                                                                       \
      evals++;                                                                \
      T mx = orc_find_max_##SFX(s, n);                                        \
      orc_compute_eigen_vector_##SFX(s, mx, eigen_vec, n);                    \
      *eigen_val = s[0];                                                      \
      if (orc_stop_##SFX(s, n, eps, cyclic))                                  \
        break;                                                                \
    }                                                                         \
    double t1 = orc_now_ms();                                                 \
    *iter_count = semantics == ORC_SEM_SYCL ? i : (i < max_itr ? i + 1 : i);  \
    if (loop_ms)                                                              \
      *loop_ms = t1 - t0;                                                     \
    if (rounds_evaluated)                                                     \
      *rounds_evaluated = evals;                                              \
    free(hist);                                                               \
    free(blk);                                                                \
    return 0;                                                                 \
  }

#ifndef _OPENMP
static void
omp_set_num_threads(int n)
{
  (void)n;
}
#endif

DEFINE_SOLVE(double, f64)
DEFINE_SOLVE(float, f32)
DEFINE_SOLVE_GEN(double, f64)
DEFINE_SOLVE_GEN(float, f32)

int
orc_max_threads(void)
{
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
