// bench_kernels.cpp — the reference's per-kernel benchmark tables
// (benchmarks/benchmark_similarity_transform.cpp, published in
// benchmarks/similarity_transform.md) for this repository's kernels,
// through the step-level C-ABI on device-resident fp32 data, sizes 2^7..2^13.
//
// The reference times one SYCL kernel per table (row sums, max, eigenvector
// update, next matrix, stop test).  Here the round is fused differently, so
// the tables are:
//   whole solve            max_eigen_value (host matrix, H2D included)
//   row sums               st_rowsum      (N^2 read)
//   round epilogue         st_epilogue    (max + eigenvector update + stop
//                                          test + bookkeeping, one launch:
//                                          the reference's three small
//                                          kernels)
//   next matrix            st_scale_rowsum (D^-1 A D in place + its row sums)
//   whole round            st_round       (everything of one round, the
//                                          solve loop's only kernel)
// Kernel times are HIP-event medians over 20 launches on data already in
// HBM; the reference's row-sum table includes its lazy host->device copy
// (SURVEY.md §6), ours does not.
//
// Build: make -C tools bench_kernels    Run: ./tools/bench_kernels
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "similarity_transform.h"

#define HIPCHECK(x)                                                            \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   hipGetErrorString(e));                                      \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

#define STCHECK(x)                                                             \
  do {                                                                         \
    if ((x) < 0) {                                                             \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   eigen_last_error());                                        \
      std::exit(3);                                                            \
    }                                                                          \
  } while (0)

template <typename F>
static double
median_ms(F launch, int reps = 20)
{
  hipEvent_t a, b;
  HIPCHECK(hipEventCreate(&a));
  HIPCHECK(hipEventCreate(&b));
  launch();
  HIPCHECK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    HIPCHECK(hipEventRecord(a, nullptr));
    launch();
    HIPCHECK(hipEventRecord(b, nullptr));
    HIPCHECK(hipEventSynchronize(b));
    float ms;
    HIPCHECK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  HIPCHECK(hipEventDestroy(a));
  HIPCHECK(hipEventDestroy(b));
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

struct Sized
{
  unsigned n;
  float* a = nullptr;  // n x n, Hilbert
  float* s0 = nullptr; // row sums
  float* s1 = nullptr;
  float* v = nullptr;
  st_state* st = nullptr;
  explicit Sized(unsigned n_) : n(n_)
  {
    HIPCHECK(hipMalloc(&a, sizeof(float) * (size_t)n * n));
    HIPCHECK(hipMalloc(&s0, sizeof(float) * n));
    HIPCHECK(hipMalloc(&s1, sizeof(float) * n));
    HIPCHECK(hipMalloc(&v, sizeof(float) * n));
    HIPCHECK(hipMalloc(&st, sizeof(st_state)));
    STCHECK(st_generate_hilbert_f32(a, n, n, 0, nullptr));
    STCHECK(st_rowsum_f32(a, s0, n, n, nullptr));
    STCHECK(st_fill_f32(v, n, 1.0f, nullptr));
    HIPCHECK(hipDeviceSynchronize());
  }
  ~Sized()
  {
    (void)hipFree(a);
    (void)hipFree(s0);
    (void)hipFree(s1);
    (void)hipFree(v);
    (void)hipFree(st);
  }
};

int
main()
{
  void* q = nullptr;
  make_queue(&q);
  if (!q) {
    std::fprintf(stderr, "make_queue: %s\n", eigen_last_error());
    return 1;
  }
  std::printf("running on MI355X (gfx950), fp32, kernels on HBM-resident data\n\n");

  std::printf("Parallel Similarity Transform for finding max eigen value (with "
              "vector)\n\n");
  for (unsigned i = 7; i <= 13; i++) {
    const unsigned n = 1u << i;
    std::vector<float> m((size_t)n * n), vec(n);
    for (unsigned r = 0; r < n; r++)
      for (unsigned c = 0; c < n; c++)
        m[(size_t)r * n + c] = 1.0f / (float)(r + c + 1); // utils.cpp:150
    float val = 0;
    unsigned iters = 0;
    STCHECK(max_eigen_value(q, m.data(), &val, vec.data(), n, &iters)); // warm
    st_stats sts;
    STCHECK(max_eigen_value_ex(q, 0, m.data(), &val, vec.data(), n, &iters,
                               nullptr, &sts));
    std::printf("%-5u x %5u\t\t\t%10.3f ms\t\t\t%6u round(s)\n", n, n,
                sts.h2d_ms + sts.loop_ms, iters);
  }

  struct Table
  {
    const char* title;
    bool square;
  };
  const Table tables[] = {
    { "Parallel Sum Across Rows of Matrix", true },
    { "Round epilogue: max + eigen vector + stop test (one launch)", false },
    { "Parallel Next Matrix Computation (with its row sums)", true },
    { "Whole round (the solve loop's one launch)", true },
  };
  for (int t = 0; t < 4; t++) {
    std::printf("\n%s\n\n", tables[t].title);
    for (unsigned i = 7; i <= 13; i++) {
      const unsigned n = 1u << i;
      Sized z(n);
      double ms = 0;
      switch (t) {
        case 0:
          ms = median_ms([&] { STCHECK(st_rowsum_f32(z.a, z.s1, n, n, nullptr)); });
          break;
        case 1:
          STCHECK(st_state_reset(z.st, nullptr)); // eps = 0: never stops
          ms = median_ms([&] {
            STCHECK(st_epilogue_f32(z.s0, z.v, n, 0.0f, 1u << 30, ST_SEM_SYCL,
                                    z.st, nullptr));
          });
          break;
        case 2:
          ms = median_ms([&] {
            STCHECK(st_scale_rowsum_f32(z.a, z.s0, z.s1, n, n, 0, ST_SEM_SYCL,
                                        nullptr, nullptr));
          });
          break;
        default:
          STCHECK(st_state_reset(z.st, nullptr));
          ms = median_ms([&] {
            STCHECK(st_round_f32(z.a, z.s0, z.s1, z.v, n, n, 0, 0.0f, 0,
                                 1u << 30, ST_SEM_SYCL, z.st, nullptr));
          });
          break;
      }
      if (tables[t].square)
        std::printf("%-5u x %5u\t\t\t%10.4f ms\n", n, n, ms);
      else
        std::printf("%5u\t\t\t%10.4f ms\n", n, ms);
    }
  }
  destroy_queue(q);
  return 0;
}
