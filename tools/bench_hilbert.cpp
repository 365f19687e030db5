// bench_hilbert.cpp — the reference's whole-solve Hilbert benchmark
// (main.cpp:23-35 + benchmarks/benchmark_similarity_transform.cpp:3-22),
// driven through this repository's drop-in C-ABI (max_eigen_value /
// max_eigen_value_f64): host Hilbert matrix 2^7 .. 2^13, one call per size,
// printed in the reference's table format, plus a JSON line per size with
// the device-side split (H2D, round loop) from max_eigen_value_ex.
//
// Build: make -C tools bench_hilbert    Run: ./tools/bench_hilbert [f32|f64]
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "similarity_transform.h"

template <typename T>
static void
hilbert(std::vector<T>& m, unsigned n)
{
  m.resize((size_t)n * n);
  for (unsigned r = 0; r < n; r++)
    for (unsigned c = 0; c < n; c++)
      m[(size_t)r * n + c] = (T)1 / (T)(r + c + 1); // utils.cpp:150
}

template <typename T>
static int
run(void* q, int dtype)
{
  std::printf("Parallel Similarity Transform for finding max eigen value (with "
              "vector) — %s, MI355X\n\n",
              dtype ? "fp64" : "fp32");
  for (unsigned i = 7; i <= 13; i++) {
    const unsigned n = 1u << i;
    std::vector<T> mat, vec(n);
    hilbert(mat, n);
    T val = 0;
    unsigned iters = 0;
    // warm the context's cached buffers for this size, then time
    st_stats st;
    if (max_eigen_value_ex(q, dtype, mat.data(), &val, vec.data(), n, &iters,
                           nullptr, &st) < 0) {
      std::fprintf(stderr, "failed: %s\n", eigen_last_error());
      return 1;
    }
    int64_t ts = dtype ? max_eigen_value_f64(q, (double*)mat.data(),
                                             (double*)&val, (double*)vec.data(),
                                             n, &iters)
                       : max_eigen_value(q, (float*)mat.data(), (float*)&val,
                                         (float*)vec.data(), n, &iters);
    if (max_eigen_value_ex(q, dtype, mat.data(), &val, vec.data(), n, &iters,
                           nullptr, &st) < 0 || ts < 0) {
      std::fprintf(stderr, "failed: %s\n", eigen_last_error());
      return 1;
    }
    std::printf("%-5u x %5u\t\t\t%10lld ms\t\t\t%6u round(s)\n", n, n,
                (long long)ts, iters);
    std::fprintf(stderr,
                 "{\"n\": %u, \"dtype\": \"%s\", \"ts_ms\": %lld, "
                 "\"iter_count\": %u, \"eigen_val\": %.17g, \"h2d_ms\": %.4f, "
                 "\"loop_ms\": %.4f, \"rounds\": %u}\n",
                 n, dtype ? "f64" : "f32", (long long)ts, iters, (double)val,
                 st.h2d_ms, st.loop_ms, st.rounds);
  }
  return 0;
}

int
main(int argc, char** argv)
{
  const bool f64 = argc > 1 && std::strcmp(argv[1], "f64") == 0;
  void* q = nullptr;
  make_queue(&q);
  if (!q) {
    std::fprintf(stderr, "make_queue failed: %s\n", eigen_last_error());
    return 1;
  }
  const int rc = f64 ? run<double>(q, 1) : run<float>(q, 0);
  destroy_queue(q);
  return rc;
}
