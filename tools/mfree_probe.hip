// mfree_probe.hip — launch shapes of the matrix-free round k_mfree
// (st_device.h) on one block: rows per group x chunks of 16 B per lane per
// row in flight (U) x workgroup cap, fp32 and fp64, non-temporal as the
// library's >= 512 MiB shape.  Median of 7 sequences of 8 launches
// (k = 1..8, stop never passes: eps = 0).
//
// Build: make -C tools mfree_probe   Run: ./tools/mfree_probe f32|f64 N ...
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "st_device.h"

using namespace st::dev;

#define HIPCHECK(x)                                                            \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   hipGetErrorString(e));                                      \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

template <typename T>
struct Buf
{
  T *a, *s0, *s1, *v0, *v1;
  st_state* st;
  uint32_t n;
};

template <typename T, int ROWS, int U>
static void
one(const Buf<T>& b, uint32_t cap)
{
  constexpr int W = 16 / sizeof(T);
  const uint32_t ng_main = b.n / ROWS, nrem = b.n % ROWS, ng = ng_main + nrem;
  const uint32_t grid = ng < cap ? ng : cap;
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  auto launch = [&](uint32_t k) {
    hipLaunchKernelGGL((k_mfree<T, ROWS, W, U, true, 256, true>), dim3(grid), dim3(256), 0, 0,
                       b.a, (k & 1) ? b.s1 : b.s0, (k & 1) ? b.s0 : b.s1,
                       (k & 1) ? b.v1 : b.v0, (k & 1) ? b.v0 : b.v1, ng_main, nrem, b.n,
                       0u, (T)0, k, 1u << 30, 0u, b.st);
  };
  for (uint32_t k = 1; k <= 8; k++)
    launch(k);
  std::vector<float> t;
  for (int r = 0; r < 7; r++) {
    HIPCHECK(hipEventRecord(e0));
    for (uint32_t k = 1; k <= 8; k++)
      launch(k);
    HIPCHECK(hipEventRecord(e1));
    HIPCHECK(hipEventSynchronize(e1));
    float ms;
    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms / 8);
  }
  std::sort(t.begin(), t.end());
  const double by = (double)b.n * b.n * sizeof(T);
  std::printf("  rows=%d U=%d cap=%4u  %8.4f ms  %7.1f GB/s\n", ROWS, U, cap, t[3],
              by / (t[3] * 1e-3) / 1e9);
  std::fflush(stdout);
  HIPCHECK(hipEventDestroy(e0));
  HIPCHECK(hipEventDestroy(e1));
}

template <typename T>
static void
run(uint32_t n)
{
  Buf<T> b{};
  b.n = n;
  HIPCHECK(hipMalloc(&b.a, sizeof(T) * (size_t)n * n));
  for (T** p : { &b.s0, &b.s1, &b.v0, &b.v1 })
    HIPCHECK(hipMalloc(p, sizeof(T) * n));
  HIPCHECK(hipMalloc(&b.st, sizeof(st_state)));
  HIPCHECK(hipMemset(b.st, 0, sizeof(st_state)));
  hipLaunchKernelGGL((k_generate<T, kRandom>), dim3(4096), dim3(256), 0, 0, b.a, n, n, 0u,
                     (uint64_t)7);
  std::vector<T> h(n, (T)1);
  for (T* p : { b.s0, b.s1, b.v0, b.v1 })
    HIPCHECK(hipMemcpy(p, h.data(), sizeof(T) * n, hipMemcpyHostToDevice));
  HIPCHECK(hipDeviceSynchronize());
  std::printf("%u^2 %s\n", n, sizeof(T) == 8 ? "f64" : "f32");
  for (uint32_t cap : { 256u, 512u, 1024u }) {
    one<T, 4, 2>(b, cap); // the library's shape (cap 512)
    one<T, 4, 4>(b, cap);
    one<T, 4, 8>(b, cap);
    one<T, 2, 4>(b, cap);
    one<T, 2, 8>(b, cap);
  }
  for (T* p : { b.a, b.s0, b.s1, b.v0, b.v1 })
    HIPCHECK(hipFree(p));
  HIPCHECK(hipFree(b.st));
}

int
main(int argc, char** argv)
{
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s f32|f64 N ...\n", argv[0]);
    return 1;
  }
  const bool f64 = std::strcmp(argv[1], "f64") == 0;
  for (int i = 2; i < argc; i++) {
    const unsigned n = (unsigned)std::atoi(argv[i]);
    if (n < 1024 || n % 16) {
      std::fprintf(stderr, "bad size %s\n", argv[i]);
      return 1;
    }
    if (f64)
      run<double>(n);
    else
      run<float>(n);
  }
  return 0;
}
