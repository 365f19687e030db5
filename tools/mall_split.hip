// mall_split.hip — can part of a block stay in the memory-side cache?
//
// A flat round over a block that is 1-4x the 256 MB memory-side cache
// (MALL) streams it with cached loads/stores and alternating piece order,
// which recovers only ~8 % over the non-temporal stream: as the round
// sweeps the block, the lines it touched first are evicted by the ones it
// touches later.  This probe splits every round into two k_flat launches
// over row ranges of one block: the first H rows with cached accesses (the
// part meant to stay resident) and the rest non-temporal (meant to pass by
// without evicting it), and times sequences of rounds for H = 0 ... N:
//   order 0  head then tail every round
//   order 1  head then tail on even rounds, tail then head on odd ones
// (FS = false: no stats, no k_parts; the row scales are 1, so the block's
// values stay put.)  Median of 7 sequences of 16 rounds.
//
// Build: make -C tools mall_split   Run: ./tools/mall_split f64 8192 [RxN ...]
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

constexpr int kSeq = 16;
constexpr int kReps = 7;

template <typename F>
static float
time_seq(F launch)
{
  hipEvent_t a, b;
  HIPCHECK(hipEventCreate(&a));
  HIPCHECK(hipEventCreate(&b));
  for (int k = 0; k < kSeq; k++)
    launch(k);
  HIPCHECK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < kReps; r++) {
    HIPCHECK(hipEventRecord(a));
    for (int k = 0; k < kSeq; k++)
      launch(k);
    HIPCHECK(hipEventRecord(b));
    HIPCHECK(hipEventSynchronize(b));
    float ms;
    HIPCHECK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms / kSeq);
  }
  HIPCHECK(hipEventDestroy(a));
  HIPCHECK(hipEventDestroy(b));
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

// one k_flat launch over rows [r0, r0 + nr) of an ncols-wide block
template <typename T, bool NT>
static void
part_round(T* a, const T* s, T* part, T* v, st_state* st, uint32_t r0, uint32_t nr,
           uint32_t ncols, uint32_t k)
{
  if (nr == 0)
    return;
  constexpr int W = 16 / sizeof(T);
  constexpr int U = (sizeof(T) == 8 && !NT) ? 2 : 1; // kFlatU (vector path)
  const uint32_t ppr = (ncols + 256 * W * U - 1) / (256 * W * U);
  const uint32_t grid = (nr + 1) / 2 * ppr;
  FlatPending<T, -1> pe{};
  pe.pt = NT ? 4u : 0u;
  hipLaunchKernelGGL((k_flat<T, W, 0, NT, 2, false, false, 2, 256, 0, kGatePlain, -1, U>),
                     dim3(grid), dim3(256), 0, 0, a + (size_t)r0 * ncols, s,
                     part + (size_t)r0 * ppr, v, nr, ncols, ppr, r0, k, st, (T)0,
                     1u << 30, 0u, 0u, 0u, 0u, pe, 0u);
}

template <typename T>
static void
run(uint32_t nr, uint32_t n)
{
  const size_t bytes = (size_t)nr * n * sizeof(T);
  T *a, *s, *part, *v;
  st_state* st;
  HIPCHECK(hipMalloc(&a, bytes));
  HIPCHECK(hipMalloc(&s, sizeof(T) * n));
  HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)nr * ((n + 255) / 256)));
  HIPCHECK(hipMalloc(&v, sizeof(T) * n));
  HIPCHECK(hipMalloc(&st, sizeof(st_state)));
  HIPCHECK(hipMemset(st, 0, sizeof(st_state)));
  hipLaunchKernelGGL((k_generate<T, kRandom>), dim3(4096), dim3(256), 0, 0, a, nr, n, 0u,
                     (uint64_t)7);
  std::vector<T> one(n, (T)1);
  HIPCHECK(hipMemcpy(s, one.data(), sizeof(T) * n, hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(v, one.data(), sizeof(T) * n, hipMemcpyHostToDevice));
  HIPCHECK(hipDeviceSynchronize());
  std::printf("%ux%u %s  %.1f MiB\n", nr, n, sizeof(T) == 8 ? "f64" : "f32",
              bytes / double(1 << 20));
  const double rb = 2.0 * bytes;
  for (int order = 0; order < 2; order++) {
    for (int eighth = 0; eighth <= 8; eighth++) {
      const uint32_t h = (uint32_t)((uint64_t)nr * eighth / 8) & ~1u;
      float ms = time_seq([&](int k) {
        const bool tail_first = order == 1 && (k & 1);
        if (tail_first) {
          part_round<T, true>(a, s, part, v, st, h, nr - h, n, k);
          part_round<T, false>(a, s, part, v, st, 0, h, n, k);
        } else {
          part_round<T, false>(a, s, part, v, st, 0, h, n, k);
          part_round<T, true>(a, s, part, v, st, h, nr - h, n, k);
        }
      });
      std::printf("  order=%d cached head %5u rows (%6.1f MiB)  %8.4f ms  %7.1f GB/s\n", order,
                  h, (double)h * n * sizeof(T) / (1 << 20), ms, rb / (ms * 1e-3) / 1e9);
      std::fflush(stdout);
    }
  }
  HIPCHECK(hipFree(a));
  HIPCHECK(hipFree(s));
  HIPCHECK(hipFree(part));
  HIPCHECK(hipFree(v));
  HIPCHECK(hipFree(st));
}

int
main(int argc, char** argv)
{
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s f64|f32 N|RxN ...\n", argv[0]);
    return 1;
  }
  const bool f64 = std::strcmp(argv[1], "f64") == 0;
  for (int i = 2; i < argc; i++) {
    unsigned nr = 0, n = 0;
    if (std::sscanf(argv[i], "%ux%u", &nr, &n) != 2) {
      n = (unsigned)std::atoi(argv[i]);
      nr = n;
    }
    if (nr < 2 || n == 0 || nr > n || n % 4) {
      std::fprintf(stderr, "bad size %s\n", argv[i]);
      return 1;
    }
    if (f64)
      run<double>(nr, n);
    else
      run<float>(nr, n);
  }
  return 0;
}
