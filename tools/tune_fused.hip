// tune_fused.hip — launch-shape sweep of the fused scale+row-sum kernel
// (st_device.h) on one MI355X, plus two ceiling references measured on the
// same device: an in-place read+write stream (the same bytes as the fused
// kernel with no reduction) and a streaming read-only sum.
//
// Build: make -C tools   Run: ./tools/tune_fused [n] [reps]
// Output: one line per variant: ms per launch and GB/s of algorithmic
// bytes (2*n*n*b for the in-place kernels, n*n*b for read-only).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

// ceiling reference 1: in-place streaming scale, 16 B per lane, grid-stride
typedef double d2 __attribute__((ext_vector_type(2)));
template <bool NT>
__global__ __launch_bounds__(256) void
k_stream_rw(d2* __restrict__ a, size_t n2, double f)
{
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (size_t)gridDim.x * 256) {
    d2 x;
    if constexpr (NT)
      x = __builtin_nontemporal_load(a + i);
    else
      x = a[i];
    x *= f;
    if constexpr (NT)
      __builtin_nontemporal_store(x, a + i);
    else
      a[i] = x;
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void
k_stream_copy(const d2* __restrict__ a, d2* __restrict__ b, size_t n2, double f)
{
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (size_t)gridDim.x * 256) {
    d2 x;
    if constexpr (NT)
      x = __builtin_nontemporal_load(a + i);
    else
      x = a[i];
    x *= f;
    if constexpr (NT)
      __builtin_nontemporal_store(x, b + i);
    else
      b[i] = x;
  }
}

// ceiling reference 2: streaming read-only sum
__global__ __launch_bounds__(256) void
k_stream_r(const d2* __restrict__ a, size_t n2, double* out)
{
  double acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n2;
       i += (size_t)gridDim.x * 256) {
    d2 x = a[i];
    acc += x[0] + x[1];
  }
  if (acc == 123.456)
    out[0] = acc;
}

struct Timer
{
  hipEvent_t a, b;
  Timer()
  {
    HIPCHECK(hipEventCreate(&a));
    HIPCHECK(hipEventCreate(&b));
  }
  template <typename F>
  float run(F f, int reps)
  {
    f(); // warm
    HIPCHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
      HIPCHECK(hipEventRecord(a));
      f();
      HIPCHECK(hipEventRecord(b));
      HIPCHECK(hipEventSynchronize(b));
      float ms;
      HIPCHECK(hipEventElapsedTime(&ms, a, b));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  }
};

static double* g_a;
static double* g_b;
static double* g_s;
static double* g_sn;
static double* g_v;
static st_state* g_st;
static unsigned g_n;

template <int ROWS, int U, bool NT, int BLK>
void
fused_variant(Timer& tm, int reps, unsigned grid_cap = 0, bool oop = false)
{
  const unsigned ng = g_n / ROWS;
  const unsigned grid = grid_cap && grid_cap < ng ? grid_cap : ng;
  double* out = oop ? g_b : g_a;
  auto f = [&] {
    hipLaunchKernelGGL((k_fused<double, ROWS, 2, U, true, true, 0, NT, BLK>),
                       dim3(grid), dim3(BLK), 0, 0, g_a, out, g_s, g_sn, 0u, ng,
                       g_n, 0u, nullptr);
  };
  float ms = tm.run(f, reps);
  double gb = 2.0 * g_n * (double)g_n * 8 / (ms * 1e-3) / 1e9;
  std::printf("fused  rows=%d u=%d nt=%d blk=%4d grid=%6u oop=%d  %8.4f ms  %7.1f GB/s\n",
              ROWS, U, (int)NT, BLK, grid, (int)oop, ms, gb);
}

template <int ROWS, int U, bool NT, int BLK>
void
round_variant(Timer& tm, int reps, unsigned grid_cap)
{
  const unsigned ng = g_n / ROWS;
  const unsigned grid = grid_cap && grid_cap < ng ? grid_cap : ng;
  auto f = [&] {
    hipLaunchKernelGGL((k_round<double, ROWS, 2, U, 0, NT ? kNtBoth : kCached, BLK>), dim3(grid),
                       dim3(BLK), 0, 0, g_a, g_s, g_sn, g_v, ng, 0u, g_n, 0u,
                       0.0, 0u, 1u << 30, 0u, g_st);
  };
  float ms = tm.run(f, reps);
  double gb = 2.0 * g_n * (double)g_n * 8 / (ms * 1e-3) / 1e9;
  std::printf("round  rows=%d u=%d nt=%d blk=%4d grid=%6u        %8.4f ms  %7.1f GB/s\n",
              ROWS, U, (int)NT, BLK, grid, ms, gb);
}

static double* g_v2;

template <int ROWS, int U, bool NT, int BLK>
void
mfree_variant(Timer& tm, int reps, unsigned grid_cap)
{
  const unsigned ng = g_n / ROWS;
  const unsigned grid = grid_cap && grid_cap < ng ? grid_cap : ng;
  auto f = [&] {
    hipLaunchKernelGGL((k_mfree<double, ROWS, 2, U, NT, BLK>), dim3(grid),
                       dim3(BLK), 0, 0, g_a, g_s, g_sn, g_v, g_v2, ng, 0u, g_n,
                       0u, 0.0, 1u, 1u << 30, 0u, g_st);
  };
  float ms = tm.run(f, reps);
  double gb = 1.0 * g_n * (double)g_n * 8 / (ms * 1e-3) / 1e9;
  std::printf("mfree  rows=%d u=%d nt=%d blk=%4d grid=%6u        %8.4f ms  %7.1f GB/s\n",
              ROWS, U, (int)NT, BLK, grid, ms, gb);
}

template <int ROWS, int U, int BLK>
void
rowsum_variant(Timer& tm, int reps, unsigned grid_cap = 0)
{
  const unsigned ng = g_n / ROWS;
  const unsigned grid = grid_cap && grid_cap < ng ? grid_cap : ng;
  auto f = [&] {
    hipLaunchKernelGGL((k_fused<double, ROWS, 2, U, false, true, 0, false, BLK>),
                       dim3(grid), dim3(BLK), 0, 0, g_a, g_a, nullptr, g_sn, 0u,
                       ng, g_n, 0u, nullptr);
  };
  float ms = tm.run(f, reps);
  double gb = 1.0 * g_n * (double)g_n * 8 / (ms * 1e-3) / 1e9;
  std::printf("rowsum rows=%d u=%d blk=%4d grid=%6u        %8.4f ms  %7.1f GB/s\n",
              ROWS, U, BLK, grid, ms, gb);
}

int
main(int argc, char** argv)
{
  g_n = argc > 1 ? (unsigned)std::atoi(argv[1]) : 32768u;
  const int reps = argc > 2 ? std::atoi(argv[2]) : 20;
  const size_t nn = (size_t)g_n * g_n;
  HIPCHECK(hipMalloc(&g_a, nn * 8));
  HIPCHECK(hipMalloc(&g_b, nn * 8));
  HIPCHECK(hipMalloc(&g_s, (size_t)g_n * 8));
  HIPCHECK(hipMalloc(&g_sn, (size_t)g_n * 8));
  HIPCHECK(hipMalloc(&g_v, (size_t)g_n * 8));
  HIPCHECK(hipMalloc(&g_v2, (size_t)g_n * 8));
  HIPCHECK(hipMalloc(&g_st, sizeof(st_state)));
  HIPCHECK(hipMemset(g_st, 0, sizeof(st_state)));
  hipLaunchKernelGGL((k_generate<double, kRandom>), dim3(65536), dim3(256), 0,
                     0, g_a, g_n, g_n, 0u, 0ull);
  hipLaunchKernelGGL(k_fill<double>, dim3(256), dim3(256), 0, 0, g_s,
                     (uint64_t)g_n, 1.0);
  hipLaunchKernelGGL(k_fill<double>, dim3(256), dim3(256), 0, 0, g_v,
                     (uint64_t)g_n, 1.0);
  HIPCHECK(hipDeviceSynchronize());
  std::printf("n=%u  matrix %.2f GiB  reps=%d\n", g_n, nn * 8.0 / (1 << 30),
              reps);
  Timer tm;
  for (unsigned grid : { 1024u, 2048u, 4096u, 8192u }) {
    auto f = [&] {
      hipLaunchKernelGGL(k_stream_rw<false>, dim3(grid), dim3(256), 0, 0,
                         (d2*)g_a, nn / 2, 1.0);
    };
    float ms = tm.run(f, reps);
    std::printf("stream_rw grid=%5u          %8.4f ms  %7.1f GB/s\n", grid, ms,
                2.0 * nn * 8 / (ms * 1e-3) / 1e9);
    auto g = [&] {
      hipLaunchKernelGGL(k_stream_rw<true>, dim3(grid), dim3(256), 0, 0,
                         (d2*)g_a, nn / 2, 1.0);
    };
    ms = tm.run(g, reps);
    std::printf("stream_rw_nt grid=%5u       %8.4f ms  %7.1f GB/s\n", grid, ms,
                2.0 * nn * 8 / (ms * 1e-3) / 1e9);
    auto h = [&] {
      hipLaunchKernelGGL(k_stream_r, dim3(grid), dim3(256), 0, 0,
                         (const d2*)g_a, nn / 2, g_sn);
    };
    ms = tm.run(h, reps);
    std::printf("stream_r  grid=%5u          %8.4f ms  %7.1f GB/s\n", grid, ms,
                1.0 * nn * 8 / (ms * 1e-3) / 1e9);
  }
  for (unsigned grid : { 1024u, 2048u }) {
    auto f = [&] {
      hipLaunchKernelGGL(k_stream_copy<false>, dim3(grid), dim3(256), 0, 0,
                         (const d2*)g_a, (d2*)g_b, nn / 2, 1.0);
    };
    float ms = tm.run(f, reps);
    std::printf("stream_copy grid=%5u        %8.4f ms  %7.1f GB/s\n", grid, ms,
                2.0 * nn * 8 / (ms * 1e-3) / 1e9);
    auto g = [&] {
      hipLaunchKernelGGL(k_stream_copy<true>, dim3(grid), dim3(256), 0, 0,
                         (const d2*)g_a, (d2*)g_b, nn / 2, 1.0);
    };
    ms = tm.run(g, reps);
    std::printf("stream_copy_nt grid=%5u     %8.4f ms  %7.1f GB/s\n", grid, ms,
                2.0 * nn * 8 / (ms * 1e-3) / 1e9);
  }
  round_variant<2, 2, true, 256>(tm, reps, 256);
  mfree_variant<4, 2, true, 256>(tm, reps, 512);
  for (unsigned cap : { 256u, 512u, 1024u, 2048u }) {
    mfree_variant<1, 4, true, 256>(tm, reps, cap);
    mfree_variant<2, 4, true, 256>(tm, reps, cap);
    mfree_variant<4, 4, true, 256>(tm, reps, cap);
    mfree_variant<4, 2, true, 256>(tm, reps, cap);
    mfree_variant<2, 2, true, 256>(tm, reps, cap);
    mfree_variant<2, 8, true, 256>(tm, reps, cap);
    mfree_variant<2, 4, false, 256>(tm, reps, cap);
    mfree_variant<2, 4, true, 512>(tm, reps, cap);
  }
  for (unsigned cap : { 256u, 512u, 1024u }) {
    fused_variant<2, 4, true, 256>(tm, reps, cap);
    round_variant<1, 4, true, 256>(tm, reps, cap);
    round_variant<2, 2, true, 256>(tm, reps, cap);
    round_variant<2, 4, true, 256>(tm, reps, cap);
    round_variant<4, 2, true, 256>(tm, reps, cap);
    round_variant<4, 4, true, 256>(tm, reps, cap);
    round_variant<2, 4, false, 256>(tm, reps, cap);
    round_variant<2, 4, true, 512>(tm, reps, cap);
    round_variant<1, 8, true, 256>(tm, reps, cap);
  }
  rowsum_variant<1, 2, 256>(tm, reps);
  rowsum_variant<2, 4, 512>(tm, reps);
  rowsum_variant<2, 4, 256>(tm, reps, 1024);
  rowsum_variant<1, 4, 256>(tm, reps, 1024);
  HIPCHECK(hipFree(g_a));
  HIPCHECK(hipFree(g_b));
  HIPCHECK(hipFree(g_s));
  HIPCHECK(hipFree(g_sn));
  return 0;
}
