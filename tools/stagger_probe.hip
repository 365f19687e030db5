// stagger_probe.hip — does a staggered store pay?  (VERDICT r03 "next" #4)
//
// The deferred-write solve loop reads A every round and stores it every m-th
// round (m = 6): m - 1 read-only launches, then one launch that reads and
// writes all of A.  The storing launch runs below the read+write stream
// rate.  A staggered store would let row band b store on rounds k = b mod m
// instead, so every launch reads all of A and writes 1/m of it (the bytes
// of a cycle unchanged).  Before building that into k_flat (a launch whose
// workgroups carry different pending counts), this probe measures the
// memory side alone: the same bytes per cycle, with NO arithmetic beyond
// x * f, walked as k_flat walks them (one 256-thread workgroup per R rows of
// a 4 KB piece, 16 B per lane per row, pieces tiled by PT row groups,
// non-temporal loads and stores as on >= 2 GiB blocks):
//   seq        m - 1 read-only launches + 1 launch that stores every row
//   interleave m launches; row group g stores when (g + k) % m == 0
//   bands      m launches; the g-th of m contiguous row bands stores on k % m
// Read-only rows write one partial per workgroup and row (k_flat's part).
// Prints ms per round (cycle / m), the median of 7 passes of 4 cycles.
//
// Build: make -C tools stagger_probe
// Run:   ./tools/stagger_probe 32768x32768 8192x65536   (SP_M=6 SP_PT=4)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPCHECK(x)                                                            \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   hipGetErrorString(e));                                      \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

enum { kRead = 0, kStoreAll = 1, kInterleave = 2, kBands = 3 };

// one workgroup per R rows x 512 doubles (4 KB) of one piece
template <int R, int MODE>
__global__ __launch_bounds__(256) void
k_mix(double* a, double* part, unsigned nrows, unsigned ncols, unsigned pt,
      unsigned k, unsigned m, double f)
{
  const unsigned ppr = ncols / 512, ng = (nrows + R - 1) / R;
  const unsigned b = blockIdx.x;
  unsigned rg, p;
  if (pt > 1) {
    const unsigned tile = b / (pt * ppr), t = b - tile * (pt * ppr);
    const unsigned left = ng - tile * pt, g = left < pt ? left : pt;
    p = t / g;
    rg = tile * pt + (t - p * g);
  } else {
    rg = b / ppr;
    p = b - rg * ppr;
  }
  bool store;
  if constexpr (MODE == kRead)
    store = false;
  else if constexpr (MODE == kStoreAll)
    store = true;
  else if constexpr (MODE == kInterleave)
    store = (rg + k) % m == 0;
  else
    store = (unsigned)(((unsigned long long)rg * m) / ng) == k % m;
  d2 x[R];
  const size_t c = (size_t)p * 512 + 2 * threadIdx.x;
#pragma unroll
  for (int j = 0; j < R; j++) {
    const unsigned r = rg * R + j < nrows ? rg * R + j : nrows - 1;
    x[j] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(a + (size_t)r * ncols + c));
  }
  if (store) { // uniform per workgroup
#pragma unroll
    for (int j = 0; j < R; j++)
      if (rg * R + j < nrows)
        __builtin_nontemporal_store(x[j] * f,
                                    reinterpret_cast<d2*>(a + (size_t)(rg * R + j) * ncols + c));
  }
  // every row's partial sum (the round's row sums), one per workgroup and row
#pragma unroll
  for (int j = 0; j < R; j++) {
    double s = (x[j].x + x[j].y) * f;
    for (int o = 32; o >= 1; o >>= 1)
      s += __shfl_xor(s, o);
    __shared__ double red[R][4];
    if ((threadIdx.x & 63) == 0)
      red[j][threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0 && rg * R + j < nrows)
      part[(size_t)(rg * R + j) * ppr + p] = (red[j][0] + red[j][1]) + (red[j][2] + red[j][3]);
  }
}

__global__ void
k_fill(double* a, size_t n)
{
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (size_t)gridDim.x * 256) {
    unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    a[i] = 0.5 + (double)(z >> 11) * (1.0 / 9007199254740992.0);
  }
}

template <int R, int MODE>
static void
launch(double* a, double* part, unsigned nr, unsigned nc, unsigned pt, unsigned k,
       unsigned m, unsigned lds)
{
  const unsigned grid = ((nr + R - 1) / R) * (nc / 512);
  hipLaunchKernelGGL((k_mix<R, MODE>), dim3(grid), dim3(256), lds, 0, a, part, nr, nc, pt, k,
                     m, 1.0);
}

// one cycle of m rounds in the given form
template <int RR, int RS, int MODE>
static void
cycle(double* a, double* part, unsigned nr, unsigned nc, unsigned pt, unsigned m,
      unsigned cap_store)
{
  const unsigned lds = cap_store ? (160u << 10) / cap_store - 2048u : 0u;
  for (unsigned k = 0; k < m; k++) {
    if constexpr (MODE == kRead) { // "seq": read-only rounds, then the store
      if (k + 1 < m)
        launch<RR, kRead>(a, part, nr, nc, pt, k, m, 0);
      else
        launch<RS, kStoreAll>(a, part, nr, nc, pt, k, m, lds);
    } else {
      launch<RR, MODE>(a, part, nr, nc, pt, k, m, lds);
    }
  }
}

template <int RR, int RS, int MODE>
static float
timed(double* a, double* part, unsigned nr, unsigned nc, unsigned pt, unsigned m,
      unsigned cap)
{
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  cycle<RR, RS, MODE>(a, part, nr, nc, pt, m, cap); // warm-up
  std::vector<float> t;
  for (int rep = 0; rep < 7; rep++) {
    HIPCHECK(hipEventRecord(e0));
    for (int c = 0; c < 4; c++)
      cycle<RR, RS, MODE>(a, part, nr, nc, pt, m, cap);
    HIPCHECK(hipEventRecord(e1));
    HIPCHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms / (4 * m));
  }
  HIPCHECK(hipGetLastError());
  std::sort(t.begin(), t.end());
  HIPCHECK(hipEventDestroy(e0));
  HIPCHECK(hipEventDestroy(e1));
  return t[t.size() / 2];
}

int
main(int argc, char** argv)
{
  const unsigned m = std::getenv("SP_M") ? (unsigned)std::atoi(std::getenv("SP_M")) : 6u;
  const unsigned pt = std::getenv("SP_PT") ? (unsigned)std::atoi(std::getenv("SP_PT")) : 4u;
  for (int i = 1; i < argc; i++) {
    unsigned nr = 0, nc = 0;
    if (std::sscanf(argv[i], "%ux%u", &nr, &nc) != 2 || nc % 512 != 0 || nr < 8) {
      std::fprintf(stderr, "bad size %s (RxC, C a multiple of 512)\n", argv[i]);
      return 2;
    }
    const size_t n = (size_t)nr * nc;
    double *a = nullptr, *part = nullptr;
    HIPCHECK(hipMalloc(&a, n * sizeof(double)));
    HIPCHECK(hipMalloc(&part, (size_t)nr * (nc / 512) * sizeof(double)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, n);
    HIPCHECK(hipDeviceSynchronize());
    const double gb = n * sizeof(double) / 1e9, cyc = gb * (m + 1.0) / m;
    std::printf("%ux%u fp64 %.3f GB, m = %u, tiles of %u row groups; per round %.3f GB "
                "(read all, write 1/m)\n", nr, nc, gb, m, pt, cyc);
#define SP_RUN(RR, RS, MODE, CAP, NAME)                                        \
  {                                                                            \
    const float ms = timed<RR, RS, MODE>(a, part, nr, nc, pt, m, CAP);         \
    std::printf("  %-44s %8.4f ms/round  %7.1f GB/s\n", NAME, ms,              \
                cyc / (ms * 1e-3));                                            \
    std::fflush(stdout);                                                       \
  }
    SP_RUN(2, 2, kRead, 0, "seq: read R2, store R2");
    SP_RUN(4, 8, kRead, 0, "seq: read R4, store R8");
    SP_RUN(8, 8, kRead, 0, "seq: read R8, store R8");
    SP_RUN(8, 8, kRead, 3, "seq: read R8, store R8 capped 3/CU");
    SP_RUN(2, 8, kRead, 0, "seq: read R2, store R8");
    SP_RUN(2, 8, kRead, 3, "seq: read R2, store R8 capped 3/CU");
    SP_RUN(2, 2, kInterleave, 0, "interleave R2");
    SP_RUN(4, 4, kInterleave, 0, "interleave R4");
    SP_RUN(8, 8, kInterleave, 0, "interleave R8");
    SP_RUN(2, 2, kBands, 0, "bands R2");
    SP_RUN(4, 4, kBands, 0, "bands R4");
    SP_RUN(8, 8, kBands, 0, "bands R8");
    SP_RUN(8, 8, kBands, 3, "bands R8 capped 3/CU");
    SP_RUN(8, 8, kInterleave, 3, "interleave R8 capped 3/CU");
#undef SP_RUN
    // the pure streams for scale
    {
      hipEvent_t e0, e1;
      HIPCHECK(hipEventCreate(&e0));
      HIPCHECK(hipEventCreate(&e1));
      for (int mode = 0; mode < 4; mode++) {
        std::vector<float> t;
        for (int rep = 0; rep < 8; rep++) {
          HIPCHECK(hipEventRecord(e0));
          for (int j = 0; j < 8; j++) {
            if (mode == 0)
              launch<2, kRead>(a, part, nr, nc, pt, j, m, 0);
            else if (mode == 1)
              launch<2, kStoreAll>(a, part, nr, nc, pt, j, m, 0);
            else if (mode == 2)
              launch<8, kRead>(a, part, nr, nc, pt, j, m, 0);
            else
              launch<8, kStoreAll>(a, part, nr, nc, pt, j, m, 0);
          }
          HIPCHECK(hipEventRecord(e1));
          HIPCHECK(hipEventSynchronize(e1));
          float ms = 0;
          HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
          if (rep)
            t.push_back(ms / 8);
        }
        std::sort(t.begin(), t.end());
        const float ms = t[t.size() / 2];
        static const char* names[] = { "stream: read all, R2", "stream: read + write all, R2",
                                       "stream: read all, R8", "stream: read + write all, R8" };
        std::printf("  %-44s %8.4f ms/launch %7.1f GB/s\n", names[mode], ms,
                    (mode & 1 ? 2 : 1) * gb / (ms * 1e-3));
      }
      HIPCHECK(hipEventDestroy(e0));
      HIPCHECK(hipEventDestroy(e1));
    }
    HIPCHECK(hipFree(a));
    HIPCHECK(hipFree(part));
  }
  return 0;
}
