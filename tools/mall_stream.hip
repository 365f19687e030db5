// mall_stream.hip — the memory ceiling of the flat round's access pattern.
//
// k_flat's every-round launch on a cached fp64 block (configs[1], 8192^2
// fp64 = 512 MiB, about twice the 256 MB memory-side cache) reads and
// rewrites every 8 KB row piece once per round, in tiles of PT rows per
// piece, with the odd rounds walking the workgroups backwards in steps of 8
// (flat_reverse<2>: every piece stays on its XCD).  This probe runs exactly
// that walk with NO arithmetic beyond x * 1.0 (values unchanged, so the
// data stays the random fp64 it starts as: the cache's rate depends on the
// values) and the loads' / stores' cache policy chosen
// apart, so the round's time can be set against the pattern's own ceiling.
//   MODE rw: in place, read + write (the every-round launch)
//   MODE r:  read only, one partial sum per workgroup (the deferred rounds)
// Median of 7 sequences of 16 rounds (k = 0..15, so the reversal alternates).
//
// Build: make -C tools mall_stream
// Run:   ./tools/mall_stream 8192x8192 6144x6144 32768x32768  (MS_PT=8: tile rows)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <bool NT>
__device__ __forceinline__ d2
ld2(const d2* p)
{
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

template <bool NT>
__device__ __forceinline__ void
st2(d2* p, d2 x)
{
  if constexpr (NT)
    __builtin_nontemporal_store(x, p);
  else
    *p = x;
}

// one 256-thread workgroup per 8 KB piece of one row (two 16 B accesses per
// lane, 4 KB apart), pieces walked in tiles of pt rows (k_flat's map)
template <bool LNT, bool SNT, bool RW>
__global__ __launch_bounds__(256) void
k_walk(double* a, double* part, unsigned nrows, unsigned ppr, unsigned pt,
       unsigned k, double f)
{
  const unsigned nb = gridDim.x;
  unsigned b = blockIdx.x;
  if (k & 1u) {
    const unsigned g8 = nb & ~7u;
    b = b < g8 ? g8 - 8 - (b & ~7u) + (b & 7u) : b;
  }
  unsigned r, p;
  if (pt > 1) {
    const unsigned tile = b / (pt * ppr), t = b - tile * (pt * ppr);
    const unsigned left = nrows - tile * pt, g = left < pt ? left : pt;
    p = t / g;
    r = tile * pt + (t - p * g);
  } else {
    r = b / ppr;
    p = b - r * ppr;
  }
  d2* row = reinterpret_cast<d2*>(a + (size_t)r * ppr * 1024u + (size_t)p * 1024u);
  d2 x0 = ld2<LNT>(row + threadIdx.x);
  d2 x1 = ld2<LNT>(row + 256 + threadIdx.x);
  if constexpr (RW) {
    st2<SNT>(row + threadIdx.x, x0 * f);
    st2<SNT>(row + 256 + threadIdx.x, x1 * f);
  } else {
    const double s = x0.x + x0.y + x1.x + x1.y;
    if (s == -1.0) // never: keeps the loads live without a reduction
      part[b] = s;
  }
}

// the walk with k_flat's reduction after the loads: RED = 1 sums the lane's
// values, reduces each wave (xor shuffles) and the workgroup's 4 waves
// through LDS behind a barrier, one partial per piece (k_flat's shape);
// RED = 2 stores one partial per wave, no barrier (k_flat's PW variant)
template <int RED>
__global__ __launch_bounds__(256) void
k_walk_red(double* a, double* part, unsigned nrows, unsigned ppr, unsigned pt,
           unsigned k, double f)
{
  const unsigned nb = gridDim.x;
  unsigned b = blockIdx.x;
  if (k & 1u) {
    const unsigned g8 = nb & ~7u;
    b = b < g8 ? g8 - 8 - (b & ~7u) + (b & 7u) : b;
  }
  const unsigned tile = b / (pt * ppr), t = b - tile * (pt * ppr);
  const unsigned left = nrows - tile * pt, g = left < pt ? left : pt;
  const unsigned p = t / g, r = tile * pt + (t - p * g);
  d2* row = reinterpret_cast<d2*>(a + (size_t)r * ppr * 1024u + (size_t)p * 1024u);
  d2 x0 = ld2<false>(row + threadIdx.x);
  d2 x1 = ld2<false>(row + 256 + threadIdx.x);
  x0 *= f;
  x1 *= f;
  st2<true>(row + threadIdx.x, x0);
  st2<true>(row + 256 + threadIdx.x, x1);
  double s = (x0.x + x0.y) + (x1.x + x1.y);
  for (int o = 32; o >= 1; o >>= 1)
    s += __shfl_xor(s, o);
  const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if constexpr (RED == 2) {
    if (lane == 0)
      part[(size_t)b * 4 + wave] = s;
  } else {
    __shared__ double red[4];
    if (lane == 0)
      red[wave] = s;
    __syncthreads();
    if (threadIdx.x == 0)
      part[b] = (red[0] + red[1]) + (red[2] + red[3]);
  }
}

template <int RED>
static float
run_red(double* a, double* part, unsigned nrows, unsigned ppr, unsigned pt,
        unsigned lds)
{
  const unsigned grid = nrows * ppr;
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  for (unsigned k = 0; k < 16; k++)
    hipLaunchKernelGGL((k_walk_red<RED>), dim3(grid), dim3(256), lds, 0, a, part,
                       nrows, ppr, pt, k, 1.0);
  std::vector<float> t;
  for (int rep = 0; rep < 7; rep++) {
    HIPCHECK(hipEventRecord(e0));
    for (unsigned k = 0; k < 16; k++)
      hipLaunchKernelGGL((k_walk_red<RED>), dim3(grid), dim3(256), lds, 0, a,
                         part, nrows, ppr, pt, k, 1.0);
    HIPCHECK(hipEventRecord(e1));
    HIPCHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms / 16);
  }
  HIPCHECK(hipGetLastError());
  std::sort(t.begin(), t.end());
  HIPCHECK(hipEventDestroy(e0));
  HIPCHECK(hipEventDestroy(e1));
  return t[t.size() / 2];
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

template <bool LNT, bool SNT, bool RW>
static float
run(double* a, double* part, unsigned nrows, unsigned ppr, unsigned pt,
    unsigned lds = 0)
{
  const unsigned grid = nrows * ppr;
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  for (unsigned k = 0; k < 16; k++) // warm-up
    hipLaunchKernelGGL((k_walk<LNT, SNT, RW>), dim3(grid), dim3(256), lds, 0, a,
                       part, nrows, ppr, pt, k, 1.0);
  std::vector<float> t;
  for (int rep = 0; rep < 7; rep++) {
    HIPCHECK(hipEventRecord(e0));
    for (unsigned k = 0; k < 16; k++)
      hipLaunchKernelGGL((k_walk<LNT, SNT, RW>), dim3(grid), dim3(256), lds, 0,
                         a, part, nrows, ppr, pt, k, 1.0);
    HIPCHECK(hipEventRecord(e1));
    HIPCHECK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms / 16);
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
  unsigned pt = 8;
  if (const char* e = std::getenv("MS_PT"))
    pt = (unsigned)std::atoi(e);
  for (int i = 1; i < argc; i++) {
    unsigned nr = 0, nc = 0;
    if (std::sscanf(argv[i], "%ux%u", &nr, &nc) != 2 || nc % 1024 != 0 || nr == 0) {
      std::fprintf(stderr, "bad size %s (RxC, C a multiple of 1024)\n", argv[i]);
      return 2;
    }
    const size_t n = (size_t)nr * nc;
    const unsigned ppr = nc / 1024;
    double *a = nullptr, *part = nullptr;
    HIPCHECK(hipMalloc(&a, n * sizeof(double)));
    HIPCHECK(hipMalloc(&part, (size_t)nr * ppr * 4 * sizeof(double)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, n);
    HIPCHECK(hipDeviceSynchronize());
    const double gb = n * sizeof(double) / 1e9;
    std::printf("%ux%u fp64  %.3f GB  tiles of %u rows\n", nr, nc, gb, pt);
#define ST_RUN(L, S, RW, NAME)                                                 \
  {                                                                            \
    const float ms = run<L, S, RW>(a, part, nr, ppr, pt);                      \
    std::printf("  %-26s %8.4f ms  %7.1f GB/s\n", NAME, ms,                    \
                (RW ? 2 : 1) * gb / (ms * 1e-3));                              \
    std::fflush(stdout);                                                       \
  }
    ST_RUN(false, false, true, "rw cached / cached");
    ST_RUN(false, true, true, "rw cached / nt-store");
    ST_RUN(true, false, true, "rw nt-load / cached");
    ST_RUN(true, true, true, "rw nt / nt");
    ST_RUN(false, false, false, "read cached");
    ST_RUN(true, false, false, "read nt");
#undef ST_RUN
    // workgroups per CU capped with dynamic LDS the kernel does not use
    for (unsigned cap : { 2u, 3u, 4u, 6u, 8u, 12u }) {
      const unsigned lds = (160u << 10) / cap - 2048u;
      const float ms = run<false, true, true>(a, part, nr, ppr, pt, lds);
      std::printf("  rw cached / nt-store, %2u per CU %8.4f ms  %7.1f GB/s\n", cap, ms,
                  2 * gb / (ms * 1e-3));
      std::fflush(stdout);
    }
    // + the reduction (cached loads, non-temporal stores, as k_flat ships)
    for (unsigned cap : { 0u, 3u, 4u, 6u }) {
      const unsigned lds = cap ? (160u << 10) / cap - 2048u : 0u;
      const float m1 = run_red<1>(a, part, nr, ppr, pt, lds);
      const float m2 = run_red<2>(a, part, nr, ppr, pt, lds);
      std::printf("  + reduction, %2u per CU: one partial per piece %8.4f ms, per wave "
                  "%8.4f ms\n", cap, m1, m2);
      std::fflush(stdout);
    }
    HIPCHECK(hipFree(a));
    HIPCHECK(hipFree(part));
  }
  return 0;
}
