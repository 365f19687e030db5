// pitch_probe.hip — is the long rows' 1.5-3 % (configs[3] rank blocks, e.g.
// 8192 x 65536 fp64 against 32768^2 at the same bytes) a DRAM-side effect
// of the power-of-two row pitch?  Round 3 padded the rows by streaming
// wider blocks (more bytes); this probe keeps the bytes
// and changes only the pitch: the every-round flat walk of non-temporal
// blocks (256-thread workgroups, 2 rows x one 4 KB piece, pieces tiled by 4
// row groups, non-temporal loads and stores, x * f with f = 1.0 passed at
// run time (a constant 1.0 lets the compiler drop the store), one partial per
// workgroup and row as k_flat writes) over R x C doubles stored with a row
// pitch of C + pad doubles.  Median of 7 passes of 8 rounds.
//
// Build: make -C tools pitch_probe
// Run:   ./tools/pitch_probe 8192x65536 16384x32768 32768x32768
//        (PP_PADS=0,64,512,1024 PP_PT=4 tiles of row groups, PP_RO=1 read only)
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

__global__ __launch_bounds__(256) void
k_walk(double* a, double* part, unsigned nrows, unsigned ncols, size_t pitch, unsigned pt,
       double f, int ro)
{
  const unsigned ppr = ncols / 512, ng = nrows / 2;
  const unsigned b = blockIdx.x;
  const unsigned tile = b / (pt * ppr), t = b - tile * (pt * ppr);
  const unsigned left = ng - tile * pt, g = left < pt ? left : pt;
  const unsigned p = t / g, rg = tile * pt + (t - p * g);
  double s[2];
#pragma unroll
  for (int j = 0; j < 2; j++) {
    d2* x = reinterpret_cast<d2*>(a + (size_t)(2 * rg + j) * pitch + (size_t)p * 512) + threadIdx.x;
    const d2 v = __builtin_nontemporal_load(x);
    if (!ro) // uniform
      __builtin_nontemporal_store(v * f, x); // f = 1.0 at run time: the store stays
    s[j] = v.x + v.y;
  }
#pragma unroll
  for (int j = 0; j < 2; j++) {
    for (int o = 32; o >= 1; o >>= 1)
      s[j] += __shfl_xor(s[j], o);
  }
  __shared__ double red[2][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s[0];
    red[1][threadIdx.x >> 6] = s[1];
  }
  __syncthreads();
  if (threadIdx.x < 2)
    part[(size_t)(2 * rg + threadIdx.x) * ppr + p] =
      (red[threadIdx.x][0] + red[threadIdx.x][1]) + (red[threadIdx.x][2] + red[threadIdx.x][3]);
}

__global__ void
k_fill(double* a, size_t n)
{
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    unsigned long long z = (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    a[i] = 0.5 + (double)(z >> 11) * (1.0 / 9007199254740992.0);
  }
}

int
main(int argc, char** argv)
{
  std::vector<unsigned> pads = { 0, 64, 512, 1024 };
  const int ro = std::getenv("PP_RO") ? std::atoi(std::getenv("PP_RO")) : 0; // read only
  const unsigned pt = std::getenv("PP_PT") ? (unsigned)std::atoi(std::getenv("PP_PT")) : 4u;
  if (const char* e = std::getenv("PP_PADS")) {
    pads.clear();
    for (const char* q = e; *q;) {
      pads.push_back((unsigned)std::strtoul(q, const_cast<char**>(&q), 10));
      if (*q == ',')
        q++;
    }
  }
  for (int i = 1; i < argc; i++) {
    unsigned nr = 0, nc = 0;
    if (std::sscanf(argv[i], "%ux%u", &nr, &nc) != 2 || nc % 512 != 0 || nr % 8 != 0) {
      std::fprintf(stderr, "bad size %s (RxC, C a multiple of 512, R of 8)\n", argv[i]);
      return 2;
    }
    const double gb = (ro ? 1.0 : 2.0) * nr * (double)nc * 8 / 1e9;
    for (unsigned pad : pads) {
      const size_t pitch = (size_t)nc + pad, n = (size_t)nr * pitch;
      double *a = nullptr, *part = nullptr;
      HIPCHECK(hipMalloc(&a, n * sizeof(double)));
      HIPCHECK(hipMalloc(&part, (size_t)nr * (nc / 512) * sizeof(double)));
      hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, a, n);
      HIPCHECK(hipDeviceSynchronize());
      const unsigned grid = (nr / 2) * (nc / 512);
      hipEvent_t e0, e1;
      HIPCHECK(hipEventCreate(&e0));
      HIPCHECK(hipEventCreate(&e1));
      for (int k = 0; k < 4; k++)
        hipLaunchKernelGGL(k_walk, dim3(grid), dim3(256), 0, 0, a, part, nr, nc, pitch, pt, 1.0, ro);
      std::vector<float> t;
      for (int rep = 0; rep < 7; rep++) {
        HIPCHECK(hipEventRecord(e0));
        for (int k = 0; k < 8; k++)
          hipLaunchKernelGGL(k_walk, dim3(grid), dim3(256), 0, 0, a, part, nr, nc, pitch, pt, 1.0, ro);
        HIPCHECK(hipEventRecord(e1));
        HIPCHECK(hipEventSynchronize(e1));
        float ms = 0;
        HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms / 8);
      }
      HIPCHECK(hipGetLastError());
      std::sort(t.begin(), t.end());
      std::printf("%ux%u fp64 %s tiles %u, pitch %zu (+%u): %.4f ms per round, %.1f GB/s\n", nr,
                  nc, ro ? "read" : "read+write", pt, pitch, pad, t[3], gb / (t[3] * 1e-3));
      std::fflush(stdout);
      HIPCHECK(hipEventDestroy(e0));
      HIPCHECK(hipEventDestroy(e1));
      HIPCHECK(hipFree(a));
      HIPCHECK(hipFree(part));
    }
  }
  return 0;
}
