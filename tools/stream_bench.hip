// stream_bench.hip — what access shape gets the most HBM bandwidth for an
// IN-PLACE read+write stream on MI355X (the byte pattern of the fused
// similarity-transform kernel), and for out-of-place copy and read-only
// sweeps.  Sweeps block size, grid size, per-lane unroll, partitioning
// (grid-stride vs contiguous chunk per workgroup) and the cache policy.
//
// Build: make -C tools stream_bench   Run: ./tools/stream_bench [MiB] [reps]
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

template <int POL>
__device__ __forceinline__ d2
ld(const d2* p)
{
  if constexpr (POL == 1)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}
template <int POL>
__device__ __forceinline__ void
st(d2* p, d2 v)
{
  if constexpr (POL == 1)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// MODE 0: in place a[i] *= f; 1: copy b[i] = a[i]*f; 2: read-only sum
template <int BLK, int U, int POL, bool CHUNK, int MODE>
__global__ __launch_bounds__(BLK) void
k_stream(d2* a, d2* b, size_t n2, double f, double* sink)
{
  double acc = 0;
  size_t begin, end, step;
  if constexpr (CHUNK) {
    const size_t per = (n2 + gridDim.x - 1) / gridDim.x;
    begin = (size_t)blockIdx.x * per;
    end = begin + per < n2 ? begin + per : n2;
    step = (size_t)BLK * U;
    begin += threadIdx.x;
  } else {
    begin = (size_t)blockIdx.x * BLK * U + threadIdx.x;
    end = n2;
    step = (size_t)gridDim.x * BLK * U;
  }
  // n2 is a multiple of every BLK*U*grid used here, so no tails
  for (size_t i = begin; i < end; i += step) {
    d2 x[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      x[u] = ld<POL>(a + i + u * BLK);
    if constexpr (MODE == 2) {
#pragma unroll
      for (int u = 0; u < U; u++)
        acc += x[u][0] + x[u][1];
    } else {
#pragma unroll
      for (int u = 0; u < U; u++)
        st<POL>((MODE == 0 ? a : b) + i + u * BLK, x[u] * f);
    }
  }
  if (MODE == 2 && acc == 1.2345)
    sink[0] = acc;
}

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

// in-place stream through buffer descriptors with explicit cache-policy aux
// bits on the load (LA) and the store (SA): 1 = sc0, 2 = nt, 16 = sc1
template <int BLK, int U, int LA, int SA>
__global__ __launch_bounds__(BLK) void
k_stream_buf(d2* a, size_t n2, double f)
{
  const size_t per = n2 / gridDim.x; // n2 is a multiple of grid*BLK*U
  d2* base = a + (size_t)blockIdx.x * per;
  __amdgpu_buffer_rsrc_t r =
    __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)(per * 16), 0x00020000);
  for (uint32_t i = threadIdx.x; i < per; i += BLK * U) {
    u4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      x[u] = __builtin_amdgcn_raw_buffer_load_b128(r, (i + u * BLK) * 16, 0, LA);
#pragma unroll
    for (int u = 0; u < U; u++) {
      d2 y = __builtin_bit_cast(d2, x[u]) * f;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), r,
                                             (i + u * BLK) * 16, 0, SA);
    }
  }
}

// "flat" dispatch (babelstream style): one short-lived workgroup per
// BLK*U 16-byte elements, no grid stride; MODE 0 in place, 1 copy
template <int BLK, int U, int POL, int MODE>
__global__ __launch_bounds__(BLK) void
k_flat(d2* a, d2* b, double f)
{
  const size_t base = (size_t)blockIdx.x * BLK * U + threadIdx.x;
  d2 x[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    x[u] = ld<POL>(a + base + u * BLK);
#pragma unroll
  for (int u = 0; u < U; u++)
    st<POL>((MODE == 0 ? a : b) + base + u * BLK, x[u] * f);
}

// flat read-only: one short workgroup per BLK*U 16-byte elements, a
// per-workgroup sum written out (like a row-piece partial)
template <int BLK, int U, int POL>
__global__ __launch_bounds__(BLK) void
k_flat_read(const d2* a, double* part)
{
  const size_t base = (size_t)blockIdx.x * BLK * U + threadIdx.x;
  double acc = 0;
#pragma unroll
  for (int u = 0; u < U; u++) {
    const d2 x = ld<POL>(a + base + u * BLK);
    acc += x[0] + x[1];
  }
  for (int off = 32; off > 0; off >>= 1)
    acc += __shfl_down(acc, off, 64);
  if ((threadIdx.x & 63) == 0)
    part[(size_t)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6)] = acc;
}

struct Bench
{
  d2 *a, *b;
  double* sink;
  size_t n2;
  int reps;
  hipEvent_t e0, e1;
  template <int BLK, int U, int POL, bool CHUNK, int MODE>
  void run(unsigned grid)
  {
    auto f = [&] {
      hipLaunchKernelGGL((k_stream<BLK, U, POL, CHUNK, MODE>), dim3(grid),
                         dim3(BLK), 0, 0, a, b, n2, 1.0, sink);
    };
    f();
    HIPCHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
      HIPCHECK(hipEventRecord(e0));
      f();
      HIPCHECK(hipEventRecord(e1));
      HIPCHECK(hipEventSynchronize(e1));
      float ms;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const double bytes = (MODE == 2 ? 1.0 : 2.0) * n2 * 16;
    std::printf("%-6s blk=%4d u=%d pol=%d %-6s grid=%5u  %8.4f ms  %7.1f GB/s\n",
                MODE == 0 ? "inpl" : (MODE == 1 ? "copy" : "read"), BLK, U, POL,
                CHUNK ? "chunk" : "stride", grid, t[t.size() / 2],
                bytes / (t[t.size() / 2] * 1e-3) / 1e9);
  }
  template <int BLK, int U, int POL, int MODE>
  void runflat()
  {
    const unsigned grid = (unsigned)(n2 / ((size_t)BLK * U));
    auto f = [&] {
      hipLaunchKernelGGL((k_flat<BLK, U, POL, MODE>), dim3(grid), dim3(BLK), 0,
                         0, a, b, 1.0);
    };
    f();
    HIPCHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
      HIPCHECK(hipEventRecord(e0));
      f();
      HIPCHECK(hipEventRecord(e1));
      HIPCHECK(hipEventSynchronize(e1));
      float ms;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::printf("flat   %-4s blk=%4d u=%d pol=%d grid=%9u  %8.4f ms  %7.1f GB/s\n",
                MODE == 0 ? "inpl" : "copy", BLK, U, POL, grid, t[t.size() / 2],
                2.0 * n2 * 16 / (t[t.size() / 2] * 1e-3) / 1e9);
  }
  double* part = nullptr;
  template <int BLK, int U, int POL>
  void runflatread()
  {
    const unsigned grid = (unsigned)(n2 / ((size_t)BLK * U));
    auto f = [&] {
      hipLaunchKernelGGL((k_flat_read<BLK, U, POL>), dim3(grid), dim3(BLK), 0,
                         0, a, part);
    };
    f();
    HIPCHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
      HIPCHECK(hipEventRecord(e0));
      f();
      HIPCHECK(hipEventRecord(e1));
      HIPCHECK(hipEventSynchronize(e1));
      float ms;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::printf("flat   read blk=%4d u=%d pol=%d grid=%9u  %8.4f ms  %7.1f GB/s\n",
                BLK, U, POL, grid, t[t.size() / 2],
                1.0 * n2 * 16 / (t[t.size() / 2] * 1e-3) / 1e9);
  }
  template <int BLK, int U, int LA, int SA>
  void runbuf(unsigned grid)
  {
    auto f = [&] {
      hipLaunchKernelGGL((k_stream_buf<BLK, U, LA, SA>), dim3(grid), dim3(BLK),
                         0, 0, a, n2, 1.0);
    };
    f();
    HIPCHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int r = 0; r < reps; r++) {
      HIPCHECK(hipEventRecord(e0));
      f();
      HIPCHECK(hipEventRecord(e1));
      HIPCHECK(hipEventSynchronize(e1));
      float ms;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::printf("inbuf  blk=%4d u=%d la=%2d sa=%2d grid=%5u  %8.4f ms  %7.1f GB/s\n",
                BLK, U, LA, SA, grid, t[t.size() / 2],
                2.0 * n2 * 16 / (t[t.size() / 2] * 1e-3) / 1e9);
  }
  template <int LA, int SA>
  void bufgrids()
  {
    for (unsigned g : { 256u, 512u, 1024u }) {
      runbuf<256, 4, LA, SA>(g);
      runbuf<256, 2, LA, SA>(g);
    }
  }
  template <int BLK, int U, int POL, int MODE>
  void grids()
  {
    for (unsigned g : { 256u, 512u, 1024u, 2048u }) {
      run<BLK, U, POL, false, MODE>(g);
      run<BLK, U, POL, true, MODE>(g);
    }
  }
};

int
main(int argc, char** argv)
{
  const size_t mib = argc > 1 ? std::atoll(argv[1]) : 8192;
  Bench B;
  B.reps = argc > 2 ? std::atoi(argv[2]) : 10;
  B.n2 = mib * 1024 * 1024 / 16;
  HIPCHECK(hipMalloc(&B.a, B.n2 * 16));
  HIPCHECK(hipMalloc(&B.b, B.n2 * 16));
  HIPCHECK(hipMalloc(&B.sink, 64));
  HIPCHECK(hipMemset(B.a, 0x3f, B.n2 * 16));
  HIPCHECK(hipMemset(B.b, 0x3f, B.n2 * 16));
  HIPCHECK(hipEventCreate(&B.e0));
  HIPCHECK(hipEventCreate(&B.e1));
  std::printf("buffer %zu MiB, reps %d\n", mib, B.reps);
  if (std::getenv("STREAM_FLAT_READ")) { // flat read-only variants
    HIPCHECK(hipMalloc(&B.part, B.n2 / 64 * 8 + 64));
    B.runflatread<256, 1, 1>();
    B.runflatread<256, 2, 1>();
    B.runflatread<256, 4, 1>();
    B.runflatread<256, 1, 0>();
    B.runflatread<256, 2, 0>();
    B.runflatread<256, 4, 0>();
    B.runflatread<512, 2, 1>();
    B.runflatread<1024, 1, 1>();
    B.grids<256, 4, 1, 2>();
    B.grids<256, 2, 0, 2>();
    return 0;
  }
  if (std::getenv("STREAM_FLAT_BLK")) { // flat in-place: workgroup size
    B.runflat<64, 1, 1, 0>();
    B.runflat<128, 1, 1, 0>();
    B.runflat<256, 1, 1, 0>();
    B.runflat<512, 1, 1, 0>();
    B.runflat<64, 2, 1, 0>();
    B.runflat<128, 2, 1, 0>();
    B.runflat<64, 1, 0, 0>();
    B.runflat<128, 1, 0, 0>();
    B.runflat<256, 1, 0, 0>();
    return 0;
  }
  if (std::getenv("STREAM_FLAT")) { // babelstream-style flat dispatch only
    B.runflat<256, 1, 0, 0>();
    B.runflat<256, 1, 1, 0>();
    B.runflat<256, 2, 1, 0>();
    B.runflat<256, 4, 1, 0>();
    B.runflat<256, 4, 0, 0>();
    B.runflat<1024, 1, 1, 0>();
    B.runflat<256, 1, 0, 1>();
    B.runflat<256, 1, 1, 1>();
    B.runflat<256, 4, 1, 1>();
    B.grids<256, 4, 1, 0>();
    B.grids<256, 4, 1, 1>();
    return 0;
  }
  B.grids<256, 4, 1, 0>();
  B.grids<256, 2, 1, 0>();
  B.bufgrids<0, 0>();
  B.bufgrids<2, 2>();
  B.bufgrids<2, 18>();
  B.bufgrids<18, 18>();
  B.bufgrids<16, 16>();
  B.bufgrids<17, 17>();
  B.bufgrids<19, 19>();
  B.bufgrids<3, 3>();
  B.bufgrids<2, 16>();
  B.bufgrids<0, 2>();
  B.bufgrids<2, 0>();
  B.grids<256, 4, 1, 2>();
  return 0;
}
