// Device-reduction unit test (GPU): the wave reductions every kernel of the
// library sums rows with (st_device.h) must agree bit for bit, whatever
// form a kernel uses - otherwise a row sum would depend on which kernel or
// partition computed it.
//   wave_sum(x)               the reference tree (lane 63 broadcast)
//   wave_sum_l63(x)           the same tree left in lane 63
//   wave_sum_pair(x0, x1)     two rows in one tree: lane 62 = wave_sum(x0),
//                             lane 63 = wave_sum(x1)
//   wave_sum_rows<NR>(x)      NR rows stepwise, lane 63
// Inputs: random magnitudes over many binades and signs (so that every
// association gives a different rounding), 4096 waves per dtype.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
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
      return 2;                                                                \
    }                                                                          \
  } while (0)

template <typename T>
__global__ __launch_bounds__(256) void
k_reduce(const T* in, T* out)
{
  // wave w of the launch: rows in[w][0][64], in[w][1][64]
  const uint32_t w = (blockIdx.x * 256 + threadIdx.x) >> 6, lane = threadIdx.x & 63;
  const T x0 = in[(size_t)w * 128 + lane], x1 = in[(size_t)w * 128 + 64 + lane];
  const T a = wave_sum(x0), b = wave_sum(x1);
  const T l0 = wave_sum_l63(x0);
  const T pr = wave_sum_pair(x0, x1);
  T rows[2] = { x0, x1 };
  wave_sum_rows<T, 2>(rows);
  T* o = out + (size_t)w * 8;
  if (lane == 0) {
    o[0] = a;
    o[1] = b;
  }
  if (lane == 63) {
    o[2] = l0;
    o[3] = pr;
    o[5] = rows[0];
    o[6] = rows[1];
  }
  if (lane == 62)
    o[4] = pr;
}

static uint64_t
mix(uint64_t z)
{
  z += 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

template <typename T>
static int
run(const char* name)
{
  const int waves = 4096;
  std::vector<T> h((size_t)waves * 128);
  for (size_t i = 0; i < h.size(); i++) {
    const uint64_t z = mix(i * 7 + sizeof(T));
    const double u = (double)((z >> 11) + 1) * 0x1.0p-53;           // (0, 1]
    const int e = (int)((z >> 3) % 40) - 20;                         // 2^-20 .. 2^19
    h[i] = (T)(((z & 1) ? -1.0 : 1.0) * u * std::ldexp(1.0, e));
  }
  T *d_in, *d_out;
  HIPCHECK(hipMalloc(&d_in, sizeof(T) * h.size()));
  HIPCHECK(hipMalloc(&d_out, sizeof(T) * waves * 8));
  HIPCHECK(hipMemcpy(d_in, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
  hipLaunchKernelGGL((k_reduce<T>), dim3(waves / 4), dim3(256), 0, 0, d_in, d_out);
  HIPCHECK(hipGetLastError());
  std::vector<T> o((size_t)waves * 8);
  HIPCHECK(hipMemcpy(o.data(), d_out, sizeof(T) * o.size(), hipMemcpyDeviceToHost));
  HIPCHECK(hipFree(d_in));
  HIPCHECK(hipFree(d_out));
  int bad = 0;
  auto same = [](T x, T y) { return std::memcmp(&x, &y, sizeof(T)) == 0; };
  for (int w = 0; w < waves; w++) {
    const T* r = &o[(size_t)w * 8];
    // r: wave_sum(x0), wave_sum(x1), l63(x0), pair lane 63 (x1), pair lane 62
    // (x0), rows[0], rows[1]
    if (!same(r[0], r[2]) || !same(r[0], r[4]) || !same(r[0], r[5]) || !same(r[1], r[3]) ||
        !same(r[1], r[6])) {
      if (bad++ < 5)
        std::printf("%s wave %d: sum %.17g %.17g  l63 %.17g  pair %.17g %.17g  rows %.17g "
                    "%.17g\n",
                    name, w, (double)r[0], (double)r[1], (double)r[2], (double)r[4],
                    (double)r[3], (double)r[5], (double)r[6]);
    }
  }
  std::printf("%s: %d waves, %d mismatches\n", name, waves, bad);
  return bad ? 1 : 0;
}

int
main()
{
  const int rc = run<double>("f64") | run<float>("f32");
  if (rc == 0)
    std::printf("wave reductions bit-identical\n");
  return rc;
}
