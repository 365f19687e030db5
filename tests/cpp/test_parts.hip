// Device unit test (GPU): k_parts_seg (4 / 2 rows per wave for rows of at
// most 16 / 32 partials) against k_parts (a wave per row) - the row sums
// s_{k+1}, their reciprocals and the eigenvector update must agree bit for
// bit, for every partial count up to 32 and row counts that leave a wave
// partly empty.  Partials: positive, over 40 binades (every association
// rounds differently).
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
run_case(const char* name, uint32_t nrows, uint32_t ppr, uint32_t seed)
{
  const uint32_t row0 = 5; // the block's first row in v / s_cur
  std::vector<T> part((size_t)nrows * ppr), scur(row0 + nrows), v(row0 + nrows);
  for (size_t i = 0; i < part.size(); i++) {
    const uint64_t z = mix(i * 131 + seed);
    const double u = (double)((z >> 11) + 1) * 0x1.0p-53;
    const int e = (int)((z >> 3) % 40) - 20;
    part[i] = (T)(u * std::ldexp(1.0, e));
  }
  for (size_t i = 0; i < scur.size(); i++) {
    scur[i] = (T)(1.0 + (double)(mix(i + 77 * seed) >> 11) * 0x1.0p-53);
    v[i] = (T)(0.5 + (double)(mix(i + 91 * seed) >> 11) * 0x1.0p-53);
  }
  st_state hs{};
  hs.max = 1.75;
  T *d_part, *d_scur, *d_v[2], *d_s[2], *d_inv[2];
  st_state* d_st;
  HIPCHECK(hipMalloc(&d_part, sizeof(T) * part.size()));
  HIPCHECK(hipMalloc(&d_scur, sizeof(T) * scur.size()));
  HIPCHECK(hipMalloc(&d_st, sizeof(st_state)));
  HIPCHECK(hipMemcpy(d_part, part.data(), sizeof(T) * part.size(), hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(d_scur, scur.data(), sizeof(T) * scur.size(), hipMemcpyHostToDevice));
  HIPCHECK(hipMemcpy(d_st, &hs, sizeof(hs), hipMemcpyHostToDevice));
  for (int i = 0; i < 2; i++) {
    HIPCHECK(hipMalloc(&d_v[i], sizeof(T) * v.size()));
    HIPCHECK(hipMalloc(&d_s[i], sizeof(T) * nrows));
    HIPCHECK(hipMalloc(&d_inv[i], sizeof(T) * nrows));
    HIPCHECK(hipMemcpy(d_v[i], v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice));
  }
  hipLaunchKernelGGL((k_parts<T>), dim3((nrows + 3) / 4), dim3(256), 0, 0, d_part, d_s[0],
                     nrows, ppr, 0u, d_st, d_scur, d_v[0], row0, nullptr, 0u, 0u, 0u,
                     d_inv[0]);
  if (ppr <= 16)
    hipLaunchKernelGGL((k_parts_seg<T, 16>), dim3((nrows + 15) / 16), dim3(256), 0, 0, d_part,
                       d_s[1], nrows, ppr, 0u, d_st, d_scur, d_v[1], row0, d_inv[1]);
  else
    hipLaunchKernelGGL((k_parts_seg<T, 32>), dim3((nrows + 7) / 8), dim3(256), 0, 0, d_part,
                       d_s[1], nrows, ppr, 0u, d_st, d_scur, d_v[1], row0, d_inv[1]);
  HIPCHECK(hipGetLastError());
  HIPCHECK(hipDeviceSynchronize());
  std::vector<T> s[2], inv[2], vo[2];
  for (int i = 0; i < 2; i++) {
    s[i].resize(nrows);
    inv[i].resize(nrows);
    vo[i].resize(v.size());
    HIPCHECK(hipMemcpy(s[i].data(), d_s[i], sizeof(T) * nrows, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(inv[i].data(), d_inv[i], sizeof(T) * nrows, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(vo[i].data(), d_v[i], sizeof(T) * v.size(), hipMemcpyDeviceToHost));
    HIPCHECK(hipFree(d_v[i]));
    HIPCHECK(hipFree(d_s[i]));
    HIPCHECK(hipFree(d_inv[i]));
  }
  HIPCHECK(hipFree(d_part));
  HIPCHECK(hipFree(d_scur));
  HIPCHECK(hipFree(d_st));
  const bool ok = std::memcmp(s[0].data(), s[1].data(), sizeof(T) * nrows) == 0 &&
                  std::memcmp(inv[0].data(), inv[1].data(), sizeof(T) * nrows) == 0 &&
                  std::memcmp(vo[0].data(), vo[1].data(), sizeof(T) * v.size()) == 0;
  // and the sums are not trivially equal: the association matters on this data
  T seq = 0;
  for (uint32_t p = 0; p < ppr; p++)
    seq += part[p];
  if (!ok)
    std::printf("%s nrows %u ppr %u: MISMATCH (row 0: %.17g vs %.17g; sequential %.17g)\n",
                name, nrows, ppr, (double)s[0][0], (double)s[1][0], (double)seq);
  return ok ? 0 : 1;
}

// launch time of k_parts vs k_parts_seg (printed, not asserted): rows of
// the configs[1] flat round (8192 rows x 8 partials) and the N = 2 rank
// block (5824 x 12)
template <typename T>
static int
time_case(uint32_t nrows, uint32_t ppr)
{
  T *d_part, *d_s, *d_scur, *d_v, *d_inv;
  st_state* d_st;
  HIPCHECK(hipMalloc(&d_part, sizeof(T) * nrows * ppr));
  HIPCHECK(hipMemset(d_part, 0, sizeof(T) * nrows * ppr));
  HIPCHECK(hipMalloc(&d_s, sizeof(T) * nrows));
  HIPCHECK(hipMalloc(&d_inv, sizeof(T) * nrows));
  HIPCHECK(hipMalloc(&d_scur, sizeof(T) * nrows));
  HIPCHECK(hipMalloc(&d_v, sizeof(T) * nrows));
  HIPCHECK(hipMalloc(&d_st, sizeof(st_state)));
  HIPCHECK(hipMemset(d_st, 0, sizeof(st_state)));
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  float ms[2];
  for (int which = 0; which < 2; which++) {
    for (int rep = 0; rep < 2; rep++) { // warm-up pass, then the timed one
      HIPCHECK(hipEventRecord(e0));
      for (int i = 0; i < 200; i++) {
        if (which == 0)
          hipLaunchKernelGGL((k_parts<T>), dim3((nrows + 3) / 4), dim3(256), 0, 0, d_part, d_s,
                             nrows, ppr, 0u, d_st, d_scur, d_v, 0u, nullptr, 0u, 0u, 0u, d_inv);
        else
          hipLaunchKernelGGL((k_parts_seg<T, 16>), dim3((nrows + 15) / 16), dim3(256), 0, 0,
                             d_part, d_s, nrows, ppr, 0u, d_st, d_scur, d_v, 0u, d_inv);
      }
      HIPCHECK(hipEventRecord(e1));
      HIPCHECK(hipEventSynchronize(e1));
      HIPCHECK(hipEventElapsedTime(&ms[which], e0, e1));
    }
  }
  std::printf("timing %u rows x %u partials: k_parts %.2f us, k_parts_seg %.2f us per launch "
              "(back to back)\n", nrows, ppr, ms[0] * 5.0f, ms[1] * 5.0f);
  HIPCHECK(hipFree(d_part));
  HIPCHECK(hipFree(d_s));
  HIPCHECK(hipFree(d_inv));
  HIPCHECK(hipFree(d_scur));
  HIPCHECK(hipFree(d_v));
  HIPCHECK(hipFree(d_st));
  return 0;
}

int
main()
{
  time_case<double>(8192, 8);
  time_case<double>(5824, 12);
  int bad = 0, cases = 0;
  for (uint32_t ppr = 1; ppr <= 32; ppr++)
    for (uint32_t nrows : { 1u, 3u, 17u, 1003u, 8192u }) {
      bad += run_case<double>("f64", nrows, ppr, ppr * 1000 + nrows);
      bad += run_case<float>("f32", nrows, ppr, ppr * 1000 + nrows + 1);
      cases += 2;
    }
  std::printf("%d cases, %d mismatches\n", cases, bad);
  if (bad == 0)
    std::printf("k_parts_seg bit-identical to k_parts\n");
  return bad ? 1 : 0;
}
