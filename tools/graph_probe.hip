// graph_probe.hip — per-launch cost of short dependent kernels on one
// stream: plain launches vs the same launches captured in a hipGraph.
//
// The solve loop's rounds below 144 MiB are 1.6-4 us kernels separated by
// 3.5-5 us (profiles/r03_state_mirror_trace_excerpt.csv).  This probe
// times chains of K launches of a kernel that touches a small buffer
// (1 MiB, so each kernel is a couple of microseconds like a 512^2 round):
//   stream   K hipLaunchKernelGGL on one stream
//   graph    the same K launches captured once, the executable graph
//            replayed
// per launch = total / K, median of 9 repeats.  Then the library's own
// round (st_round_f32, one k_round launch, eps = 0 so no round stops) at
// 512^2 ... 4096^2: the host's time to enqueue K rounds against the GPU's
// time per round, to tell a host-bound chain from a device-bound one.
//
// Build: make -C tools graph_probe      Run: ./tools/graph_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "similarity_transform.h"

#define HIPCHECK(x)                                                            \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   hipGetErrorString(e));                                      \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

__global__ __launch_bounds__(256) void
k_touch(float* a, unsigned n, unsigned k)
{
  const unsigned i = blockIdx.x * 256 + threadIdx.x;
  if (i < n)
    a[i] = a[i] * 0.999f + (float)(k & 1u);
}

int
main()
{
  const unsigned n = 1u << 18; // 1 MiB of floats
  const unsigned grid = (n + 255) / 256;
  float* a = nullptr;
  HIPCHECK(hipMalloc(&a, n * sizeof(float)));
  HIPCHECK(hipMemset(a, 0, n * sizeof(float)));
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  HIPCHECK(hipEventCreate(&e0));
  HIPCHECK(hipEventCreate(&e1));
  for (unsigned K : { 8u, 16u, 64u }) {
    std::vector<float> ts, tg;
    // stream launches
    for (int rep = 0; rep < 10; rep++) {
      HIPCHECK(hipEventRecord(e0, s));
      for (unsigned k = 0; k < K; k++)
        hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, s, a, n, k);
      HIPCHECK(hipEventRecord(e1, s));
      HIPCHECK(hipEventSynchronize(e1));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep)
        ts.push_back(ms * 1e3f / K);
    }
    // the same chain as a graph
    hipGraph_t g;
    hipGraphExec_t ge;
    HIPCHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (unsigned k = 0; k < K; k++)
      hipLaunchKernelGGL(k_touch, dim3(grid), dim3(256), 0, s, a, n, k);
    HIPCHECK(hipStreamEndCapture(s, &g));
    HIPCHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 10; rep++) {
      HIPCHECK(hipEventRecord(e0, s));
      HIPCHECK(hipGraphLaunch(ge, s));
      HIPCHECK(hipEventRecord(e1, s));
      HIPCHECK(hipEventSynchronize(e1));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep)
        tg.push_back(ms * 1e3f / K);
    }
    HIPCHECK(hipGraphExecDestroy(ge));
    HIPCHECK(hipGraphDestroy(g));
    std::sort(ts.begin(), ts.end());
    std::sort(tg.begin(), tg.end());
    std::printf("K=%3u  per launch: stream %6.2f us   graph %6.2f us\n", K,
                ts[ts.size() / 2], tg[tg.size() / 2]);
    std::fflush(stdout);
  }
  HIPCHECK(hipFree(a));
  // the library's round
  for (unsigned N : { 512u, 1024u, 2048u, 4096u }) {
    float *m = nullptr, *sv = nullptr, *v = nullptr;
    st_state* st = nullptr;
    HIPCHECK(hipMalloc(&m, (size_t)N * N * sizeof(float)));
    HIPCHECK(hipMalloc(&sv, 2 * (size_t)N * sizeof(float)));
    HIPCHECK(hipMalloc(&v, (size_t)N * sizeof(float)));
    HIPCHECK(hipMalloc(&st, sizeof(st_state)));
    if (st_generate_hilbert_f32(m, N, N, 0, s) || st_rowsum_f32(m, sv, N, N, s) ||
        st_state_reset(st, s)) {
      std::fprintf(stderr, "setup failed: %s\n", eigen_last_error());
      return 2;
    }
    HIPCHECK(hipMemcpyAsync(v, sv, N * sizeof(float), hipMemcpyDeviceToDevice, s));
    HIPCHECK(hipStreamSynchronize(s));
    const unsigned K = 64;
    std::vector<float> host, gpu;
    unsigned k = 0;
    for (int rep = 0; rep < 10; rep++) {
      HIPCHECK(hipEventRecord(e0, s));
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned j = 0; j < K; j++, k++)
        if (st_round_f32(m, sv + (k & 1u) * N, sv + ((k + 1) & 1u) * N, v, N, N, 0,
                         0.0f, k, 1u << 30, 0, st, s)) {
          std::fprintf(stderr, "round failed: %s\n", eigen_last_error());
          return 2;
        }
      const double h_us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
          .count();
      HIPCHECK(hipEventRecord(e1, s));
      HIPCHECK(hipEventSynchronize(e1));
      float ms = 0;
      HIPCHECK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) {
        host.push_back((float)(h_us / K));
        gpu.push_back(ms * 1e3f / K);
      }
    }
    std::sort(host.begin(), host.end());
    std::sort(gpu.begin(), gpu.end());
    std::printf("st_round_f32 %4u^2: host enqueue %6.2f us per round, GPU %6.2f us per round\n",
                N, host[host.size() / 2], gpu[gpu.size() / 2]);
    std::fflush(stdout);
    HIPCHECK(hipFree(m));
    HIPCHECK(hipFree(sv));
    HIPCHECK(hipFree(v));
    HIPCHECK(hipFree(st));
  }
  return 0;
}
