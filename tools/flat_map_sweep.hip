// flat_map_sweep.hip — k_flat per pending count NP, by workgroup order and
// rows per workgroup.
//
// The deferred-write rounds that re-apply NP pending scalings load one more
// 16-byte column-scale vector per lane per pending round.  The matrix
// streams from HBM; the scale vectors come from L2 into every CU's L1 anew
// for every workgroup (a workgroup covers one 4 KB column piece of R rows,
// and the workgroups a CU runs in turn are on other pieces).  This probe
// times single launches of k_flat<..., NP> on a block with a ring of
// distinct s / 1/s vectors (as the solve keeps them) for
//   PT = 0      the row-major flat order (the library's)
//   PT = g > 0  piece-tiled: g row groups of one piece back to back, spread
//               over the XCDs (FlatPending::pt; FMS_PT=0,4,8,... picks the
//               values, default 0,16; g = 16 ... 1024 in
//               profiles/r02_flat_map_tiles_*.log)
// and R = 2, 4 rows per workgroup (4, 8 with FMS_R8=1), NP = -1 (every-round store), 0, 1, 2 and
// 3 (+ store, the storing round of a 4-round group).  Median of 7
// sequences of 8 launches (k = 0..7, so the ALT reversal alternates).
//
// Build: make -C tools flat_map_sweep flat_map_sweep_vload (the latter with
//        the row scales as vector loads, ST_ROW_VLOAD=1, for A/B)
// Run:   ./tools/flat_map_sweep f64 32768 8192x65536 8192
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

constexpr int kSeq = 8;
constexpr int kReps = 7;
constexpr int kRing = 7; // s_k and up to 5 pending + 1
static std::vector<unsigned> g_pts = { 0, 16 };
static std::vector<unsigned> g_pcs = { 0 }; // FMS_PC: column blocks of pc pieces (0 = none)
static int g_store_np = 3; // FMS_STORE_NP: the pending count of the storing round
static int g_max_np = 3;   // FMS_MAX_NP (<= 5)
static bool g_r8 = false;  // FMS_R8=1: 8 rows per workgroup instead of 2 and 4
static bool g_r1 = false;  // FMS_R1=1: 1 and 2 rows per workgroup (every NP)
static bool g_every = false; // FMS_EVERY=1: the every-round launch (NP = -1) only,
                             // R = 1, 2, 4 by PT

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

template <typename T>
struct Block
{
  unsigned nr, n;
  T* a;
  T* s[kRing];
  T* inv[kRing];
  T *part, *v;
  st_state* st;
};

template <typename T, bool NT, int R, int NP, int UF = 0>
static void
one(const Block<T>& b, unsigned pt, unsigned pc = 0)
{
  constexpr int W = 16 / sizeof(T);
  // kFlatU (vector path), or UF chunks per piece
  constexpr int U = UF ? UF : (sizeof(T) == 8 && !NT) ? 2 : 1;
  const unsigned ppr = (b.n + 256 * W * U - 1) / (256 * W * U);
  const unsigned grid = (b.nr + R - 1) / R * ppr;
  constexpr int NPK = NP < 0 ? -1 : NP;
  const bool store = NP < 0 || NP == g_store_np;
  float ms = time_seq([&](int k) {
    FlatPending<T, NPK> pd{};
    for (int i = 0; i < (NP > 0 ? NP : 0); i++) {
      pd.s[i] = b.s[1 + i];
      pd.inv[i] = b.inv[1 + i];
    }
    pd.inv_cur = b.inv[0];
    pd.store = store ? 1u : 0u;
    pd.pt = pt;
    pd.pc = pc;
    hipLaunchKernelGGL((k_flat<T, W, 0, NT, R, false, true, 2, 256, 0, kGatePlain, NPK, U>),
                       dim3(grid), dim3(256), 0, 0, b.a, b.s[0], b.part, b.v, b.nr, b.n,
                       ppr, 0u, (uint32_t)k, b.st, (T)0, 1u << 30, 0u, 0u, 0u, 0u, pd);
  });
  const double bytes = (store ? 2.0 : 1.0) * b.nr * (double)b.n * sizeof(T);
  std::printf("  NP=%2d R=%d PT=%5u PC=%4u nt=%d%s  %8.4f ms  %7.1f GB/s\n", NP, R, pt, pc,
              (int)NT, UF ? (UF == 1 ? " U=1" : UF == 2 ? " U=2" : " U=4") : "", ms,
              bytes / (ms * 1e-3) / 1e9);
  std::fflush(stdout);
}


template <typename T, bool NT, int R, int NP, int UF = 0>
static void
by_pt(const Block<T>& b)
{
  for (unsigned pt : g_pts)
    if (NP >= 0 || pt == 0 || g_every)
      for (unsigned pc : g_pcs)
        if (pc == 0 || pt != 0)
          one<T, NT, R, NP, UF>(b, pt, pc);
}

template <typename T, bool NT, int R>
static void
by_np(const Block<T>& b)
{
  by_pt<T, NT, R, -1>(b);
  by_pt<T, NT, R, 0>(b);
  by_pt<T, NT, R, 1>(b);
  by_pt<T, NT, R, 2>(b);
  by_pt<T, NT, R, 3>(b);
  if (g_max_np >= 4)
    by_pt<T, NT, R, 4>(b);
  if (g_max_np >= 5)
    by_pt<T, NT, R, 5>(b);
}

template <typename T, bool NT>
static void
by_np_quick(const Block<T>& b)
{
  one<T, NT, 2, -1>(b, 0);
  one<T, NT, 2, 0>(b, 0);
  one<T, NT, 2, 1>(b, 0);
  one<T, NT, 2, 2>(b, 0);
  one<T, NT, 2, 3>(b, 0);
}

template <typename T>
static void
run(unsigned nr, unsigned n)
{
  Block<T> b{};
  b.nr = nr;
  b.n = n;
  const size_t bytes = (size_t)nr * n * sizeof(T);
  HIPCHECK(hipMalloc(&b.a, (size_t)nr * n * sizeof(T)));
  for (int i = 0; i < kRing; i++) {
    HIPCHECK(hipMalloc(&b.s[i], sizeof(T) * n));
    HIPCHECK(hipMalloc(&b.inv[i], sizeof(T) * n));
  }
  HIPCHECK(hipMalloc(&b.part, sizeof(T) * (size_t)nr * ((n + 255) / 256)));
  HIPCHECK(hipMalloc(&b.v, sizeof(T) * n));
  HIPCHECK(hipMalloc(&b.st, sizeof(st_state)));
  HIPCHECK(hipMemset(b.st, 0, sizeof(st_state)));
  hipLaunchKernelGGL((k_generate<T, kRandom>), dim3(4096), dim3(256), 0, 0, b.a, nr,
                     n, 0u, (uint64_t)7);
  // row sums of a full square matrix of U(0,1] entries are ~n/2: every
  // ring slot holds n/2 (the scales then keep the matrix's magnitude)
  std::vector<T> h(n, (T)(n / 2));
  for (int i = 0; i < kRing; i++) {
    HIPCHECK(hipMemcpy(b.s[i], h.data(), sizeof(T) * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL((k_recip<T>), dim3(64), dim3(256), 0, 0, b.s[i], b.inv[i], n);
  }
  HIPCHECK(hipMemset(b.v, 0, sizeof(T) * n));
  HIPCHECK(hipDeviceSynchronize());
  const bool nt = bytes >= ((size_t)2 << 30); // flat_round_nt
  std::printf("%ux%u %s  %.3f GiB  nt=%d\n", nr, n, sizeof(T) == 8 ? "f64" : "f32",
              bytes / double(1 << 30), (int)nt);
  if (std::getenv("FMS_QUICK")) { // R = 2, PT = 0 only (PMC passes)
    if (nt)
      by_np_quick<T, true>(b);
    else
      by_np_quick<T, false>(b);
  } else if (g_every) {
    if (nt && std::getenv("FMS_U2")) { // 8 KB pieces on a non-temporal block
      by_pt<T, true, 2, -1>(b);
      by_pt<T, true, 2, -1, 2>(b);
      by_pt<T, true, 1, -1, 2>(b);
    } else if (nt) {
      by_pt<T, true, 1, -1>(b);
      by_pt<T, true, 2, -1>(b);
      by_pt<T, true, 4, -1>(b);
    } else if (std::getenv("FMS_U1")) { // 4 KB pieces on a cached fp64 block
      by_pt<T, false, 1, -1>(b);
      by_pt<T, false, 1, -1, 1>(b);
      by_pt<T, false, 2, -1, 1>(b);
    } else {
      by_pt<T, false, 1, -1>(b);
      by_pt<T, false, 2, -1>(b);
      by_pt<T, false, 4, -1>(b);
    }
  } else if (g_r1) {
    if (nt) {
      by_np<T, true, 1>(b);
      by_np<T, true, 2>(b);
    } else {
      by_np<T, false, 1>(b);
      by_np<T, false, 2>(b);
    }
  } else if (g_r8) {
    if (nt) {
      by_np<T, true, 4>(b);
      by_np<T, true, 8>(b);
    } else {
      by_np<T, false, 4>(b);
      by_np<T, false, 8>(b);
    }
  } else if (nt) {
    by_np<T, true, 2>(b);
    by_np<T, true, 4>(b);
  } else {
    by_np<T, false, 2>(b);
    by_np<T, false, 4>(b);
  }
  HIPCHECK(hipFree(b.a));
  for (int i = 0; i < kRing; i++) {
    HIPCHECK(hipFree(b.s[i]));
    HIPCHECK(hipFree(b.inv[i]));
  }
  HIPCHECK(hipFree(b.part));
  HIPCHECK(hipFree(b.v));
  HIPCHECK(hipFree(b.st));
}

int
main(int argc, char** argv)
{
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s f64|f32 N|RxN ...\n", argv[0]);
    return 1;
  }
  const bool f64 = std::strcmp(argv[1], "f64") == 0;
  if (const char* e = std::getenv("FMS_STORE_NP"))
    g_store_np = std::atoi(e);
  if (const char* e = std::getenv("FMS_MAX_NP"))
    g_max_np = std::atoi(e);
  g_r8 = std::getenv("FMS_R8") != nullptr;
  g_r1 = std::getenv("FMS_R1") != nullptr;
  g_every = std::getenv("FMS_EVERY") != nullptr;
  auto parse_list = [](const char* e, std::vector<unsigned>& out) {
    out.clear();
    for (const char* q = e; *q;) {
      out.push_back((unsigned)std::strtoul(q, nullptr, 10));
      while (*q && *q != ',')
        q++;
      if (*q == ',')
        q++;
    }
  };
  if (const char* e = std::getenv("FMS_PT")) // e.g. FMS_PT=0,4,8,16,32
    parse_list(e, g_pts);
  if (const char* e = std::getenv("FMS_PC")) // e.g. FMS_PC=0,32,64
    parse_list(e, g_pcs);
  for (int i = 2; i < argc; i++) {
    unsigned nr = 0, n = 0;
    if (std::sscanf(argv[i], "%ux%u", &nr, &n) != 2) {
      n = (unsigned)std::atoi(argv[i]);
      nr = n;
    }
    if (nr == 0 || n == 0 || nr > n) {
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
