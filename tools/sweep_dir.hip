// sweep_dir.hip — does alternating the sweep direction between rounds pay?
//
// A round rewrites the whole matrix; the rows written last may still sit in
// the MI355X memory-side cache (MALL, 256 MB) when the next round starts.
// Forward-every-round sweeps start on the rows written FIRST (long evicted);
// alternating forward/backward starts on the rows written LAST.  This tool
// times sequences of consecutive rounds (k = 0, 1, 2, ...) of k_round and
// k_mfree with ALT off/on, cache policies, plus a plain in-place stream pass for
// reference, at the sizes given on the command line.
//
// Build: make -C tools sweep_dir   Run: ./tools/sweep_dir 8192 16384 32768
//        (or RxN: a sharded rank's R-row block of an N-column matrix)
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

template <typename T, bool NT>
__global__ __launch_bounds__(256) void
k_stream_rw(T* __restrict__ a, size_t n, T f, int rev)
{
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n;
       i += (size_t)gridDim.x * 256) {
    const size_t j = rev ? n - 1 - i : i;
    T x;
    if constexpr (NT)
      x = __builtin_nontemporal_load(a + j);
    else
      x = a[j];
    x *= f;
    if constexpr (NT)
      __builtin_nontemporal_store(x, a + j);
    else
      a[j] = x;
  }
}

constexpr int kSeq = 16; // rounds per timed sequence
constexpr int kReps = 7; // sequences; median reported

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
struct Bufs
{
  unsigned n;  // columns
  unsigned nr; // rows (a sharded rank's block: nr < n)
  T *a, *s, *sn, *v, *v2;
  st_state* st;
};

template <typename T, int ROWS, int NT, bool ALT, int U = 2>
static void
round_seq(const Bufs<T>& b, unsigned cap)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ng = b.nr / ROWS;
  const unsigned grid = cap < ng ? cap : ng;
  float ms = time_seq([&](int k) {
    hipLaunchKernelGGL((k_round<T, ROWS, W, U, 0, NT, 256, ALT>), dim3(grid),
                       dim3(256), 0, 0, b.a, b.s, b.sn, b.v, ng, 0u, b.n, 0u,
                       (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
  });
  const double bytes = 2.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  k_round rows=%d nt=%d alt=%d grid=%4u  %8.4f ms  %7.1f GB/s%s\n",
              ROWS, (int)NT, (int)ALT, grid, ms, bytes / (ms * 1e-3) / 1e9,
              U == 2 ? "" : (U == 1 ? "  u=1" : (U == 4 ? "  u=4" : "  u=8")));
}

// one launch (k_round) vs the split pair (k_round_split local + remote,
// back to back, no exchange) on the same block: the cost of splitting the
// round for the overlapped exchange, local columns = [c0, c0 + nr)
template <typename T, int ROWS, int NT, int NTL = NT>
static void
split_seq(const Bufs<T>& b, unsigned cap, unsigned c0)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ng = b.nr / ROWS;
  const unsigned grid = cap < ng ? cap : ng;
  const unsigned q0 = c0 / W, q1 = (c0 + b.nr) / W;
  float one = time_seq([&](int k) {
    hipLaunchKernelGGL((k_round<T, ROWS, W, 2, 0, NT, 256, true>), dim3(grid),
                       dim3(256), 0, 0, b.a, b.s, b.sn, b.v, ng, 0u, b.n, c0,
                       (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
  });
  float loc = time_seq([&](int k) {
    hipLaunchKernelGGL((k_round_split<T, ROWS, W, 2, 0, NTL, kSpanLocal>),
                       dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v2, b.v,
                       ng, 0u, b.n, c0, q0, q1, (T)0, (uint32_t)k, 1u << 30, 0u,
                       b.st);
  });
  float rem = time_seq([&](int k) {
    hipLaunchKernelGGL((k_round_split<T, ROWS, W, 2, 0, NT, kSpanRemote>),
                       dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v2, b.v,
                       ng, 0u, b.n, c0, q0, q1, (T)0, (uint32_t)k, 1u << 30, 0u,
                       b.st);
  });
  float both = time_seq([&](int k) {
    hipLaunchKernelGGL((k_round_split<T, ROWS, W, 2, 0, NTL, kSpanLocal>),
                       dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v2, b.v,
                       ng, 0u, b.n, c0, q0, q1, (T)0, (uint32_t)k, 1u << 30, 0u,
                       b.st);
    hipLaunchKernelGGL((k_round_split<T, ROWS, W, 2, 0, NT, kSpanRemote>),
                       dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v2, b.v,
                       ng, 0u, b.n, c0, q0, q1, (T)0, (uint32_t)k, 1u << 30, 0u,
                       b.st);
  });
  std::printf("  split rows=%d nt=%d ntl=%d grid=%4u local=[%u,%u)  k_round %8.4f  "
              "local %8.4f  remote %8.4f  local+remote %8.4f ms\n",
              ROWS, NT, NTL, grid, c0, c0 + b.nr, one, loc, rem, both);
}

// the flat round (k_stats + k_flat + k_parts) against one k_round launch
template <typename T, int NTF, int R, bool PW>
static void
flat_seq(const Bufs<T>& b, T* part)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ppr = (b.n + 256 * W - 1) / (256 * W);
  const unsigned nparts = ppr * (PW ? 4 : 1);
  const unsigned sgrid = (b.n + 255) / 256 < 256 ? (b.n + 255) / 256 : 256;
  const unsigned grid = (b.nr + R - 1) / R * ppr;
  float flat = time_seq([&](int k) {
    hipLaunchKernelGGL((k_stats<T>), dim3(sgrid), dim3(256), 0, 0, b.s, b.n,
                       (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
    hipLaunchKernelGGL((k_flat<T, W, 0, NTF != 0, R, PW>), dim3(grid),
                       dim3(256), 0, 0, b.a, b.s, part, b.v, b.nr, b.n, ppr, 0u,
                       (uint32_t)k, b.st);
    hipLaunchKernelGGL((k_parts<T>), dim3((b.nr + 3) / 4), dim3(256), 0, 0,
                       part, b.sn, b.nr, nparts, (uint32_t)k, b.st);
  });
  float only = time_seq([&](int k) {
    hipLaunchKernelGGL((k_flat<T, W, 0, NTF != 0, R, PW>), dim3(grid),
                       dim3(256), 0, 0, b.a, b.s, part, b.v, b.nr, b.n, ppr, 0u,
                       (uint32_t)k, b.st);
  });
  const double bytes = 2.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  flat nt=%d r=%d pw=%d  round (3 launches) %8.4f ms %7.1f GB/s | "
              "k_flat alone %8.4f ms %7.1f GB/s\n",
              NTF, R, (int)PW, flat, bytes / (flat * 1e-3) / 1e9, only,
              bytes / (only * 1e-3) / 1e9);
}

// the two-launch flat round: stats folded into k_flat's first row group,
// the v update into k_parts
template <typename T, int R, bool NT = true, int ALT = 0, int FB = 256,
          int GATE = kGateAtomic, int PT = 0, int U = 1>
static void
flat2_seq(const Bufs<T>& b, T* part, unsigned lds = 0)
{
  // lds: dynamic LDS reserved per workgroup (limits workgroups per CU)
  // PT: k_parts with one wave (0) or one thread (1) per row
  // U: chunks of FB * W columns per piece
  constexpr int W = 16 / sizeof(T);
  const unsigned ppr = (b.n + FB * W * U - 1) / (FB * W * U);
  const unsigned grid = (b.nr + R - 1) / R * ppr;
  float flat = time_seq([&](int k) {
    hipLaunchKernelGGL((k_flat<T, W, 0, NT, R, false, true, ALT, FB, 0, GATE, -1, U>),
                       dim3(grid), dim3(FB), lds, 0, b.a, b.s, part, b.v, b.nr,
                       b.n, ppr, 0u, (uint32_t)k, b.st, (T)0, 1u << 30, 0u);
    if constexpr (PT == 0)
      hipLaunchKernelGGL((k_parts<T>), dim3((b.nr + 3) / 4), dim3(256), 0, 0,
                         part, b.sn, b.nr, ppr, (uint32_t)k, b.st, b.s, b.v, 0u);
    else
      hipLaunchKernelGGL((k_parts_t<T>), dim3((b.nr + 255) / 256), dim3(256), 0,
                         0, part, b.sn, b.nr, ppr, (uint32_t)k, b.st, b.s, b.v,
                         0u);
  });
  const double bytes = 2.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  flat2 r=%d u=%d nt=%d alt=%d blk=%d gate=%d lds=%5u pt=%d  round (2 launches) "
              "%8.4f ms %7.1f GB/s\n",
              R, U, (int)NT, (int)ALT, FB, GATE, lds, PT, flat, bytes / (flat * 1e-3) / 1e9);
}

// the flat round with k_parts folded into k_flat (the last of a row group's
// workgroups sums the group's partials; no v update): one launch per round
template <typename T, int R, bool NT, int ALT, int U = 1>
static void
fold_seq(const Bufs<T>& b, T* part, uint32_t* cnt)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ppr = (b.n + 256 * W * U - 1) / (256 * W * U);
  const unsigned grid = (b.nr + R - 1) / R * ppr;
  float t = time_seq([&](int k) {
    hipLaunchKernelGGL((k_flat<T, W, 0, NT, R, false, true, ALT, 256, 0, kGatePlain, -1, U, true>),
                       dim3(grid), dim3(256), 0, 0, b.a, b.s, part, b.v, b.nr,
                       b.n, ppr, 0u, (uint32_t)k, b.st, (T)0, 1u << 30, 0u, 0u, 0u, 0u,
                       FlatPending<T, -1>{}, 0u, b.sn, cnt);
  });
  const double bytes = 2.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  fold  r=%d u=%d nt=%d alt=%d  round (1 launch) %8.4f ms %7.1f GB/s\n",
              R, U, (int)NT, ALT, t, bytes / (t * 1e-3) / 1e9);
}

// k_round with the library's launch shape (round_shape in st_kernels.hip)
template <typename T, int ROWS, int NT>
static float
round_shape_seq(const Bufs<T>& b, unsigned cap)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ng = b.nr / ROWS;
  const unsigned grid = cap < ng ? cap : ng;
  return time_seq([&](int k) {
    hipLaunchKernelGGL((k_round<T, ROWS, W, 2, 0, NT, 256, true>), dim3(grid),
                       dim3(256), 0, 0, b.a, b.s, b.sn, b.v, ng, 0u, b.n, 0u,
                       (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
  });
}

template <typename T>
static void
round_lib(const Bufs<T>& b)
{
  const size_t by = (size_t)b.nr * b.n * sizeof(T);
  float t;
  int rows;
  if (b.nr < 1024) {
    rows = 1;
    t = round_shape_seq<T, 1, kCached>(b, 512);
  } else if (by <= ((size_t)32 << 20)) {
    rows = 2;
    t = round_shape_seq<T, 2, kCached>(b, 1024);
  } else if (by < ((size_t)128 << 20)) {
    rows = 2;
    t = round_shape_seq<T, 2, kCached>(b, 512);
  } else if (by < ((size_t)1 << 30)) {
    rows = b.n <= 12288 ? 4 : 2;
    t = rows == 4 ? round_shape_seq<T, 4, kCached>(b, 256)
                  : round_shape_seq<T, 2, kCached>(b, 256);
  } else {
    rows = (size_t)b.n * sizeof(T) <= ((size_t)96 << 10) ? 4 : 2;
    t = rows == 4 ? round_shape_seq<T, 4, kNtBoth>(b, 256)
                  : round_shape_seq<T, 2, kNtBoth>(b, 256);
  }
  const double bytes = 2.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  k_round (library shape, rows=%d)  %8.4f ms %7.1f GB/s\n", rows, t,
              bytes / (t * 1e-3) / 1e9);
}

// the flat round with deferred writes: A stored every m = MAXP + 1 rounds,
// the rounds in between re-apply the pending scalings in registers; the
// time per round averaged over the 16-round sequence
template <typename T, bool NT, int R, int NP>
static void
defer_launch(const Bufs<T>& b, T* part, unsigned ppr, unsigned grid, int k,
             const T* s_cur, const T* inv_cur, T* const* ps, T* const* pi,
             bool store)
{
  constexpr int W = 16 / sizeof(T);
  FlatPending<T, NP> pend{};
  for (int i = 0; i < NP; i++) {
    pend.s[i] = ps[i];
    pend.inv[i] = pi[i];
  }
  pend.inv_cur = inv_cur;
  pend.store = store ? 1u : 0u;
  hipLaunchKernelGGL((k_flat<T, W, 0, NT, R, false, true, 2, 256, 0, kGatePlain, NP>),
                     dim3(grid), dim3(256), 0, 0, b.a, s_cur, part, b.v, b.nr, b.n,
                     ppr, 0u, (uint32_t)k, b.st, (T)0, 1u << 30, 0u, 0u, 0u, 0u, pend);
}

template <typename T, bool NT, int MAXP, int R = 2, bool RING = false, int RS = R,
          int R2 = R, bool RO = false>
static void
defer_seq(const Bufs<T>& b, T* part)
{
  // RO: never store (with MAXP = 0: a read-only flat pass every round)
  // RS: rows per workgroup of the storing round; R2: of the read-only rounds
  // with 2 or more pending rounds (R for the others)
  // RING: s / 1/s in a ring of M + 1 distinct vectors as the solve loop
  // keeps them (otherwise every slot is the same vector)
  static_assert(MAXP <= 3, "pending rounds");
  constexpr int W = 16 / sizeof(T);
  constexpr int M = MAXP + 1;
  const unsigned ppr = (b.n + 256 * W - 1) / (256 * W);
  const unsigned grid = (b.nr + R - 1) / R * ppr;
  const unsigned grid_s = (b.nr + RS - 1) / RS * ppr;
  const unsigned grid_2 = (b.nr + R2 - 1) / R2 * ppr;
  T* ring = nullptr;
  HIPCHECK(hipMalloc(&ring, sizeof(T) * (size_t)b.n * 2 * (M + 1)));
  for (int i = 0; i <= M; i++) {
    HIPCHECK(hipMemcpy(ring + (size_t)i * b.n, b.s, sizeof(T) * b.n,
                       hipMemcpyDeviceToDevice));
    hipLaunchKernelGGL((k_recip<T>), dim3(64), dim3(256), 0, 0, b.s,
                       ring + (size_t)(M + 1 + i) * b.n, b.n);
  }
  auto rs = [&](int i) { return RING ? ring + (size_t)(i % (M + 1)) * b.n : ring; };
  auto ri = [&](int i) {
    return RING ? ring + (size_t)(M + 1 + i % (M + 1)) * b.n : ring + (size_t)(M + 1) * b.n;
  };
  float t = time_seq([&](int k) {
    const int j0 = k - k % M, np = k % M;
    T* ps[4];
    T* pi[4];
    for (int i = 0; i < np; i++) {
      ps[i] = rs(j0 + i);
      pi[i] = ri(j0 + i);
    }
    const bool store = !RO && np == M - 1;
    if (store || (RO && np == MAXP && MAXP > 2)) {
      defer_launch<T, NT, RS, MAXP>(b, part, ppr, grid_s, k, rs(k), ri(k), ps, pi, store);
    } else {
      switch (np) {
      case 0: defer_launch<T, NT, R, 0>(b, part, ppr, grid, k, rs(k), ri(k), ps, pi, false); break;
      case 1: defer_launch<T, NT, R, 1>(b, part, ppr, grid, k, rs(k), ri(k), ps, pi, false); break;
      default: defer_launch<T, NT, R2, 2>(b, part, ppr, grid_2, k, rs(k), ri(k), ps, pi, false); break;
      }
    }
    hipLaunchKernelGGL((k_parts<T>), dim3((b.nr + 3) / 4), dim3(256), 0, 0,
                       part, b.sn, b.nr, ppr, (uint32_t)k, b.st, rs(k), b.v, 0u,
                       nullptr, 0u, 0u, 0u, (T*)nullptr);
  });
  HIPCHECK(hipFree(ring));
  const double bytes = (double)(M + 1) / M * b.nr * (double)b.n * sizeof(T);
  std::printf("  defer m=%d r=%d r2=%d rs=%d ring=%d nt=%d  per round %8.4f ms  (%.3f N^2 b "
              "per round) %7.1f GB/s\n",
              M, R, R2, RS, (int)RING, (int)NT, t, (double)(M + 1) / M,
              bytes / (t * 1e-3) / 1e9);
}

template <typename T>
static void
round_ref(const Bufs<T>& b, int rows_round, unsigned cap_round)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ng = b.nr / rows_round;
  const unsigned grid = cap_round < ng ? cap_round : ng;
  float one;
  const bool big = (double)b.nr * b.n * sizeof(T) >= (double)(1u << 30);
  if (rows_round == 2 && !big)
    one = time_seq([&](int k) {
      hipLaunchKernelGGL((k_round<T, 2, W, 2, 0, kCached, 256, true>),
                         dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v, ng,
                         0u, b.n, 0u, (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
    });
  else if (rows_round == 2)
    one = time_seq([&](int k) {
      hipLaunchKernelGGL((k_round<T, 2, W, 2, 0, kNtBoth, 256, true>),
                         dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v, ng,
                         0u, b.n, 0u, (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
    });
  else
    one = time_seq([&](int k) {
      hipLaunchKernelGGL((k_round<T, 4, W, 2, 0, kCached, 256, true>),
                         dim3(grid), dim3(256), 0, 0, b.a, b.s, b.sn, b.v, ng,
                         0u, b.n, 0u, (T)0, (uint32_t)k, 1u << 30, 0u, b.st);
    });
  const double bytes = 2.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  k_round rows=%d  %8.4f ms %7.1f GB/s\n", rows_round, one,
              bytes / (one * 1e-3) / 1e9);
}

template <typename T, int ROWS, bool NT, bool ALT>
static void
mfree_seq(const Bufs<T>& b, unsigned cap)
{
  constexpr int W = 16 / sizeof(T);
  const unsigned ng = b.nr / ROWS;
  const unsigned grid = cap < ng ? cap : ng;
  float ms = time_seq([&](int k) {
    hipLaunchKernelGGL((k_mfree<T, ROWS, W, 2, NT, 256, ALT>), dim3(grid),
                       dim3(256), 0, 0, b.a, b.s, b.sn, b.v, b.v2, ng, 0u,
                       b.n, 0u, (T)0, (uint32_t)(k + 1), 1u << 30, 0u, b.st);
  });
  const double bytes = 1.0 * b.nr * (double)b.n * sizeof(T);
  std::printf("  k_mfree rows=%d nt=%d alt=%d grid=%4u  %8.4f ms  %7.1f GB/s\n",
              ROWS, (int)NT, (int)ALT, grid, ms, bytes / (ms * 1e-3) / 1e9);
}

template <typename T, bool NT>
static void
stream_seq(const Bufs<T>& b, bool alt)
{
  const size_t nn = (size_t)b.nr * b.n;
  float ms = time_seq([&](int k) {
    hipLaunchKernelGGL((k_stream_rw<T, NT>), dim3(2048), dim3(256), 0, 0, b.a,
                       nn, (T)1, alt ? (k & 1) : 0);
  });
  std::printf("  stream_rw nt=%d alt=%d            %8.4f ms  %7.1f GB/s\n",
              (int)NT, (int)alt, ms, 2.0 * nn * sizeof(T) / (ms * 1e-3) / 1e9);
}

template <typename T>
static void
run(unsigned nr, unsigned n)
{
  Bufs<T> b;
  b.n = n;
  b.nr = nr;
  const size_t nn = (size_t)nr * n;
  HIPCHECK(hipMalloc(&b.a, nn * sizeof(T)));
  HIPCHECK(hipMalloc(&b.s, n * sizeof(T)));
  HIPCHECK(hipMalloc(&b.sn, n * sizeof(T)));
  HIPCHECK(hipMalloc(&b.v, n * sizeof(T)));
  HIPCHECK(hipMalloc(&b.v2, n * sizeof(T)));
  HIPCHECK(hipMalloc(&b.st, sizeof(st_state)));
  HIPCHECK(hipMemset(b.st, 0, sizeof(st_state)));
  hipLaunchKernelGGL((k_generate<T, kRandom>), dim3(65536), dim3(256), 0, 0,
                     b.a, nr, n, 0u, 0ull);
  hipLaunchKernelGGL(k_fill<T>, dim3(256), dim3(256), 0, 0, b.s, (uint64_t)n,
                     (T)1);
  hipLaunchKernelGGL(k_fill<T>, dim3(256), dim3(256), 0, 0, b.v, (uint64_t)n,
                     (T)1);
  HIPCHECK(hipDeviceSynchronize());
  if (nr == n)
    std::printf("n=%u %s  matrix %.3f GiB\n", n, sizeof(T) == 8 ? "f64" : "f32",
                nn * sizeof(T) / (double)(1u << 30));
  else
    std::printf("n=%ux%u %s  block %.3f GiB\n", nr, n,
                sizeof(T) == 8 ? "f64" : "f32",
                nn * sizeof(T) / (double)(1u << 30));
  stream_seq<T, true>(b, false);
  stream_seq<T, true>(b, true);
  stream_seq<T, false>(b, false);
  stream_seq<T, false>(b, true);
  if (std::getenv("SWEEP_RO")) { // read-only flat passes vs k_mfree
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    for (int rep = 0; rep < 2; rep++) {
      if (big) {
        defer_seq<T, true, 0, 2, true, 2, 2, true>(b, part);
        defer_seq<T, true, 0, 4, true, 4, 4, true>(b, part);
      } else {
        defer_seq<T, false, 0, 2, true, 2, 2, true>(b, part);
        defer_seq<T, false, 0, 4, true, 4, 4, true>(b, part);
      }
      for (unsigned cap : { 512u }) {
        mfree_seq<T, 4, true, false>(b, cap);
        mfree_seq<T, 2, false, true>(b, cap);
        mfree_seq<T, 4, false, true>(b, cap);
      }
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_DEFER_RS")) { // rows of the storing round vs the others
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    for (int rep = 0; rep < 2; rep++) {
      if (big) {
        defer_seq<T, true, 2, 2, true, 2>(b, part);
        defer_seq<T, true, 2, 2, true, 4>(b, part);
        defer_seq<T, true, 3, 2, true, 4>(b, part);
        defer_seq<T, true, 3, 2, true, 4, 4>(b, part);
        defer_seq<T, true, 3, 2, true, 4, 1>(b, part);
      } else {
        defer_seq<T, false, 2, 2, true, 2>(b, part);
        defer_seq<T, false, 2, 2, true, 4>(b, part);
        defer_seq<T, false, 2, 2, true, 1>(b, part);
        defer_seq<T, false, 3, 4, true, 4>(b, part);
        defer_seq<T, false, 3, 4, true, 2>(b, part);
        defer_seq<T, false, 3, 2, true, 4>(b, part);
      }
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_DEFER")) { // deferred writes: store A every m rounds
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    const bool ring_only = std::getenv("SWEEP_DEFER_RING") != nullptr;
    for (int rep = 0; rep < 2; rep++) {
      if (big) {
        flat2_seq<T, 2, true, 2, 256, kGatePlain>(b, part);
        if (!ring_only) {
          defer_seq<T, true, 1>(b, part);
          defer_seq<T, true, 2>(b, part);
          defer_seq<T, true, 3>(b, part);
        } else {
          defer_seq<T, true, 2, 2, false>(b, part);
          defer_seq<T, true, 1, 2, true>(b, part);
          defer_seq<T, true, 2, 2, true>(b, part);
          defer_seq<T, true, 3, 2, true>(b, part);
          defer_seq<T, true, 1, 4, true>(b, part);
          defer_seq<T, true, 2, 4, true>(b, part);
          defer_seq<T, true, 3, 4, true>(b, part);
        }
      } else {
        flat2_seq<T, 2, false, 2, 256, kGatePlain>(b, part);
        if (!ring_only) {
          defer_seq<T, false, 1>(b, part);
          defer_seq<T, false, 2>(b, part);
          defer_seq<T, false, 3>(b, part);
        } else {
          defer_seq<T, false, 2, 2, false>(b, part);
          defer_seq<T, false, 1, 2, true>(b, part);
          defer_seq<T, false, 2, 2, true>(b, part);
          defer_seq<T, false, 3, 2, true>(b, part);
          defer_seq<T, false, 1, 4, true>(b, part);
          defer_seq<T, false, 2, 4, true>(b, part);
          defer_seq<T, false, 3, 4, true>(b, part);
        }
      }
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_FOLD")) { // k_parts folded into k_flat (last arriver)
    T* part = nullptr;
    uint32_t* cnt = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    HIPCHECK(hipMalloc(&cnt, sizeof(uint32_t) * (size_t)b.nr));
    HIPCHECK(hipMemset(cnt, 0, sizeof(uint32_t) * (size_t)b.nr));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    const bool u2 = !big && sizeof(T) == 8;
    for (int rep = 0; rep < 3; rep++) {
      if (big) {
        flat2_seq<T, 2, true, 0, 256, kGatePlain>(b, part);
        fold_seq<T, 2, true, 0>(b, part, cnt);
      } else if (u2) {
        flat2_seq<T, 2, false, 2, 256, kGatePlain, 0, 2>(b, part);
        fold_seq<T, 2, false, 2, 2>(b, part, cnt);
      } else {
        flat2_seq<T, 2, false, 2, 256, kGatePlain>(b, part);
        fold_seq<T, 2, false, 2>(b, part, cnt);
      }
    }
    HIPCHECK(hipFree(cnt));
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_PARTS")) { // k_parts: one wave vs one thread per row
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    for (int rep = 0; rep < 3; rep++) {
      if (big) {
        flat2_seq<T, 2, true, 2, 256, kGatePlain, 0>(b, part);
        flat2_seq<T, 2, true, 2, 256, kGatePlain, 1>(b, part);
      } else {
        flat2_seq<T, 2, false, 2, 256, kGatePlain, 0>(b, part);
        flat2_seq<T, 2, false, 2, 256, kGatePlain, 1>(b, part);
      }
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_RB")) { // flat rows per workgroup x workgroup size (plain gate)
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
#define RB(R, FB)                                                              \
  (big ? flat2_seq<T, R, true, 2, FB, kGatePlain>(b, part)                     \
       : flat2_seq<T, R, false, 2, FB, kGatePlain>(b, part))
#define RBU(R, U)                                                              \
  (big ? flat2_seq<T, R, true, 2, 256, kGatePlain, 0, U>(b, part)              \
       : flat2_seq<T, R, false, 2, 256, kGatePlain, 0, U>(b, part))
    if (std::getenv("SWEEP_RBU")) { // chunks of 256 x 16 B per piece
      RBU(2, 1); RBU(2, 2); RBU(1, 2); RBU(1, 4); RBU(2, 1); RBU(2, 2);
    } else if (std::getenv("SWEEP_RB8")) {
      RB(2, 256); RB(8, 64); RB(8, 128); RB(4, 64); RB(2, 256);
    } else {
      RB(1, 256); RB(2, 256); RB(4, 256);
      RB(1, 128); RB(2, 128); RB(4, 128);
      RB(1, 64);  RB(2, 64);  RB(4, 64);
      RB(1, 512); RB(2, 512);
    }
#undef RB
#undef RBU
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_XCD")) { // odd-round piece order: global vs per-XCD reversal
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    for (int rep = 0; rep < 2; rep++) {
      if (std::getenv("SWEEP_XCD_ROUND"))
        round_lib<T>(b);
      if (big) {
        flat2_seq<T, 2, true, 1, 256, kGatePlain>(b, part);
        flat2_seq<T, 2, true, 2, 256, kGatePlain>(b, part);
        flat2_seq<T, 2, true, 0, 256, kGatePlain>(b, part);
      }
      flat2_seq<T, 2, false, 1, 256, kGatePlain>(b, part);
      flat2_seq<T, 2, false, 2, 256, kGatePlain>(b, part);
      flat2_seq<T, 2, false, 0, 256, kGatePlain>(b, part);
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_OCC")) { // flat workgroups per CU (LDS-limited)
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    for (unsigned lds : { 0u, 18u << 10, 22u << 10, 26u << 10, 32u << 10, 40u << 10 }) {
      if (big) {
        flat2_seq<T, 2, true, true, 256, kGatePlain>(b, part, lds);
        flat2_seq<T, 2, true, true, 256, kGateAtomic>(b, part, lds);
      } else {
        flat2_seq<T, 2, false, true, 256, kGatePlain>(b, part, lds);
        flat2_seq<T, 2, false, true, 256, kGateAtomic>(b, part, lds);
      }
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_GATE")) { // how the flat workgroups read the gate
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)2 << 30);
    for (int rep = 0; rep < 2; rep++) {
      if (big) {
        flat2_seq<T, 2, true, true, 256, kGateAtomic>(b, part);
        flat2_seq<T, 2, true, true, 256, kGatePlain>(b, part);
        flat2_seq<T, 2, true, true, 256, kGateSpec>(b, part);
        flat2_seq<T, 2, true, true, 256, kGateNone>(b, part);
        flat2_seq<T, 2, true, true, 64, kGatePlain>(b, part);
        flat2_seq<T, 2, true, true, 64, kGateNone>(b, part);
        flat2_seq<T, 4, true, true, 64, kGatePlain>(b, part);
      } else {
        flat2_seq<T, 2, false, true, 256, kGateAtomic>(b, part);
        flat2_seq<T, 2, false, true, 256, kGatePlain>(b, part);
        flat2_seq<T, 2, false, true, 256, kGateSpec>(b, part);
        flat2_seq<T, 2, false, true, 256, kGateNone>(b, part);
        flat2_seq<T, 2, false, true, 64, kGatePlain>(b, part);
        flat2_seq<T, 2, false, true, 64, kGateNone>(b, part);
        flat2_seq<T, 4, false, true, 64, kGatePlain>(b, part);
      }
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_FLAT")) { // the flat round vs k_round
    T* part = nullptr;
    const unsigned ppr = (b.n + 63) / 64;
    HIPCHECK(hipMalloc(&part, sizeof(T) * (size_t)b.nr * ppr * 4));
    const bool big = nn * sizeof(T) >= ((size_t)1 << 30);
    round_ref<T>(b, big ? 2 : (b.n > 12288 ? 2 : 4), big ? 256 : 256);
    if (big) {
      flat2_seq<T, 2, true, true>(b, part);
      flat2_seq<T, 2, true, true, 64>(b, part);
      flat2_seq<T, 4, true, true, 64>(b, part);
      flat2_seq<T, 2, true, true, 128>(b, part);
    } else {
      flat2_seq<T, 2, false, true>(b, part);
      flat2_seq<T, 2, false, true, 64>(b, part);
      flat2_seq<T, 4, false, true, 64>(b, part);
      flat2_seq<T, 2, false, true, 128>(b, part);
    }
    HIPCHECK(hipFree(part));
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  if (std::getenv("SWEEP_SPLIT")) { // split-round cost only
    const unsigned c0 = b.nr < b.n ? b.n / 2 - b.nr / 2 : 0;
    const unsigned c0a = c0 - c0 % 64;
    split_seq<T, 2, kCached>(b, 256, c0a);
    split_seq<T, 4, kCached>(b, 256, c0a);
    split_seq<T, 2, kCached, kNtBoth>(b, 256, c0a);
    split_seq<T, 4, kCached, kNtBoth>(b, 256, c0a);
    split_seq<T, 2, kCached, kNtLoads>(b, 256, c0a);
    split_seq<T, 2, kCached, kNtStores>(b, 256, c0a);
    HIPCHECK(hipFree(b.a));
    HIPCHECK(hipFree(b.s));
    HIPCHECK(hipFree(b.sn));
    HIPCHECK(hipFree(b.v));
    HIPCHECK(hipFree(b.v2));
    HIPCHECK(hipFree(b.st));
    return;
  }
  // k_round cache policy: nt = 0 cached, 1 non-temporal loads, 2
  // non-temporal stores, 3 both; U = chunks in flight per lane per row
  const bool big = nn * sizeof(T) >= ((size_t)1 << 30);
  for (unsigned cap : { 256u, 512u }) {
    if (big) {
      round_seq<T, 1, kNtBoth, true, 4>(b, cap);
      round_seq<T, 2, kNtBoth, true>(b, cap);
      round_seq<T, 2, kNtBoth, true, 4>(b, cap);
      round_seq<T, 4, kNtBoth, true>(b, cap);
      round_seq<T, 4, kNtBoth, true, 1>(b, cap);
    } else {
      round_seq<T, 1, kCached, true, 2>(b, cap);
      round_seq<T, 1, kCached, true, 4>(b, cap);
      round_seq<T, 1, kCached, true, 8>(b, cap);
      round_seq<T, 2, kCached, true>(b, cap);
      round_seq<T, 2, kCached, true, 4>(b, cap);
      round_seq<T, 4, kCached, true>(b, cap);
      round_seq<T, 4, kCached, true, 1>(b, cap);
    }
  }
  for (unsigned cap : { 512u, 1024u, 2048u }) {
    mfree_seq<T, 2, true, false>(b, cap);
    mfree_seq<T, 2, false, false>(b, cap);
    mfree_seq<T, 2, false, true>(b, cap);
    mfree_seq<T, 4, true, false>(b, cap);
    mfree_seq<T, 4, true, true>(b, cap);
    mfree_seq<T, 4, false, false>(b, cap);
    mfree_seq<T, 4, false, true>(b, cap);
  }
  HIPCHECK(hipFree(b.a));
  HIPCHECK(hipFree(b.s));
  HIPCHECK(hipFree(b.sn));
  HIPCHECK(hipFree(b.v));
  HIPCHECK(hipFree(b.v2));
  HIPCHECK(hipFree(b.st));
}

int
main(int argc, char** argv)
{
  // arguments: N (square) or RxN (a rank's row block of an N-column matrix)
  std::vector<std::pair<unsigned, unsigned>> shapes;
  for (int i = 1; i < argc; i++) {
    unsigned r = 0, c = 0;
    if (std::sscanf(argv[i], "%ux%u", &r, &c) != 2)
      r = c = (unsigned)std::atoi(argv[i]);
    shapes.push_back({ r, c });
  }
  if (shapes.empty())
    shapes = { { 8192u, 8192u }, { 16384u, 16384u }, { 32768u, 32768u } };
  for (auto [r, n] : shapes) {
    if (r == 0 || r % 64 || n % 64 || r > n) {
      std::fprintf(stderr, "rows must be a positive multiple of 64 <= cols, "
                           "cols a multiple of 64\n");
      return 1;
    }
    run<double>(r, n);
    run<float>(r, n);
  }
  return 0;
}
