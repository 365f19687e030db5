// store_probe.hip — the deferred-write STORING round (k_flat with NP = m - 1
// pending scalings, A stored) against alternative ways to feed it its row
// scales, on non-temporal fp64 blocks.
//
// The shipped storing launch (k_flat<..., R = 8, NP = 5>, runtime
// pend.store) re-applies 5 pending rounds and its own (12 fp64 multiplies per
// element) and needs 6 x R row scales per workgroup (1/s of each round for
// its R rows).  It loads them as scalar loads, one per row behind a
// row-in-block branch: 48 conditional s_loads, each waited for alone
// (scalar loads return out of order, a wave can only wait for all of them),
// and their SGPRs spill into VGPR lanes.  The probe kernel k_sp takes the
// same element math and partial sums (bitwise: checked against k_flat) with
//   RS = 0  the row scales as unconditional scalar loads (adjacent rows
//           merge into s_load_dwordx4 ... x16, one wait)
//   RS = 1  the row scales staged through LDS: the first 6 R lanes of the
//           workgroup load one each (vector loads, issued before the matrix
//           loads so waiting for them does not wait for the matrix), one
//           barrier, then every lane reads them as LDS broadcasts (VGPR
//           operands: no SGPR pressure, no scalar waits)
// by rows per workgroup R and piece tile PT (FlatPending::pt's order).
//
// Build: make -C tools store_probe
// Run:   ./tools/store_probe 32768 8192x65536      (SP_CHECK=1: bitwise check)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
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

using T = double;
using V = vec<double, 2>::type;
constexpr int W = 2;
constexpr int BLK = 256;
constexpr int NW = BLK / 64;
constexpr int kRing = 9; // s_k and up to 7 pending + 1

template <int NP>
struct Pend
{
  const T* s[NP > 0 ? NP : 1];
  const T* inv[NP > 0 ? NP : 1];
};

// workgroup b -> (row group, piece): row-major (pt = 0) or pt row groups of
// one piece back to back (k_flat's piece-tiled order)
__device__ __forceinline__ void
sp_map(uint32_t b, uint32_t ppr, uint32_t ng, uint32_t pt, uint32_t& rg, uint32_t& p)
{
  if (pt != 0) {
    const uint32_t tile = b / (pt * ppr), t = b - tile * (pt * ppr);
    const uint32_t left = ng - tile * pt, g = left < pt ? left : pt;
    p = t / g;
    rg = tile * pt + (t - p * g);
  } else {
    rg = b / ppr;
    p = b - rg * ppr;
  }
}

// full blocks only (nrows % R == 0, ncols % 512 == 0): the probe compares the
// row-scale feeds, not the ragged edges
template <int R, int NP, int RS, bool STORE, bool NTS = true>
__global__ __launch_bounds__(BLK) void
k_sp(T* a, const T* __restrict__ s_cur, const T* __restrict__ inv_cur, T* __restrict__ part,
     uint32_t nrows, uint32_t ncols, uint32_t ppr, uint32_t pt, const st_state* state,
     uint32_t k, Pend<NP> pend)
{
  if (flat_gated<kGatePlain>(state, k))
    return;
  constexpr int NS = NP + 1; // row-scale vectors: the pending rounds', then s_k's
  __shared__ T rsh[RS == 1 ? NS : 1][R];
  __shared__ T red[NW][R];
  uint32_t rg, p;
  sp_map(blockIdx.x, ppr, nrows / R, pt, rg, p);
  const uint32_t r0 = rg * R;
  if constexpr (RS == 1) {
    // first: the row scales (before the matrix loads, so that waiting for
    // them waits for nothing else)
    if (threadIdx.x < NS * R) {
      const uint32_t i = threadIdx.x / R, j = threadIdx.x - i * R;
      const T* src = i < (uint32_t)NP ? pend.inv[i < NP ? i : 0] : inv_cur;
      rsh[i][j] = src[r0 + j];
    }
  }
  const uint32_t c0 = (p * BLK + threadIdx.x) * W;
  const T* arow = a + (size_t)r0 * ncols + c0;
  V x[R];
#pragma unroll
  for (int j = 0; j < R; j++)
    x[j] = __builtin_nontemporal_load(reinterpret_cast<const V*>(arow + (size_t)j * ncols));
  const V sc = *reinterpret_cast<const V*>(s_cur + c0);
  V spc[NP > 0 ? NP : 1];
#pragma unroll
  for (int i = 0; i < NP; i++)
    spc[i] = *reinterpret_cast<const V*>(pend.s[i] + c0);
  T sr[RS == 0 ? NS : 1][R];
  if constexpr (RS == 0) {
#pragma unroll
    for (int i = 0; i < NS; i++) {
      const T* src = i < NP ? pend.inv[i < NP ? i : 0] : inv_cur;
#pragma unroll
      for (int j = 0; j < R; j++)
        sr[i][j] = src[r0 + j];
    }
  } else {
    __syncthreads();
  }
  T acc[R];
#pragma unroll
  for (int i = 0; i < NP; i++) {
#pragma unroll
    for (int j = 0; j < R; j++) {
      const T inv = RS == 0 ? sr[i][j] : rsh[i][j];
      x[j] = x[j] * (inv * spc[i]);
    }
  }
  T* wrow = a + (size_t)r0 * ncols + c0;
#pragma unroll
  for (int j = 0; j < R; j++) {
    const T inv = RS == 0 ? sr[NP][j] : rsh[NP][j];
    const V y = x[j] * (inv * sc); // cpp:324-325
    if constexpr (STORE && NTS)
      __builtin_nontemporal_store(y, reinterpret_cast<V*>(wrow + (size_t)j * ncols));
    else if constexpr (STORE)
      *reinterpret_cast<V*>(wrow + (size_t)j * ncols) = y;
    acc[j] = hsum<T, W>(y);
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j + 1 < R; j += 2) {
    const T t = wave_sum_pair(acc[j], acc[j + 1]);
    if (lane >= 62)
      red[wave][j + (lane - 62)] = t;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    T t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; w++)
      t += red[w][threadIdx.x];
    part[(size_t)(r0 + threadIdx.x) * ppr + p] = t;
  }
}

// k_pipe: R = RB * NB rows per workgroup walked in NB steps of RB rows, the
// next step's matrix loads issued before the current step's math and stores
// (double-buffered registers; sched_barrier keeps the order), so a
// workgroup keeps loads in flight through its compute; the column scales
// load once for the R rows, the row scales per step (scalar, unconditional).
// Element math, row sums and partials as k_flat (bitwise).
template <int RB, int NB, int NP, bool STORE>
__global__ __launch_bounds__(BLK) void
k_pipe(T* a, const T* __restrict__ s_cur, const T* __restrict__ inv_cur, T* __restrict__ part,
       uint32_t nrows, uint32_t ncols, uint32_t ppr, uint32_t pt, const st_state* state,
       uint32_t k, Pend<NP> pend)
{
  constexpr int R = RB * NB;
  if (flat_gated<kGatePlain>(state, k))
    return;
  __shared__ T red[NW][R];
  uint32_t rg, p;
  sp_map(blockIdx.x, ppr, nrows / R, pt, rg, p);
  const uint32_t r0 = rg * R;
  const uint32_t c0 = (p * BLK + threadIdx.x) * W;
  const T* ap = a + (size_t)r0 * ncols + c0;
  T* wp = a + (size_t)r0 * ncols + c0;
  V xa[RB], xb[RB];
#pragma unroll
  for (int j = 0; j < RB; j++)
    xa[j] = __builtin_nontemporal_load(reinterpret_cast<const V*>(ap + (size_t)j * ncols));
  const V sc = *reinterpret_cast<const V*>(s_cur + c0);
  V spc[NP > 0 ? NP : 1];
#pragma unroll
  for (int i = 0; i < NP; i++)
    spc[i] = *reinterpret_cast<const V*>(pend.s[i] + c0);
  T acc[R];
  auto load = [&](V (&x)[RB], int step) {
#pragma unroll
    for (int j = 0; j < RB; j++)
      x[j] = __builtin_nontemporal_load(
        reinterpret_cast<const V*>(ap + (size_t)(step * RB + j) * ncols));
  };
  auto work = [&](V (&x)[RB], int step) {
    const uint32_t rr = r0 + step * RB;
    T sr[NP + 1][RB];
#pragma unroll
    for (int i = 0; i <= NP; i++) {
      const T* src = i < NP ? pend.inv[i < NP ? i : 0] : inv_cur;
#pragma unroll
      for (int j = 0; j < RB; j++)
        sr[i][j] = src[rr + j];
    }
#pragma unroll
    for (int i = 0; i < NP; i++) {
#pragma unroll
      for (int j = 0; j < RB; j++)
        x[j] = x[j] * (sr[i][j] * spc[i]);
    }
#pragma unroll
    for (int j = 0; j < RB; j++) {
      const V y = x[j] * (sr[NP][j] * sc); // cpp:324-325
      if constexpr (STORE)
        __builtin_nontemporal_store(
          y, reinterpret_cast<V*>(wp + (size_t)(step * RB + j) * ncols));
      acc[step * RB + j] = hsum<T, W>(y);
    }
  };
#pragma unroll
  for (int st = 0; st < NB; st += 2) {
    if (st + 1 < NB)
      load(xb, st + 1);
    __builtin_amdgcn_sched_barrier(0);
    work(xa, st);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 2 < NB)
      load(xa, st + 2);
    __builtin_amdgcn_sched_barrier(0);
    if (st + 1 < NB)
      work(xb, st + 1);
    __builtin_amdgcn_sched_barrier(0);
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j + 1 < R; j += 2) {
    const T t = wave_sum_pair(acc[j], acc[j + 1]);
    if (lane >= 62)
      red[wave][j + (lane - 62)] = t;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    T t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; w++)
      t += red[w][threadIdx.x];
    part[(size_t)(r0 + threadIdx.x) * ppr + p] = t;
  }
}

template <typename F>
static float
time_seq(F launch, int seq = 8, int reps = 7)
{
  hipEvent_t a, b;
  HIPCHECK(hipEventCreate(&a));
  HIPCHECK(hipEventCreate(&b));
  for (int k = 0; k < seq; k++)
    launch(k);
  HIPCHECK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; r++) {
    HIPCHECK(hipEventRecord(a));
    for (int k = 0; k < seq; k++)
      launch(k);
    HIPCHECK(hipEventRecord(b));
    HIPCHECK(hipEventSynchronize(b));
    float ms;
    HIPCHECK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms / seq);
  }
  HIPCHECK(hipEventDestroy(a));
  HIPCHECK(hipEventDestroy(b));
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

struct Block
{
  unsigned nr, n, ppr;
  T* a;
  T* s[kRing];
  T* inv[kRing];
  T* part;
  T* v;
  st_state* st;
};

static void
report(const Block& b, const char* what, float ms, bool store)
{
  const double bytes = (store ? 2.0 : 1.0) * b.nr * (double)b.n * sizeof(T);
  std::printf("  %-34s %8.4f ms  %7.1f GB/s\n", what, ms, bytes / (ms * 1e-3) / 1e9);
  std::fflush(stdout);
}

// the library's launch: k_flat fp64 (non-temporal, 4 KB pieces, or cached,
// 8 KB pieces), FS stats, ALT, NP pending; `lds` bytes of dynamic LDS per
// workgroup cap the workgroups per CU
template <int R, int NP, bool NT = true, int DS = -1>
static void
lib_launch(const Block& b, int k, unsigned pt, bool store, unsigned lds = 0)
{
  constexpr int NPK = NP < 0 ? -1 : NP;
  constexpr int U = NT ? 1 : 2;
  FlatPending<T, NPK> pd{};
  for (int i = 0; i < (NP > 0 ? NP : 0); i++) {
    pd.s[i] = b.s[1 + i];
    pd.inv[i] = b.inv[1 + i];
  }
  pd.inv_cur = b.inv[0];
  pd.store = store ? 1u : 0u;
  pd.pt = pt;
  const unsigned ppr = b.n / (256 * W * U);
  const unsigned grid = b.nr / R * ppr;
  hipLaunchKernelGGL((k_flat<T, W, 0, NT, R, false, true, 2, 256, 0, kGatePlain, NPK, U, false,
                             DS>),
                     dim3(grid), dim3(256), lds, 0, b.a, b.s[0], b.part, b.v, b.nr, b.n, ppr,
                     0u, (uint32_t)k, b.st, (T)0, 1u << 30, 0u, 0u, 0u, 0u, pd);
}

// dynamic LDS that leaves room for `c` workgroups per CU (160 KB of LDS per
// CU; 0 = no cap)
static unsigned
lds_for(unsigned c)
{
  return c == 0 ? 0u : 163840u / c - 2048u;
}

// the shipped launch shapes of one store cycle (launch_flat_deferred) and
// the every-round launch, each under workgroup-per-CU caps
template <bool NT>
static void
cap_sweep(const Block& b)
{
  const unsigned caps[] = { 0, 8, 6, 5, 4, 3, 2 };
  const char* only = std::getenv("SP_ONLY");
  auto one = [&](const char* what, auto launch, bool store) {
    if (only && !std::strstr(what, only))
      return;
    for (unsigned c : caps) {
      const unsigned lds = lds_for(c);
      const float ms = time_seq([&](int k) { launch(k, lds); });
      char w[96];
      std::snprintf(w, sizeof w, "%s cap=%u/CU", what, c);
      report(b, w, ms, store);
    }
  };
  if (NT) {
    one("every R=2 PT=4", [&](int k, unsigned l) { lib_launch<2, -1, NT>(b, k, 4, true, l); }, true);
    one("NP=0 R=2 PT=8", [&](int k, unsigned l) { lib_launch<2, 0, NT>(b, k, 8, false, l); }, false);
    one("NP=1 R=4 PT=32", [&](int k, unsigned l) { lib_launch<4, 1, NT>(b, k, 32, false, l); }, false);
    one("NP=2 R=8 PT=32", [&](int k, unsigned l) { lib_launch<8, 2, NT>(b, k, 32, false, l); }, false);
    one("NP=3 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 3, NT>(b, k, 16, false, l); }, false);
    one("NP=4 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 4, NT>(b, k, 16, false, l); }, false);
    one("store NP=5 R=8 PT=0", [&](int k, unsigned l) { lib_launch<8, 5, NT>(b, k, 0, true, l); }, true);
    one("store NP=5 R=8 PT=0 DS=1", [&](int k, unsigned l) { lib_launch<8, 5, NT, 1>(b, k, 0, true, l); }, true);
    one("store NP=5 R=8 PT=4 DS=1", [&](int k, unsigned l) { lib_launch<8, 5, NT, 1>(b, k, 4, true, l); }, true);
    one("store NP=5 R=8 PT=4", [&](int k, unsigned l) { lib_launch<8, 5, NT>(b, k, 4, true, l); }, true);
    one("store NP=5 R=4 PT=0", [&](int k, unsigned l) { lib_launch<4, 5, NT>(b, k, 0, true, l); }, true);
    // two rows, the every-round launch's shape with the five pending scalings
    one("store NP=5 R=2 PT=0 DS=1", [&](int k, unsigned l) { lib_launch<2, 5, NT, 1>(b, k, 0, true, l); }, true);
    one("store NP=5 R=2 PT=4 DS=1", [&](int k, unsigned l) { lib_launch<2, 5, NT, 1>(b, k, 4, true, l); }, true);
    one("store NP=5 R=2 PT=16 DS=1", [&](int k, unsigned l) { lib_launch<2, 5, NT, 1>(b, k, 16, true, l); }, true);
  } else {
    // cached fp64 blocks (< 2 GiB): 8 KB pieces
    one("every R=1 PT=8", [&](int k, unsigned l) { lib_launch<1, -1, NT>(b, k, 8, true, l); }, true);
    one("NP=0 R=1 PT=4", [&](int k, unsigned l) { lib_launch<1, 0, NT>(b, k, 4, false, l); }, false);
    one("NP=1 R=4 PT=16", [&](int k, unsigned l) { lib_launch<4, 1, NT>(b, k, 16, false, l); }, false);
    one("NP=4 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 4, NT>(b, k, 16, false, l); }, false);
    one("store NP=5 R=8 PT=4", [&](int k, unsigned l) { lib_launch<8, 5, NT>(b, k, 4, true, l); }, true);
    one("store NP=5 R=8 PT=4 DS=1", [&](int k, unsigned l) { lib_launch<8, 5, NT, 1>(b, k, 4, true, l); }, true);
    one("NP=2 R=4 PT=16", [&](int k, unsigned l) { lib_launch<4, 2, NT>(b, k, 16, false, l); }, false);
    one("NP=3 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 3, NT>(b, k, 16, false, l); }, false);
  }
}

static unsigned g_lds = 0; // SP_LDS: dynamic LDS bytes per workgroup (caps workgroups per CU)

template <int R, int NP, int RS, bool STORE, bool NTS = true>
static void
sp_launch(const Block& b, int k, unsigned pt)
{
  Pend<NP> pd{};
  for (int i = 0; i < NP; i++) {
    pd.s[i] = b.s[1 + i];
    pd.inv[i] = b.inv[1 + i];
  }
  const unsigned grid = b.nr / R * b.ppr;
  hipLaunchKernelGGL((k_sp<R, NP, RS, STORE, NTS>), dim3(grid), dim3(BLK), g_lds, 0, b.a, b.s[0],
                     b.inv[0], b.part, b.nr, b.n, b.ppr, pt, b.st, (uint32_t)k, pd);
}

template <int R, int NP, int RS, bool NTS = true>
static void
sp_time(const Block& b, unsigned pt)
{
  const float ms = time_seq([&](int k) { sp_launch<R, NP, RS, true, NTS>(b, k, pt); });
  char w[96];
  std::snprintf(w, sizeof w, "k_sp NP=%d R=%d RS=%s PT=%u%s LDS=%u", NP, R, RS ? "lds" : "sgpr",
                pt, NTS ? "" : " cached-st", g_lds);
  report(b, w, ms, true);
}

static std::vector<unsigned> g_pts = { 0, 4, 16 };

// the matrix-free round in the flat form (k_flat<..., MF> + k_mparts) by
// rows per workgroup and piece tile, against k_mfree (the library's shape:
// 4 rows, 2 chunks, 512 workgroups, non-temporal on >= 512 MiB); v_prev =
// b.v, v_cur = b.inv[6], s_next = b.s[6]
template <int R, bool NT>
static void
mf_launch(const Block& b, int k, unsigned pt, unsigned lds)
{
  constexpr int U = NT ? 1 : 2;
  FlatPending<T, -1> pe{};
  pe.pt = pt;
  const unsigned ppr = b.n / (256 * W * U);
  const unsigned grid = b.nr / R * ppr;
  hipLaunchKernelGGL((k_flat<T, W, 0, NT, R, false, true, 2, 256, 0, kGatePlain, -1, U, false,
                             -1, true>),
                     dim3(grid), dim3(256), lds, 0, b.a, b.s[0], b.part, b.v, b.nr, b.n, ppr,
                     0u, (uint32_t)(k + 1), b.st, (T)0, 1u << 30, 0u, 0u, 0u, 0u, pe);
  const unsigned rb = (b.nr + 3) / 4, vb = std::min(256u, (b.n + 255) / 256);
  hipLaunchKernelGGL((k_mparts<T>), dim3(rb + vb), dim3(256), 0, 0, b.part, b.s[6], b.nr, ppr,
                     (uint32_t)(k + 1), b.st, b.s[0], b.v, b.inv[6], 0u, b.n, rb);
}

template <bool NT>
static void
mf_sweep(const Block& b)
{
  {
    std::vector<T> ones(b.n, (T)1);
    (void)hipMemcpy(b.v, ones.data(), sizeof(T) * b.n, hipMemcpyHostToDevice);
  }
  const unsigned ng = b.nr / 4;
  report(b, "k_mfree R=4 (library shape)", time_seq([&](int k) {
           hipLaunchKernelGGL((k_mfree<T, 4, W, 2, NT, 256, true>), dim3(std::min(512u, ng)),
                              dim3(256), 0, 0, b.a, b.s[0], b.s[6], b.v, b.inv[6], ng, 0u, b.n,
                              0u, (T)0, (uint32_t)(k + 1), 1u << 30, 0u, b.st);
         }), false);
  for (unsigned cap : { 0u, 5u, 4u }) {
    for (unsigned pt : { 0u, 8u, 16u, 32u }) {
      char w[96];
      std::snprintf(w, sizeof w, "MF R=2 PT=%u cap=%u", pt, cap);
      report(b, w, time_seq([&](int k) { mf_launch<2, NT>(b, k, pt, lds_for(cap)); }), false);
      std::snprintf(w, sizeof w, "MF R=4 PT=%u cap=%u", pt, cap);
      report(b, w, time_seq([&](int k) { mf_launch<4, NT>(b, k, pt, lds_for(cap)); }), false);
      std::snprintf(w, sizeof w, "MF R=8 PT=%u cap=%u", pt, cap);
      report(b, w, time_seq([&](int k) { mf_launch<8, NT>(b, k, pt, lds_for(cap)); }), false);
      if (!NT) {
        std::snprintf(w, sizeof w, "MF R=1 PT=%u cap=%u", pt, cap);
        report(b, w, time_seq([&](int k) { mf_launch<1, NT>(b, k, pt, lds_for(cap)); }), false);
      }
    }
  }
}



template <int RB, int NB, int NP, bool STORE>
static void
pipe_launch(const Block& b, int k, unsigned pt, unsigned lds)
{
  Pend<NP> pd{};
  for (int i = 0; i < NP; i++) {
    pd.s[i] = b.s[1 + i];
    pd.inv[i] = b.inv[1 + i];
  }
  const unsigned grid = b.nr / (RB * NB) * b.ppr;
  hipLaunchKernelGGL((k_pipe<RB, NB, NP, STORE>), dim3(grid), dim3(BLK), lds, 0, b.a,
                     b.s[0], b.inv[0], b.part, b.nr, b.n, b.ppr, pt, b.st, (uint32_t)k, pd);
}

template <int RB, int NB, int NP, bool STORE>
static void
pipe_time(const Block& b, unsigned pt, unsigned cap)
{
  const unsigned lds = lds_for(cap);
  const float ms = time_seq([&](int k) { pipe_launch<RB, NB, NP, STORE>(b, k, pt, lds); });
  char w[96];
  std::snprintf(w, sizeof w, "k_pipe NP=%d %s RB=%d NB=%d PT=%u cap=%u", NP,
                STORE ? "store" : "read", RB, NB, pt, cap);
  report(b, w, ms, STORE);
}



static void
run(unsigned nr, unsigned n, bool check)
{
  Block b{};
  b.nr = nr;
  b.n = n;
  b.ppr = n / (256 * W);
  const size_t bytes = (size_t)nr * n * sizeof(T);
  HIPCHECK(hipMalloc(&b.a, bytes));
  for (int i = 0; i < kRing; i++) {
    HIPCHECK(hipMalloc(&b.s[i], sizeof(T) * n));
    HIPCHECK(hipMalloc(&b.inv[i], sizeof(T) * n));
  }
  HIPCHECK(hipMalloc(&b.part, sizeof(T) * (size_t)nr * b.ppr));
  HIPCHECK(hipMalloc(&b.v, sizeof(T) * n));
  HIPCHECK(hipMalloc(&b.st, sizeof(st_state)));
  HIPCHECK(hipMemset(b.st, 0, sizeof(st_state)));
  hipLaunchKernelGGL((k_generate<T, kRandom>), dim3(4096), dim3(256), 0, 0, b.a, nr, n, 0u,
                     (uint64_t)7);
  // distinct scale vectors (ring slot i: s = n/2 * (1 + (i+1) * c / n / 64))
  for (int i = 0; i < kRing; i++) {
    std::vector<T> h(n);
    for (unsigned c = 0; c < n; c++)
      h[c] = (T)(n / 2) * (1.0 + (i + 1) * (double)c / n / 64.0);
    HIPCHECK(hipMemcpy(b.s[i], h.data(), sizeof(T) * n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL((k_recip<T>), dim3(64), dim3(256), 0, 0, b.s[i], b.inv[i], n);
  }
  HIPCHECK(hipDeviceSynchronize());
  std::printf("%ux%u f64  %.3f GiB (%s)\n", nr, n, bytes / double(1 << 30),
              std::getenv("SP_CACHED") ? "cached launch shapes" : "non-temporal");
  if (check) {
    // one launch each from the same A: k_flat NP = 5 store vs k_sp RS = 0, 1
    std::vector<T> a0(bytes / sizeof(T));
    HIPCHECK(hipMemcpy(a0.data(), b.a, bytes, hipMemcpyDeviceToHost));
    const size_t np = (size_t)nr * b.ppr;
    std::vector<T> ra(a0.size()), rp(np), xa(a0.size()), xp(np);
    lib_launch<8, 5>(b, 0, 0, true);
    HIPCHECK(hipMemcpy(ra.data(), b.a, bytes, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(rp.data(), b.part, np * sizeof(T), hipMemcpyDeviceToHost));
    bool ok = true;
    for (int rs = 0; rs < 4; rs++) {
      HIPCHECK(hipMemcpy(b.a, a0.data(), bytes, hipMemcpyHostToDevice));
      HIPCHECK(hipMemset(b.part, 0, np * sizeof(T)));
      if (rs == 0)
        sp_launch<8, 5, 0, true>(b, 0, 16);
      else if (rs == 1)
        sp_launch<8, 5, 1, true>(b, 0, 16);
      else if (rs == 2)
        pipe_launch<2, 4, 5, true>(b, 0, 4, 0);
      else
        pipe_launch<4, 2, 5, true>(b, 0, 0, lds_for(3));
      HIPCHECK(hipMemcpy(xa.data(), b.a, bytes, hipMemcpyDeviceToHost));
      HIPCHECK(hipMemcpy(xp.data(), b.part, np * sizeof(T), hipMemcpyDeviceToHost));
      const bool same = std::memcmp(ra.data(), xa.data(), bytes) == 0 &&
                        std::memcmp(rp.data(), xp.data(), np * sizeof(T)) == 0;
      std::printf("  check %s vs k_flat NP=5 store: %s\n",
                  rs == 0 ? "k_sp RS=0" : rs == 1 ? "k_sp RS=1" : rs == 2 ? "k_pipe 2x4" : "k_pipe 4x2",
                  same ? "bitwise equal" : "DIFFERENT");
      ok = ok && same;
    }
    HIPCHECK(hipMemcpy(b.a, a0.data(), bytes, hipMemcpyHostToDevice));
    if (!ok)
      std::exit(3);
  }
  // references: the library's every-round launch (2 rows, tiles of 4) and
  // its storing launch (8 rows, row-major, 5 pending)
  if (!std::getenv("SP_CAPS")) {
    report(b, "k_flat every-round R=2 PT=4",
           time_seq([&](int k) { lib_launch<2, -1>(b, k, 4, true); }), true);
    report(b, "k_flat store NP=5 R=8 PT=0 (lib)",
           time_seq([&](int k) { lib_launch<8, 5>(b, k, 0, true); }), true);
  }
  if (std::getenv("SP_LONGM")) { // longer store cycles: the launches m = 7, 8 would add
    const bool nt = !std::getenv("SP_CACHED");
    auto row = [&](const char* what, auto launch, bool store) {
      for (unsigned c : { 0u, 5u, 4u, 3u }) {
        char w[96];
        std::snprintf(w, sizeof w, "%s cap=%u", what, c);
        report(b, w, time_seq([&](int k) { launch(k, lds_for(c)); }), store);
      }
    };
    if (nt) {
      row("read NP=4 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 4, true, 0>(b, k, 16, false, l); }, false);
      row("read NP=5 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 5, true, 0>(b, k, 16, false, l); }, false);
      row("read NP=6 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 6, true, 0>(b, k, 16, false, l); }, false);
      row("store NP=5 R=8 PT=0", [&](int k, unsigned l) { lib_launch<8, 5, true, 1>(b, k, 0, true, l); }, true);
      row("store NP=6 R=8 PT=0", [&](int k, unsigned l) { lib_launch<8, 6, true, 1>(b, k, 0, true, l); }, true);
      row("store NP=7 R=8 PT=0", [&](int k, unsigned l) { lib_launch<8, 7, true, 1>(b, k, 0, true, l); }, true);
    } else {
      row("read NP=4 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 4, false, 0>(b, k, 16, false, l); }, false);
      row("read NP=5 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 5, false, 0>(b, k, 16, false, l); }, false);
      row("read NP=6 R=8 PT=16", [&](int k, unsigned l) { lib_launch<8, 6, false, 0>(b, k, 16, false, l); }, false);
      row("store NP=5 R=8 PT=4", [&](int k, unsigned l) { lib_launch<8, 5, false, 1>(b, k, 4, true, l); }, true);
      row("store NP=6 R=8 PT=4", [&](int k, unsigned l) { lib_launch<8, 6, false, 1>(b, k, 4, true, l); }, true);
      row("store NP=7 R=8 PT=4", [&](int k, unsigned l) { lib_launch<8, 7, false, 1>(b, k, 4, true, l); }, true);
    }
  } else if (std::getenv("SP_MF")) { // the flat matrix-free round's shapes
    if (std::getenv("SP_CACHED"))
      mf_sweep<false>(b);
    else
      mf_sweep<true>(b);
  } else if (std::getenv("SP_PIPE")) { // the software-pipelined k_pipe against k_flat (capped)
    for (unsigned cap : { 0u, 4u, 3u }) {
      report(b, (std::string("k_flat store NP=5 R=8 PT=0 cap=") + std::to_string(cap)).c_str(),
             time_seq([&](int k) { lib_launch<8, 5>(b, k, 0, true, lds_for(cap)); }), true);
      report(b, (std::string("k_flat read NP=4 R=8 PT=16 cap=") + std::to_string(cap)).c_str(),
             time_seq([&](int k) { lib_launch<8, 4>(b, k, 16, false, lds_for(cap)); }), false);
    }
    for (unsigned pt : { 0u, 4u, 16u })
      for (unsigned cap : { 0u, 6u, 4u, 3u }) {
        pipe_time<2, 4, 5, true>(b, pt, cap);
        pipe_time<4, 2, 5, true>(b, pt, cap);
        pipe_time<2, 2, 5, true>(b, pt, cap);
        pipe_time<2, 4, 4, false>(b, pt, cap);
        pipe_time<4, 2, 4, false>(b, pt, cap);
      }
  } else if (std::getenv("SP_CAPS")) { // the library's shapes under workgroup-per-CU caps
    if (std::getenv("SP_CACHED"))
      cap_sweep<false>(b);
    else
      cap_sweep<true>(b);
  } else if (std::getenv("SP_OCC")) { // workgroups per CU capped through dynamic LDS
    for (unsigned lds : { 0u, 20480u, 32768u, 40960u, 54272u, 81920u }) {
      g_lds = lds;
      for (unsigned pt : g_pts) {
        sp_time<8, 5, 0>(b, pt);
        sp_time<8, 0, 1>(b, pt);
        sp_time<2, 0, 1>(b, pt);
        sp_time<4, 5, 0>(b, pt);
      }
    }
    g_lds = 0;
  } else {
    for (unsigned pt : g_pts) {
      sp_time<8, 5, 0>(b, pt);
      sp_time<8, 5, 0, false>(b, pt);
      sp_time<8, 5, 1>(b, pt);
      sp_time<4, 5, 0>(b, pt);
      sp_time<4, 5, 1>(b, pt);
      sp_time<2, 5, 1>(b, pt);
      sp_time<8, 0, 1>(b, pt);
      sp_time<2, 0, 1>(b, pt);
    }
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
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s N|RxN ...\n", argv[0]);
    return 1;
  }
  const bool check = std::getenv("SP_CHECK") != nullptr;
  if (const char* e = std::getenv("SP_PT")) {
    g_pts.clear();
    for (const char* q = e; *q;) {
      g_pts.push_back((unsigned)std::strtoul(q, nullptr, 10));
      while (*q && *q != ',')
        q++;
      if (*q == ',')
        q++;
    }
  }
  for (int i = 1; i < argc; i++) {
    unsigned nr = 0, n = 0;
    if (std::sscanf(argv[i], "%ux%u", &nr, &n) != 2) {
      n = (unsigned)std::atoi(argv[i]);
      nr = n;
    }
    if (nr == 0 || n == 0 || nr > n || n % 512 || nr % 8) {
      std::fprintf(stderr, "bad size %s (n %% 512 == 0, rows %% 8 == 0)\n", argv[i]);
      return 1;
    }
    run(nr, n, check);
  }
  return 0;
}
