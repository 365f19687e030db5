// st_device.h — device code of the similarity-transform iteration for
// gfx950 (CDNA4).  Included by st_kernels.hip (the library; earlier
// rounds' launch-shape sweeps are in the git history); not a public header.
//
// Reference behaviour (paths into itzmeanjan/eigen_value):
//   sum_across_rows       similarity_transform.cpp:77-152
//   find_max              similarity_transform.cpp:154-227
//   compute_eigen_vector  similarity_transform.cpp:229-265
//   compute_next_matrix   similarity_transform.cpp:286-330
//   stop                  similarity_transform.cpp:332-460
//   generators            utils.cpp:5-27, 125-154
//
// The path is an HBM-bound O(N^2) stream: no MFMA.  One fused kernel per
// round reads A_k once, writes A_{k+1} = D^-1 A_k D in place and reduces the
// STORED values into the next round's row sums (the reference sums the
// stored matrix, similarity_transform.cpp:40,52): 2*N^2*b bytes per round
// against the reference's 3*N^2*b.  Row sums are reduced without atomics
// (per-lane running sums in column order -> wave64 shuffle tree -> fixed
// order LDS combine), so every result is bitwise reproducible.
//
// Floating-point contraction must stay off (the stored A_{k+1} element is
// the rounded product and the sum adds exactly that value): this header
// sets `#pragma clang fp contract(off)` and the build passes
// -ffp-contract=off.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "similarity_transform.h"

#pragma clang fp contract(off)

namespace st {
namespace dev {

constexpr int kBlock = 256; // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kEpiBlock = 1024; // 16 waves

template <typename T, int W>
struct vec
{
  typedef T type __attribute__((ext_vector_type(W)));
};
template <typename T>
struct vec<T, 1>
{
  typedef T type;
};

template <typename T, int W>
__device__ __forceinline__ T
hsum(const typename vec<T, W>::type& y)
{
  if constexpr (W == 1) {
    return y;
  } else {
    T t = y[0];
#pragma unroll
    for (int k = 1; k < W; k++)
      t += y[k];
    return t;
  }
}

// DPP lane move (gfx9 data-parallel primitives; 64-bit values move as two
// dwords).  Lanes outside ROW_MASK receive an UNDEFINED value (mov_dpp: no
// zero-initialised `old` operand, which cost two v_mov per 64-bit step -
// 12 of the 30 VALU instructions of a double wave_sum): every reduction
// below reads its result in lane 63 only, and lane 63's dependency chain
// never passes through a masked-out lane (row_bcast 15 writes rows 1 and 3,
// row_bcast 31 rows 2 and 3, and lane 63 sums lanes 31 and 47 from those).
#ifndef ST_DPP_NOINIT
#define ST_DPP_NOINIT 1
#endif
template <int CTRL, int ROW_MASK = 0xf, typename T>
__device__ __forceinline__ T
dpp_mov(T x)
{
#if ST_DPP_NOINIT
#define ST_DPP32(v) __builtin_amdgcn_mov_dpp((v), CTRL, ROW_MASK, 0xf, false)
#else
#define ST_DPP32(v) __builtin_amdgcn_update_dpp(0, (v), CTRL, ROW_MASK, 0xf, false)
#endif
  if constexpr (sizeof(T) == 4) {
    return __int_as_float(ST_DPP32(__float_as_int((float)x)));
  } else {
    const long long b = __double_as_longlong((double)x);
    const int lo = ST_DPP32((int)b);
    const int hi = ST_DPP32((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
#undef ST_DPP32
}

template <typename T>
__device__ __forceinline__ T
read_lane63(T x)
{
  if constexpr (sizeof(T) == 4) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int((float)x), 63));
  } else {
    const long long b = __double_as_longlong((double)x);
    const int lo = __builtin_amdgcn_readlane((int)b, 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
  }
}

// Sum over the 64 lanes in a fixed tree, returned in every lane: pairs and
// quads (quad_perm), the four quads of each row of 16 (row_ror 4, 8), then
// the rows (row_bcast 15 into rows 1 and 3, row_bcast 31 into rows 2 and
// 3); lane 63 ends with ((R3 + R2) + (R1 + R0)) and is broadcast.  All DPP
// (VALU) - no LDS permutes - and the same order in every kernel, so a row
// sum never depends on which kernel or partition computed it.
template <typename T>
__device__ __forceinline__ T
wave_sum_l63(T x) // the sum, valid in lane 63 only
{
  x += dpp_mov<0xB1>(x);       // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);       // quad_perm [2,3,0,1]
  x += dpp_mov<0x124>(x);      // row_ror 4
  x += dpp_mov<0x128>(x);      // row_ror 8
  x += dpp_mov<0x142, 0xa>(x); // row_bcast 15
  x += dpp_mov<0x143, 0xc>(x); // row_bcast 31
  return x;
}

template <typename T>
__device__ __forceinline__ T
wave_sum(T x)
{
  return read_lane63(wave_sum_l63(x));
}

// x + (x of lane l ^ PL), PL = 16 (the same lane of the neighbouring row
// of 16) or 32 (of the other half-wave), with the gfx950 permlane swaps:
// swapping a value with itself leaves {own, partner} in the two results -
// which one is which depends on the lane, and the sum does not
template <int PL, typename T>
__device__ __forceinline__ T
permlane_add(T x)
{
  auto sw = [](int v) {
    return PL == 16 ? __builtin_amdgcn_permlane16_swap(v, v, false, false)
                    : __builtin_amdgcn_permlane32_swap(v, v, false, false);
  };
  if constexpr (sizeof(T) == 4) {
    const auto r = sw(__float_as_int((float)x));
    return __int_as_float((int)r[0]) + __int_as_float((int)r[1]);
  } else {
    const long long b = __double_as_longlong((double)x);
    const auto lo = sw((int)b), hi = sw((int)(b >> 32));
    const double a0 = __longlong_as_double(((long long)(int)hi[0] << 32) | (unsigned)lo[0]);
    const double a1 = __longlong_as_double(((long long)(int)hi[1] << 32) | (unsigned)lo[1]);
    return a0 + a1;
  }
}

// Two rows' wave sums in one tree (rows x0, x1 of every lane): the first
// step hands each lane of a pair the other's value of ONE row (even lanes
// keep row 0, odd lanes row 1), the next three run wave_sum's DPP steps on
// the interleaved rows (lane l ^ 2, ror 4, ror 8 keep a lane's parity), and
// the last two add the same lane of the other row of 16 / half-wave
// (permlane swaps keep the position).  Every addition is one of
// wave_sum's, operands in the same pairs, so lane 62 ends with
// wave_sum(x0) and lane 63 with wave_sum(x1), bit for bit, in 22 VALU
// instructions for the two (fp64) instead of 36.
template <typename T>
__device__ __forceinline__ T
wave_sum_pair(T x0, T x1)
{
  const bool odd = (threadIdx.x & 1u) != 0; // blocks are whole waves
  const T keep = odd ? x1 : x0;
  const T send = odd ? x0 : x1;
  T x = keep + dpp_mov<0xB1>(send); // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);            // quad_perm [2,3,0,1]
  x += dpp_mov<0x124>(x);           // row_ror 4
  x += dpp_mov<0x128>(x);           // row_ror 8
  x = permlane_add<16>(x);          // + the other row of 16
  x = permlane_add<32>(x);          // + the other half-wave
  return x;                         // lane 62: row 0, lane 63: row 1
}

// wave_sum of NR independent values, step by step across them (no stall
// between the dependent DPP steps of one value); the sums are left in lane
// 63 (bitwise wave_sum's results)
template <typename T, int NR>
__device__ __forceinline__ void
wave_sum_rows(T (&x)[NR])
{
#pragma unroll
  for (int i = 0; i < NR; i++)
    x[i] += dpp_mov<0xB1>(x[i]);
#pragma unroll
  for (int i = 0; i < NR; i++)
    x[i] += dpp_mov<0x4E>(x[i]);
#pragma unroll
  for (int i = 0; i < NR; i++)
    x[i] += dpp_mov<0x124>(x[i]);
#pragma unroll
  for (int i = 0; i < NR; i++)
    x[i] += dpp_mov<0x128>(x[i]);
#pragma unroll
  for (int i = 0; i < NR; i++)
    x[i] += dpp_mov<0x142, 0xa>(x[i]);
#pragma unroll
  for (int i = 0; i < NR; i++)
    x[i] += dpp_mov<0x143, 0xc>(x[i]);
}

template <typename T>
__device__ __forceinline__ T
wave_max(T x)
{
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T y = __shfl_down(x, off, 64);
    x = y > x ? y : x;
  }
  return x;
}

template <typename V, bool NT>
__device__ __forceinline__ V
ld(const V* p)
{
  if constexpr (NT)
    return __builtin_nontemporal_load(p);
  else
    return *p;
}

// A value every lane of the wave needs (a row's scale).  ST_ROW_VLOAD=1
// loads it through the VECTOR memory path instead of a scalar load (whose
// lgkmcnt wait - scalar loads return out of order, so a wave can only wait
// for all of them - then also holds up the next kernel-argument pointer a
// vector load needs).  Measured (flat_map_sweep{,_vload} (round 2, git history),
// profiles/r02_flat_map_rowload_*.log): 15-30 % SLOWER on non-temporal
// fp64 blocks with pending rounds (32768^2, NP = 1: 1.62 vs 1.33 ms), equal
// elsewhere, so the library keeps scalar row loads.
#ifndef ST_ROW_VLOAD
#define ST_ROW_VLOAD 0
#endif
// k_flat's unsplit rounds without load predicates (ST_FLAT_UNMASKED, see
// k_flat); 0 keeps the predicated loads of the split rounds for them too
#ifndef ST_FLAT_UNMASKED
#define ST_FLAT_UNMASKED 1
#endif
#ifndef ST_DEFER_STORE_NT
#define ST_DEFER_STORE_NT 0
#endif
template <typename T>
__device__ __forceinline__ T
ld_row(const T* p)
{
#if ST_ROW_VLOAD
  // global (not flat: a flat load counts in lgkmcnt as well)
  using GP = const __attribute__((address_space(1))) T*;
  GP g = (GP)p;
  asm volatile("" : "+v"(g));
  return *g;
#else
  return *p;
#endif
}

template <typename V, bool NT>
__device__ __forceinline__ void
st(V* p, const V& v)
{
  if constexpr (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

// ---------------------------------------------------------------------------
// fused scale + row-sum  (plain row-sum when SCALE == false)
//
// A row group is ROWS consecutive local rows [row_begin + g*ROWS, +ROWS)
// (always full; the host launches remainder rows with ROWS = 1).  Workgroup b
// takes groups g = b, b + gridDim.x, ... (grid-stride: the host may cap the
// grid below the group count), and sweeps each group's full width, W
// elements (16 bytes) per lane per access, U column chunks per iteration so
// that U*ROWS 16-byte loads are in flight per lane.  The column scale
// s_cur[c] is loaded once per chunk and reused for the ROWS rows.
//
// a_out == a_in is the in-place transform of the reference
// (similarity_transform.cpp:324); a_out != a_in writes A_{k+1} to a second
// buffer (ping-pong layout).  NT selects non-temporal (streaming) loads and
// stores for the matrix.
// ---------------------------------------------------------------------------
// A lane's chunks [c, hi) (stride BLK) left after its full groups of U:
// fewer than U, taken as groups of U/2, U/4, ..., 1 so that a group's loads
// are in flight together (a one-chunk-at-a-time tail serialises up to U - 1
// load latencies); column order, and so the sums, unchanged
template <int U, int BLK, typename F>
__device__ __forceinline__ void
sweep_tail(uint32_t c, uint32_t hi, F&& body)
{
  if constexpr (U >= 2) {
    constexpr int H = U / 2;
    if (c + (H - 1) * BLK < hi) {
      body(c, std::integral_constant<int, H>{});
      c += H * BLK;
    }
    sweep_tail<H, BLK>(c, hi, body);
  }
}

template <typename T, int ROWS, int W, int U, bool SCALE, bool SUM, int ORDER,
          bool NT, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void
k_fused(const T* a_in, T* a_out, const T* __restrict__ s_cur,
        T* __restrict__ s_next, uint32_t row_begin, uint32_t ngroups,
        uint32_t ncols, uint32_t row0, const st_state* __restrict__ state)
{
  using V = typename vec<T, W>::type;
  if (state != nullptr && state->done)
    return;

  const uint32_t nv = ncols / W;
  const V* sv = reinterpret_cast<const V*>(s_cur);
  __shared__ T red[BLK / 64][ROWS];

  for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const uint32_t rbase = row_begin + g * ROWS;
    const V* rin[ROWS];
    V* rout[ROWS];
    T inv[ROWS];
    T acc[ROWS];
#pragma unroll
    for (int j = 0; j < ROWS; j++) {
      rin[j] = reinterpret_cast<const V*>(a_in + (size_t)(rbase + j) * ncols);
      rout[j] = reinterpret_cast<V*>(a_out + (size_t)(rbase + j) * ncols);
      if constexpr (SCALE)
        inv[j] = (T)1 / s_cur[row0 + rbase + j];
      acc[j] = (T)0;
    }

    auto body = [&](uint32_t c, auto ucount) {
      constexpr int UU = decltype(ucount)::value;
      V x[UU][ROWS];
      V sc[UU];
#pragma unroll
      for (int u = 0; u < UU; u++)
#pragma unroll
        for (int j = 0; j < ROWS; j++)
          x[u][j] = ld<V, NT>(rin[j] + c + u * BLK);
      if constexpr (SCALE) {
#pragma unroll
        for (int u = 0; u < UU; u++)
          sc[u] = sv[c + u * BLK];
#pragma unroll
        for (int u = 0; u < UU; u++)
#pragma unroll
          for (int j = 0; j < ROWS; j++) {
            if constexpr (ORDER == 0)
              x[u][j] = x[u][j] * (inv[j] * sc[u]); // sim_transform.cpp:324-325
            else
              x[u][j] = (inv[j] * x[u][j]) * sc[u]; // main.py:13-16
          }
#pragma unroll
        for (int u = 0; u < UU; u++)
#pragma unroll
          for (int j = 0; j < ROWS; j++)
            st<V, NT>(rout[j] + c + u * BLK, x[u][j]);
      }
      if constexpr (SUM) {
#pragma unroll
        for (int u = 0; u < UU; u++)
#pragma unroll
          for (int j = 0; j < ROWS; j++)
            acc[j] += hsum<T, W>(x[u][j]);
      }
    };

    uint32_t c = threadIdx.x;
    for (; c + (U - 1) * BLK < nv; c += U * BLK)
      body(c, std::integral_constant<int, U>{});
    sweep_tail<U, BLK>(c, nv, body);

    if constexpr (SUM) {
      const int lane = threadIdx.x & 63;
      const int wave = threadIdx.x >> 6;
#pragma unroll
      for (int j = 0; j < ROWS; j++) {
        T t = wave_sum(acc[j]);
        if (lane == 0)
          red[wave][j] = t;
      }
      __syncthreads();
      if (threadIdx.x < ROWS) {
        T t = red[0][threadIdx.x];
#pragma unroll
        for (int w = 1; w < BLK / 64; w++)
          t += red[w][threadIdx.x];
        s_next[rbase + threadIdx.x] = t;
      }
      __syncthreads(); // red[] is reused by the next group
    }
  }
}

// ---------------------------------------------------------------------------
// one whole round in one launch (the solve loop's kernel)
//
// Round k of similarity_transform.cpp:39-53 for the local rows, given the
// FULL row-sum vector s_k (s_cur, length ncols) that the previous launch
// produced:
//   m_k    = max(0, max s_k)                       find_max        (cpp:154)
//   v[r]  *= s_k[r] / m_k   for the local rows     compute_eigen_v (cpp:260)
//   stop_k = all |s_k[i] - s_k[i+1]| < eps         stop            (cpp:413)
//   A     <- D_k^-1 A D_k, s_{k+1} = rowsum(A)     compute_next + sum_across
// Every workgroup reads all of s_k anyway (column scales), so each one
// derives m_k and stop_k redundantly from its first row group's sweep
// (max and a boolean AND are order-independent: every workgroup, and every
// rank of a sharded solve, gets the identical answer); workgroup 0 records
// the round in `state`.  There is no separate epilogue launch.
//
// After the stop round the reference performs no more transforms; here the
// stop round's launch still writes A_{k+1}/s_{k+1} (lambda, v and the count
// do not see it; the host-matrix solves work on a private copy, cpp:14,19,
// and the device-resident solves document that d_mat ends at A_end) and
// every later launch
// returns at once: state->end = k+1 is set by the stop round, and launch j
// exits if end != 0 && end <= j (a launch never gates on its own round).
// ---------------------------------------------------------------------------
// cache policy of k_round's matrix accesses (bit 0: non-temporal loads,
// bit 1: non-temporal stores)
constexpr int kCached = 0;
constexpr int kNtLoads = 1;
constexpr int kNtStores = 2;
constexpr int kNtBoth = 3;

// m / stop contribution of vector index q of s (columns q*W .. q*W+W-1):
// the running max, and |s_i - s_{i+1}| < eps for the W pairs that start in
// this vector (the last pair wraps to s[0] in the cyclic semantics)
template <typename T, int W>
__device__ __forceinline__ void
stats_at(const T* __restrict__ s, const typename vec<T, W>::type& sc,
         uint32_t q, uint32_t ncols, bool cyclic, T eps, T& mx, int& ok)
{
  T e[W + 1];
  if constexpr (W == 1) {
    e[0] = sc;
  } else {
#pragma unroll
    for (int i = 0; i < W; i++)
      e[i] = sc[i];
  }
  const uint32_t nxt = (q + 1) * W;
  const bool has_next = nxt < ncols || cyclic;
  e[W] = s[nxt < ncols ? nxt : 0];
#pragma unroll
  for (int i = 0; i < W; i++) {
    mx = e[i] > mx ? e[i] : mx;
    if (i < W - 1 || has_next) {
      const T d = e[i] - e[i + 1];
      ok &= (d < (T)0 ? -d : d) < eps ? 1 : 0; // cpp:419-421
    }
  }
}

// which columns a row-group pass covers (SPAN) and where its row sums go
constexpr int kSpanFull = 0;   // all columns -> s_next
constexpr int kSpanLocal = 1;  // vector range [q0, q1) -> part
constexpr int kSpanRemote = 2; // the rest -> s_next = part + sum

template <typename T, int R, int W, int U, int ORDER, int NT, int BLK,
          bool STATS, int SPAN = kSpanFull>
__device__ __forceinline__ void
round_group(T* a, const T* __restrict__ s_cur, T* __restrict__ s_next,
            uint32_t rbase, uint32_t ncols, uint32_t row0, bool cyclic, T eps,
            T& mx, int& ok, T (*red)[4], T* __restrict__ part = nullptr,
            uint32_t q0 = 0, uint32_t q1 = 0)
{
  using V = typename vec<T, W>::type;
  const uint32_t nv = ncols / W;
  const V* sv = reinterpret_cast<const V*>(s_cur);
  V* rows[R];
  T inv[R];
  T acc[R];
#pragma unroll
  for (int j = 0; j < R; j++) {
    rows[j] = reinterpret_cast<V*>(a + (size_t)(rbase + j) * ncols);
    inv[j] = (T)1 / s_cur[row0 + rbase + j];
    acc[j] = (T)0;
  }
  auto body = [&](uint32_t c, auto ucount) {
    constexpr int UU = decltype(ucount)::value;
    V x[UU][R];
    V sc[UU];
#pragma unroll
    for (int u = 0; u < UU; u++)
#pragma unroll
      for (int j = 0; j < R; j++)
        x[u][j] = ld<V, (NT & kNtLoads) != 0>(rows[j] + c + u * BLK);
#pragma unroll
    for (int u = 0; u < UU; u++)
      sc[u] = sv[c + u * BLK];
    if constexpr (STATS) {
#pragma unroll
      for (int u = 0; u < UU; u++)
        stats_at<T, W>(s_cur, sc[u], c + u * BLK, ncols, cyclic, eps, mx, ok);
    }
#pragma unroll
    for (int u = 0; u < UU; u++)
#pragma unroll
      for (int j = 0; j < R; j++) {
        if constexpr (ORDER == 0)
          x[u][j] = x[u][j] * (inv[j] * sc[u]); // cpp:324-325
        else
          x[u][j] = (inv[j] * x[u][j]) * sc[u]; // main.py:13-16
      }
#pragma unroll
    for (int u = 0; u < UU; u++)
#pragma unroll
      for (int j = 0; j < R; j++)
        st<V, (NT & kNtStores) != 0>(rows[j] + c + u * BLK, x[u][j]);
#pragma unroll
    for (int u = 0; u < UU; u++)
#pragma unroll
      for (int j = 0; j < R; j++)
        acc[j] += hsum<T, W>(x[u][j]);
  };
  // per-lane sweep of the vector range [lo, hi) in column order
  auto span = [&](uint32_t lo, uint32_t hi) {
    uint32_t c = lo + threadIdx.x;
    for (; c + (U - 1) * BLK < hi; c += U * BLK)
      body(c, std::integral_constant<int, U>{});
    sweep_tail<U, BLK>(c, hi, body);
  };
  if constexpr (SPAN == kSpanFull) {
    span(0, nv);
  } else if constexpr (SPAN == kSpanLocal) {
    span(q0, q1);
  } else {
    span(0, q0);
    span(q1, nv);
  }

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < R; j++) {
    T t = wave_sum(acc[j]);
    if (lane == 0)
      red[wave][j] = t;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    T t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < BLK / 64; w++)
      t += red[w][threadIdx.x];
    if constexpr (SPAN == kSpanFull)
      s_next[rbase + threadIdx.x] = t;
    else if constexpr (SPAN == kSpanLocal)
      part[rbase + threadIdx.x] = t;
    else
      s_next[rbase + threadIdx.x] = part[rbase + threadIdx.x] + t;
  }
  __syncthreads();
}

template <typename T, int ROWS, int W, int U, int ORDER, int NT, int BLK,
          bool ALT, int SPAN>
__device__ __forceinline__ void
round_body(T* a, const T* __restrict__ s_cur, T* __restrict__ s_next,
           T* __restrict__ v, uint32_t ng_main, uint32_t nrem, uint32_t ncols,
           uint32_t row0, T eps, uint32_t k, uint32_t max_itr,
           uint32_t semantics, st_state* state, T* __restrict__ part,
           uint32_t q0, uint32_t q1)
{
  static_assert(ROWS <= 4, "red[] holds 4 rows");
  {
    const uint32_t e =
      __hip_atomic_load(&state->end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e != 0 && e <= k)
      return; // a previous round stopped
  }
  __shared__ T red[BLK / 64][4];
  __shared__ T mx_sh[BLK / 64];
  __shared__ T m_sh;
  constexpr bool kStats = SPAN != kSpanLocal; // the local half only scales
  const bool cyclic = semantics == ST_SEM_SYCL;
  const uint32_t ngroups = ng_main + nrem;
  T mx = (T)0; // find_max starts from 0 (cpp:185)
  int ok = 1;
  T dummy_mx = 0;
  int dummy_ok = 1;

  // ALT: on odd rounds every workgroup walks its own row groups backwards,
  // so a round starts on the rows the previous round wrote last (still in
  // the memory-side cache) while each workgroup keeps the same rows (and
  // XCD) every round
  uint32_t cnt =
    blockIdx.x < ngroups ? (ngroups - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  if constexpr (SPAN == kSpanRemote) {
    if (q0 == 0 && q1 == ncols / W) { // nothing remote (P = 1): s_next = part
      for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
        const uint32_t rb =
          g < ng_main ? g * ROWS : ng_main * ROWS + (g - ng_main);
        const uint32_t nr = g < ng_main ? ROWS : 1;
        if (threadIdx.x < nr)
          s_next[rb + threadIdx.x] = part[rb + threadIdx.x] + (T)0;
      }
      cnt = 0;
    }
  }
  const bool rev = ALT && (k & 1u);
  for (uint32_t i = 0; i < cnt; i++) {
    const bool first = kStats && i == 0;
    const uint32_t g = blockIdx.x + (rev ? cnt - 1 - i : i) * gridDim.x;
    if (g < ng_main) {
      if (first)
        round_group<T, ROWS, W, U, ORDER, NT, BLK, kStats, SPAN>(
          a, s_cur, s_next, g * ROWS, ncols, row0, cyclic, eps, mx, ok, red,
          part, q0, q1);
      else
        round_group<T, ROWS, W, U, ORDER, NT, BLK, false, SPAN>(
          a, s_cur, s_next, g * ROWS, ncols, row0, cyclic, eps, dummy_mx,
          dummy_ok, red, part, q0, q1);
    } else {
      const uint32_t rb = ng_main * ROWS + (g - ng_main);
      if (first)
        round_group<T, 1, W, U, ORDER, NT, BLK, kStats, SPAN>(
          a, s_cur, s_next, rb, ncols, row0, cyclic, eps, mx, ok, red, part,
          q0, q1);
      else
        round_group<T, 1, W, U, ORDER, NT, BLK, false, SPAN>(
          a, s_cur, s_next, rb, ncols, row0, cyclic, eps, dummy_mx, dummy_ok,
          red, part, q0, q1);
    }
  }
  if constexpr (SPAN == kSpanLocal) {
    return;
  } else {
    if constexpr (SPAN == kSpanRemote) {
      // the remote sweep skipped the local vector range: add its m / stop,
      // 8 vectors in flight per lane (a dependent load per vector would
      // leave this short pass latency-bound)
      using V = typename vec<T, W>::type;
      const V* sv = reinterpret_cast<const V*>(s_cur);
      constexpr int kU = 8;
      uint32_t q = q0 + threadIdx.x;
      for (; q + (kU - 1) * BLK < q1; q += kU * BLK) {
        V x[kU];
#pragma unroll
        for (int u = 0; u < kU; u++)
          x[u] = sv[q + u * BLK];
#pragma unroll
        for (int u = 0; u < kU; u++)
          stats_at<T, W>(s_cur, x[u], q + u * BLK, ncols, cyclic, eps, mx, ok);
      }
      for (; q < q1; q += BLK)
        stats_at<T, W>(s_cur, sv[q], q, ncols, cyclic, eps, mx, ok);
    }

    // m_k and stop_k over the whole vector (this workgroup's copy)
    mx = wave_max(mx);
    if ((threadIdx.x & 63) == 0)
      mx_sh[threadIdx.x >> 6] = mx;
    const int stop = __syncthreads_and(ok);
    if (threadIdx.x == 0) {
      T m = mx_sh[0];
#pragma unroll
      for (int w = 1; w < BLK / 64; w++)
        m = mx_sh[w] > m ? mx_sh[w] : m;
      m_sh = m;
    }
    __syncthreads();
    const T m = m_sh;
    // v[r] *= s_k[r] / m_k for this workgroup's rows (cpp:260)
    for (uint32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {
      const uint32_t rb =
        g < ng_main ? g * ROWS : ng_main * ROWS + (g - ng_main);
      const uint32_t nr = g < ng_main ? ROWS : 1;
      if (threadIdx.x < nr) {
        const uint32_t r = row0 + rb + threadIdx.x;
        v[r] = v[r] * (s_cur[r] / m);
      }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      state->lambda = (double)s_cur[0]; // cpp:60-65
      state->max = (double)m;
      state->stop = stop ? 1u : 0u;
      state->round = k;
      if (stop) {
        state->iters = semantics == ST_SEM_SYCL ? k : k + 1; // cpp:54 / py:47
        state->end = k + 1;
        state->done = 1u;
      } else if (k + 1 >= max_itr) { // loop exhausted (cpp:39,54)
        state->iters = max_itr;
        state->end = k + 1;
        state->done = 1u;
      }
    }
  }
}

template <typename T, int ROWS, int W, int U, int ORDER, int NT,
          int BLK = kBlock, bool ALT = false>
__global__ __launch_bounds__(BLK) void
k_round(T* a, const T* __restrict__ s_cur, T* __restrict__ s_next,
        T* __restrict__ v, uint32_t ng_main, uint32_t nrem, uint32_t ncols,
        uint32_t row0, T eps, uint32_t k, uint32_t max_itr,
        uint32_t semantics, st_state* state)
{
  round_body<T, ROWS, W, U, ORDER, NT, BLK, ALT, kSpanFull>(
    a, s_cur, s_next, v, ng_main, nrem, ncols, row0, eps, k, max_itr,
    semantics, state, nullptr, 0u, 0u);
}

// ---------------------------------------------------------------------------
// the round split in two launches, for a sharded solve whose all-gather of
// s_k overlaps the first (sharded.py, overlap=True).  Rank p owns rows
// [row0, row0 + nrows) and therefore computed s_k for exactly the matching
// columns, vector range [q0, q1):
//   SPAN = kSpanLocal  (before the gather completes): those columns only —
//     A[r][c] *= s_k[c] / s_k[r], part[r] = their row sums; no stats
//   SPAN = kSpanRemote (after it): m_k / stop_k over the full s_k, the v
//     update, the remaining columns, s_{k+1}[r] = part[r] + their sum
// Element updates, m, stop and v are bit-identical to k_round; s_{k+1} adds
// the two column sets separately (fixed order, so still deterministic; for
// P = 1 the remote set is empty and s_{k+1} equals k_round's bit for bit).
// ---------------------------------------------------------------------------
template <typename T, int ROWS, int W, int U, int ORDER, int NT, int SPAN,
          int BLK = kBlock, bool ALT = true>
__global__ __launch_bounds__(BLK) void
k_round_split(T* a, const T* __restrict__ s_cur, T* __restrict__ s_next,
              T* __restrict__ part, T* __restrict__ v, uint32_t ng_main,
              uint32_t nrem, uint32_t ncols, uint32_t row0, uint32_t q0,
              uint32_t q1, T eps, uint32_t k, uint32_t max_itr,
              uint32_t semantics, st_state* state)
{
  round_body<T, ROWS, W, U, ORDER, NT, BLK, ALT, SPAN>(
    a, s_cur, s_next, v, ng_main, nrem, ncols, row0, eps, k, max_itr,
    semantics, state, part, q0, q1);
}

// ---------------------------------------------------------------------------
// flat round, for blocks of 144 MiB and more (eigen_value_amd/csrc/
// st_kernels.hip picks the form: cached accesses with ALT below 2 GiB,
// non-temporal above)
//
// tools/stream_bench.hip: an in-place stream moves 6.47 TB/s at 8 GiB when
// every workgroup takes one 4 KB piece and exits (millions of short
// workgroups: the chip sweeps a compact address window), against 5.62 TB/s
// for one long stream per CU (profiles/r01_stream_flat_8GiB.log).  The
// round then takes two launches, both gated like k_round (round k is a
// no-op once a round j < k stopped):
//   k_flat   one workgroup per (2 rows, piece of BLK*W columns): A <- D^-1 A D
//            on the piece (k_round's element update, bit for bit) and the
//            piece's sum -> part[r][p]; the first row group's workgroups,
//            whose pieces together cover s_k, also fold m_k and the stop
//            test into st_state's scratch words (order-independent atomics;
//            the last of them publishes round k, stats_publish)    2*N^2*b
//   k_parts  s_{k+1}[r] = the pieces of row r summed in a fixed order (one
//            wave per row), and v[r] *= s_k[r] / m_k      N * N/(BLK*W) * b
// (k_stats is the same stats pass as a launch of its own: the three-launch
// form, kept for the sweep tool.)  The row sums are deterministic and
// independent of the row partition (for blocks of one piece size, kFlatU
// in st_kernels.hip), but not bitwise k_round's (pieces are summed apart).
// ---------------------------------------------------------------------------
// thread 0 of each of `nwg` participating workgroups: fold the workgroup's
// max (>= 0, not NaN) and failed-pair flag into st_state's scratch words;
// the last of them to arrive publishes round k (exactly k_round's
// bookkeeping) and clears the scratch
template <typename T>
__device__ __forceinline__ void
stats_publish(T m, int fail, uint32_t nwg, const T* __restrict__ s, uint32_t k,
              uint32_t max_itr, uint32_t semantics, st_state* state)
{
  // m >= 0 and not NaN: its bit pattern orders like its value
  const uint64_t bits = sizeof(T) == 8 ? (uint64_t)__double_as_longlong((double)m)
                                       : (uint64_t)__float_as_uint((float)m);
  __hip_atomic_fetch_max(&state->max_bits, bits, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  if (fail)
    __hip_atomic_fetch_or(&state->fail, 1u, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t done_before = __hip_atomic_fetch_add(
    &state->arrivals, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (done_before != nwg - 1)
    return;
  // last arriver publishes round k
  const uint64_t mb = __hip_atomic_load(&state->max_bits, __ATOMIC_ACQUIRE,
                                        __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t f =
    __hip_atomic_load(&state->fail, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
  const T mk = sizeof(T) == 8 ? (T)__longlong_as_double((long long)mb)
                              : (T)__uint_as_float((uint32_t)mb);
  const bool stop = f == 0;
  state->lambda = (double)s[0]; // cpp:60-65
  state->max = (double)mk;
  state->stop = stop ? 1u : 0u;
  state->round = k;
  if (stop) {
    state->iters = semantics == ST_SEM_SYCL ? k : k + 1; // cpp:54 / py:47
    state->end = k + 1;
    state->done = 1u;
  } else if (k + 1 >= max_itr) { // loop exhausted (cpp:39,54)
    state->iters = max_itr;
    state->end = k + 1;
    state->done = 1u;
  }
  state->max_bits = 0; // scratch back to zero for the next round
  state->fail = 0u;
  state->arrivals = 0u;
}

template <typename T, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void
k_stats(const T* __restrict__ s, uint32_t n, T eps, uint32_t k,
        uint32_t max_itr, uint32_t semantics, st_state* state)
{
  {
    const uint32_t e =
      __hip_atomic_load(&state->end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e != 0 && e <= k)
      return;
  }
  __shared__ T mx_sh[BLK / 64];
  const bool cyclic = semantics == ST_SEM_SYCL;
  T mx = (T)0; // find_max starts from 0 (cpp:185): negatives and NaN never win
  int fail = 0;
  for (uint32_t i = blockIdx.x * BLK + threadIdx.x; i < n;
       i += gridDim.x * BLK) {
    const T x = s[i];
    mx = x > mx ? x : mx;
    if (i + 1 < n || cyclic) {
      const T d = x - s[i + 1 < n ? i + 1 : 0];
      fail |= (d < (T)0 ? -d : d) < eps ? 0 : 1; // cpp:419-421; NaN fails
    }
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0)
    mx_sh[threadIdx.x >> 6] = mx;
  fail = __syncthreads_or(fail);
  if (threadIdx.x == 0) {
    T m = mx_sh[0];
#pragma unroll
    for (int w = 1; w < BLK / 64; w++)
      m = mx_sh[w] > m ? mx_sh[w] : m;
    stats_publish<T>(m, fail, gridDim.x, s, k, max_itr, semantics, state);
  }
}

// The pieces (PWC columns each, ppr per row) lying wholly inside the local
// column range [col0, col1) of a split round: [pa, pa + nfull).  The piece
// past ncols' end counts as inside when col1 == ncols.
template <uint32_t PWC>
__host__ __device__ inline void
split_full_pieces(uint32_t ncols, uint32_t ppr, uint32_t col0, uint32_t col1,
                  uint32_t& pa, uint32_t& nfull)
{
  pa = (col0 + PWC - 1) / PWC;
  const uint32_t pb = col1 >= ncols ? ppr : col1 / PWC;
  nfull = pb > pa ? pb - pa : 0u;
}

// k_flat's workgroup count (the launchers' grids): every row group over its
// ppr pieces, or with SPLIT == 2 row group 0 over all of them and the rest
// over the pieces not wholly inside [col0, col1)
template <int R, uint32_t PWC, int SPLIT>
__host__ __device__ inline uint32_t
flat_nblocks(uint32_t nrows, uint32_t ncols, uint32_t ppr, uint32_t col0,
             uint32_t col1)
{
  const uint32_t ng = (nrows + R - 1) / R;
  if constexpr (SPLIT == 2) {
    uint32_t pa, nfull;
    split_full_pieces<PWC>(ncols, ppr, col0, col1, pa, nfull);
    return ppr + (ng - 1) * (ppr - nfull);
  } else {
    return ng * ppr;
  }
}

// How a flat workgroup learns that its launch follows the stopping round
// (state->end != 0 && end <= k).  Millions of short workgroups each pay
// this, so its latency matters: a plain load, served from the CU's L1 after
// the first workgroup of the launch on that CU.  Exact: `end` only changes
// inside the stopping launch k (to k + 1, which gates nothing in launch k),
// and every launch starts with the L1 invalidated.  It compiles to a scalar
// load (uniform address, nothing stored before it) and times like no gate
// at all: 1.8 % faster than an agent-scope atomic load per round at 32768^2
// fp64, 3.5 % on the P = 8 row block, within -0.7 % (8192^2) ... +3.5 %
// elsewhere (profiles/r01_sweep_gate*.log; the round-1 sweep tool's atomic,
// speculative and no-gate forms are in the git history).
__device__ __forceinline__ bool
flat_gated(const st_state* state, uint32_t k)
{
  const uint32_t e = state->end; // not volatile: volatile bypasses the L1 (sc0 sc1)
  return e != 0 && e <= k;
}

// The piece order of an odd round (ALT): 1 = the grid reversed; 2 = the
// grid reversed in steps of 8 workgroups with each workgroup's position in
// its step kept, so that (workgroups going to XCD blockIdx % 8) every piece
// is handled by the same XCD - and the same L2 - in every round.  The last
// gridDim % 8 workgroups keep their place.
template <int ALT>
__device__ __forceinline__ uint32_t
flat_reverse(uint32_t b, uint32_t g)
{
  if constexpr (ALT == 1) {
    return g - 1 - b;
  } else {
    const uint32_t g8 = g & ~7u;
    return b < g8 ? g8 - 8 - (b & ~7u) + (b & 7u) : b;
  }
}

// Deferred writes (NP >= 0): the matrix is stored only every few rounds.
// A round that does not store still computes A_{k+1} = D_k^-1 A_k D_k in
// registers and sums it into s_{k+1}; the next round re-reads the last
// STORED matrix A_j and first re-applies the pending rounds' scalings
// j .. k-1 - the same products, in the same order, as those rounds - so
// every value (A, s, v, the stop decisions) is bit-identical to storing
// every round, while a group of m rounds moves (m + 1) N^2 b instead of
// 2 m N^2 b.  s[i] are s_j .. s_{k-1} (oldest first), NP = k - j of them
// (a template argument: no runtime selects between the kernel arguments and
// the loads they address), and inv[i] their reciprocals 1 / s (written by
// k_parts / k_recip, the same correctly rounded quotient the round
// computed), so re-applying a round costs two multiplies per element and no
// division.
template <typename T, int NP>
struct FlatPending
{
  const T* s[NP > 0 ? NP : 1];
  const T* inv[NP > 0 ? NP : 1];
  const T* inv_cur; // 1 / s_k (the current round's row scales)
  uint32_t pt;      // piece-tiled workgroup order: pt row groups of a piece
                    // back to back (0 = row-major; see k_flat)
};

template <typename T, int W, int ORDER, bool NT, int R = 1, bool FS = false,
          int ALT = 0, int SPLIT = 0, int NP = -1, int U = 1, int DS = -1,
          bool MF = false, int FLIP = 0>
__global__ __launch_bounds__(kBlock) void
k_flat(T* a, const T* __restrict__ s_cur, T* __restrict__ part,
       T* __restrict__ v, uint32_t nrows, uint32_t ncols, uint32_t ppr,
       uint32_t row0, uint32_t k, st_state* state, T eps = (T)0,
       uint32_t max_itr = 0, uint32_t semantics = 0, uint32_t p_lo = 0,
       uint32_t col0 = 0, uint32_t col1 = 0,
       FlatPending<T, NP> pend = FlatPending<T, NP>{}, uint32_t gx2 = 0)
{
  constexpr int BLK = kBlock;
  // SPLIT (the overlapped exchange, sharded.py overlap=True): 1 = only the
  // columns [col0, col1) whose scales this rank computed itself, over the
  // ppr pieces starting at piece p_lo (no stats, no v update); 2 = every
  // other column of all pieces (with the stats when FS).  Lanes outside
  // their half are idle; col0 and col1 are multiples of W.
  // ALT: odd rounds walk the pieces from the end of the matrix, so a round
  // starts where the previous one finished (memory-side cache reuse)
  // FS: the first row group's workgroups (pieces 0..ppr-1, together all of
  // s_k) also fold m_k / stop_k into the state (stats_publish); the v update
  // then moves to k_parts, after m_k is known
  // R rows of one column piece per workgroup (the piece's column scales are
  // loaded once for the R rows)
  // U: chunks of BLK * W columns per piece, chunk u of a lane BLK * W
  // columns after chunk u - 1 (the element-wide path, W = 1, takes U =
  // 16 / sizeof(T) so that its pieces hold as many bytes as the vector
  // path's)
  // DS (deferred rounds, NP >= 0): whether the launch stores A_{k+1}, fixed
  // at compile time (1 / 0)
  // FLIP: the launch's cache policy (g_every_cache / g_defer_flip in
  // st_kernels.hip): bit 0 turns the matrix loads' policy over (cached <->
  // non-temporal), bit 1 the stores'; the shapes stay the form's
  // MF: the matrix-free round's sweep (launch k >= 1 of k_mfree's scheme,
  // with FS): `a` is A_0 (read only), `v` is v_{k-2}; each piece's partial
  // sum is Σ_c A_0[r][c] x[c] with x = v_{k-2} ∘ s_{k-1}, the first row
  // group folds round k-1's stats, nothing is stored; k_mparts finishes
  // s_k and v_{k-1}
  static_assert(!MF || (FS && NP < 0 && SPLIT == 0),
                "MF: the fused-stats unsplit round (gated on k - 1)");
  static_assert(NP < 0 || DS >= 0, "a deferred round's store is decided at compile time");
  // the matrix-free launch k evaluates round k - 1 (gated once end <= k - 1)
  const uint32_t kr = MF ? k - 1 : k;
  if (flat_gated(state, kr))
    return;
  using V = typename vec<T, W>::type;
  constexpr int NW = BLK / 64;
  constexpr uint32_t PWC = (uint32_t)BLK * W * U; // columns per piece
  __shared__ T red[NW][R];
  // a dispatch counts at most 2^32 - 1 work-items per grid dimension, so a
  // launch of more workgroups goes 2-D (gx2 = its row width, 0 = 1-D):
  // fold blockIdx.y back in and drop the padding (uniform per workgroup;
  // only huge matrices).  A kernel argument rather than gridDim.y, which
  // would put a dispatch-packet load in front of every workgroup's loads.
  uint32_t bl = blockIdx.x, nb;
  if (gx2 != 0) {
    bl += blockIdx.y * gx2;
    nb = flat_nblocks<R, PWC, SPLIT>(nrows, ncols, ppr, col0, col1);
    if (bl >= nb)
      return;
  } else {
    nb = gridDim.x;
  }
  const uint32_t b = (ALT != 0 && (k & 1u)) ? flat_reverse<ALT>(bl, nb) : bl;
  uint32_t rg, p;                                  // p: index into this row's parts
  if constexpr (SPLIT == 2) {
    // the pieces wholly inside [col0, col1) have nothing to do past row
    // group 0 (which takes the stats over every piece): the grid skips them
    uint32_t pa, nfull;
    split_full_pieces<PWC>(ncols, ppr, col0, col1, pa, nfull);
    if (b < ppr) {
      rg = 0;
      p = b;
    } else {
      const uint32_t pr = ppr - nfull, bb = b - ppr;
      rg = 1 + bb / pr;
      const uint32_t q = bb - (rg - 1) * pr;
      p = q < pa ? q : q + nfull;
    }
  } else if (SPLIT == 0 && pend.pt != 0) {
    // piece-tiled order: pt row groups of one piece run back to back (the
    // XCDs take every 8th), so the workgroups a CU runs in turn share the
    // piece's column scales - s_k and the pending rounds' - in its L1
    // instead of refetching them from L2 (deferred rounds; and the
    // every-round launch on non-temporal blocks, tiles of 4)
    const uint32_t pt = pend.pt, ng = (nrows + R - 1) / R;
    const uint32_t tile = b / (pt * ppr), t = b - tile * (pt * ppr);
    const uint32_t left = ng - tile * pt, g = left < pt ? left : pt;
    p = t / g;
    rg = tile * pt + (t - p * g);
  } else {
    rg = b / ppr;
    p = b - rg * ppr;
  }
  const uint32_t c0 = ((SPLIT == 1 ? p_lo + p : p) * (uint32_t)(BLK * U) + threadIdx.x) * W;
  const uint32_t r0 = rg * R;
  T acc[R];
  V x[U][R];
  T sr[R];
  bool in_cols[U], in[U]; // ncols % W == 0 on the vector path
#pragma unroll
  for (int u = 0; u < U; u++) {
    const uint32_t c = c0 + u * BLK * W;
    in_cols[u] = c < ncols;
    in[u] = in_cols[u] && (SPLIT == 0 || ((c >= col0 && c < col1) == (SPLIT == 1)));
  }
  // SPLIT == 0 loads without predicates: a row past the block reads the
  // block's last row and a column chunk past ncols the last chunk (valid
  // memory; their results are neither stored nor summed), so the element
  // math below runs unmasked - no exec-mask branches around the loads, no
  // v_cndmask per element and pending round
  // (only rounds with pending scalings gain: 1-2 % at NP = 2, 3 on 32768^2
  // fp64; the every-round and NP = 0 forms lose up to 3 %,
  // profiles/r02_flat_map_ab_*.log)
  constexpr bool UM = SPLIT == 0 && NP > 0 && ST_FLAT_UNMASKED;
  constexpr bool do_store = NP < 0 || DS == 1;
  // the deferred rounds' stores (probe switch ST_DEFER_STORE_NT: non-temporal
  // on cached blocks too)
  constexpr bool NTS = (NT || (NP >= 0 && ST_DEFER_STORE_NT)) != ((FLIP & 2) != 0);
  constexpr bool NTL = NT != ((FLIP & 1) != 0);
  uint32_t cl[U]; // the column each lane loads
#pragma unroll
  for (int u = 0; u < U; u++)
    cl[u] = (!UM || in_cols[u]) ? c0 + u * BLK * W : ncols - W;
  // the group's rows walked from one base pointer by the row pitch (no
  // per-row 64-bit multiply); rows past the block re-read its last row
  const size_t lda = (size_t)ncols; // row pitch
  const T* ap = a + (size_t)(r0 < nrows ? r0 : nrows - 1) * lda;
#pragma unroll
  for (int j = 0; j < R; j++) {
    acc[j] = (T)0;
    if constexpr (UM) {
#pragma unroll
      for (int u = 0; u < U; u++)
        x[u][j] = ld<V, NTL>(reinterpret_cast<const V*>(ap + cl[u]));
      if (r0 + j + 1 < nrows) // uniform
        ap += lda;
    } else {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (in[u] && r0 + j < nrows)
          x[u][j] = ld<V, NTL>(reinterpret_cast<V*>(a + (size_t)(r0 + j) * lda + c0 +
                                                   u * BLK * W));
    }
  }
  // the piece's column scales, issued with the matrix loads (the stats of
  // the first row group read them too)
  V sc[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    if (UM || in_cols[u])
      sc[u] = *reinterpret_cast<const V*>(s_cur + cl[u]);
  // matrix-free: x = v_{k-2} ∘ s_{k-1} for the piece's columns
  V xs[MF ? U : 1];
  if constexpr (MF) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (in_cols[u])
        xs[u] = *reinterpret_cast<const V*>(v + cl[u]) * sc[u];
  }
  // deferred writes: the pending rounds' column scales
  V sp_c[NP > 0 ? NP : 1][U];
  T sp_r[NP > 0 ? NP : 1][R]; // 1 / s_i[r]
  if constexpr (NP > 0) {
#pragma unroll
    for (int i = 0; i < NP; i++) {
#pragma unroll
      for (int u = 0; u < U; u++)
        if (UM || in_cols[u])
          sp_c[i][u] = *reinterpret_cast<const V*>(pend.s[i] + cl[u]);
    }
  }
  // then the row scales (vector loads, ld_row): s_k[r], or with deferred
  // writes already 1 / s_k[r], and the pending rounds' 1 / s_i[r]
  // A whole row group (every group but a ragged last one) loads its R
  // scales of a vector without per-row conditions, so that the scalar loads
  // of adjacent rows merge (s_load_dwordx4 ... x16: one load and one address
  // per vector instead of R).  fp64 rounds with 1 - 4 pending scalings only
  // (flat_map_sweep (round 2, git history) A/B, profiles/r02_rowload_merge_ab*.log: 32768^2
  // NP = 4, 8 rows, tiles of 16: 1.23 vs 1.29 ms; the storing round with 5
  // pending and fp32 lose 1 - 2 %, their merged scales crowd the SGPRs)
  const T* rs = NP >= 0 ? pend.inv_cur : s_cur;
  // (not the storing round with 5 pending: 2.895 vs 2.853 ms at 32768^2
  // fp64 with its store decision fixed at compile time too,
  // profiles/r03_store_probe_caps_nt.log "DS=1")
  constexpr bool kMergeRows = sizeof(T) == 8 && NP >= 1 && NP <= 4;
  if (kMergeRows && r0 + R <= nrows) { // uniform
#pragma unroll
    for (int j = 0; j < R; j++)
      sr[j] = ld_row(rs + row0 + r0 + j);
    if constexpr (NP > 0) {
#pragma unroll
      for (int i = 0; i < NP; i++) {
#pragma unroll
        for (int j = 0; j < R; j++)
          sp_r[i][j] = ld_row(pend.inv[i] + row0 + r0 + j);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < R; j++)
      sr[j] = r0 + j < nrows ? ld_row(rs + row0 + r0 + j) : (T)1;
    if constexpr (NP > 0) {
#pragma unroll
      for (int i = 0; i < NP; i++) {
#pragma unroll
        for (int j = 0; j < R; j++)
          sp_r[i][j] = r0 + j < nrows ? ld_row(pend.inv[i] + row0 + r0 + j) : (T)1;
      }
    }
  }
  if constexpr (FS) {
    if (rg == 0) { // uniform per workgroup
      __shared__ T mx_sh[NW];
      T mx = (T)0;
      int ok = 1;
#pragma unroll
      for (int u = 0; u < U; u++)
        if (in_cols[u])
          stats_at<T, W>(s_cur, sc[u], (c0 + u * BLK * W) / W, ncols,
                         semantics == ST_SEM_SYCL, eps, mx, ok);
      int fail = ok ? 0 : 1;
      mx = wave_max(mx);
      if ((threadIdx.x & 63) == 0)
        mx_sh[threadIdx.x >> 6] = mx;
      fail = __syncthreads_or(fail);
      if (threadIdx.x == 0) {
        T m = mx_sh[0];
#pragma unroll
        for (int w = 1; w < NW; w++)
          m = mx_sh[w] > m ? mx_sh[w] : m;
        stats_publish<T>(m, fail, ppr, s_cur, kr, max_itr, semantics, state);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < U && UM; u++) {
    // unmasked (see the loads): every lane and row computes; the stores
    // and the sums take the block's own elements only
    if constexpr (NP > 0) {
#pragma unroll
      for (int i = 0; i < NP; i++) {
#pragma unroll
        for (int j = 0; j < R; j++) {
          const T inv = sp_r[i][j];
          if constexpr (ORDER == 0)
            x[u][j] = x[u][j] * (inv * sp_c[i][u]);
          else
            x[u][j] = (inv * x[u][j]) * sp_c[i][u];
        }
      }
    }
    T* wp = a + (size_t)r0 * lda + c0 + u * BLK * W; // row r0 + j after j pitches
#pragma unroll
    for (int j = 0; j < R; j++) {
      const T inv = NP >= 0 ? sr[j] : (T)1 / sr[j];
      V y;
      if constexpr (ORDER == 0)
        y = x[u][j] * (inv * sc[u]); // cpp:324-325
      else
        y = (inv * x[u][j]) * sc[u]; // main.py:13-16
      if (do_store && in_cols[u] && r0 + j < nrows)
        st<V, NTS>(reinterpret_cast<V*>(wp), y);
      wp += lda;
      const T h = in_cols[u] ? hsum<T, W>(y) : (T)0;
      acc[j] = u == 0 ? h : acc[j] + h;
    }
  }
#pragma unroll
  for (int u = 0; u < U && !UM; u++) {
    if (!in[u])
      continue;
    if constexpr (NP > 0) {
      // A_j -> A_k: the pending rounds' element updates, as they ran
#pragma unroll
      for (int i = 0; i < NP; i++) {
#pragma unroll
        for (int j = 0; j < R; j++) {
          if (r0 + j < nrows) {
            const T inv = sp_r[i][j];
            if constexpr (ORDER == 0)
              x[u][j] = x[u][j] * (inv * sp_c[i][u]);
            else
              x[u][j] = (inv * x[u][j]) * sp_c[i][u];
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < R; j++) {
      if (r0 + j < nrows) {
        if constexpr (MF) {
          // A_0[r][c] x[c], fused, the lane's columns in order
          if constexpr (W == 1) {
            acc[j] = __builtin_fma(x[u][j], xs[u], acc[j]);
          } else {
#pragma unroll
            for (int i = 0; i < W; i++)
              acc[j] = __builtin_fma(x[u][j][i], xs[u][i], acc[j]);
          }
          continue;
        }
        const T inv = NP >= 0 ? sr[j] : (T)1 / sr[j];
        V y;
        if constexpr (ORDER == 0)
          y = x[u][j] * (inv * sc[u]); // cpp:324-325
        else
          y = (inv * x[u][j]) * sc[u]; // main.py:13-16
        if (do_store)
          st<V, NTS>(reinterpret_cast<V*>(a + (size_t)(r0 + j) * lda + c0 + u * BLK * W),
                    y);
        acc[j] = u == 0 ? hsum<T, W>(y) : acc[j] + hsum<T, W>(y);
      }
    }
  }
  if (!FS && SPLIT == 0 && p == 0 && threadIdx.x < R && r0 + threadIdx.x < nrows) {
    // v[r] *= s_k[r] / m_k (cpp:260), m_k from k_stats
    const uint32_t r = row0 + r0 + threadIdx.x;
    const T m = (T)state->max;
    v[r] = v[r] * (s_cur[r] / m);
  }
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // the wave sums stay in lanes 62 / 63 (no broadcast), which write them:
  // rows in pairs through one tree (wave_sum_pair), an odd last row alone
#pragma unroll
  for (int j = 0; j + 1 < R; j += 2) {
    const T t = wave_sum_pair(acc[j], acc[j + 1]);
    if (lane >= 62)
      red[wave][j + (lane - 62)] = t;
  }
  if constexpr (R % 2 == 1) {
    const T t = wave_sum_l63(acc[R - 1]);
    if (lane == 63)
      red[wave][R - 1] = t;
  }
  __syncthreads();
  if (threadIdx.x < R && r0 + threadIdx.x < nrows) {
    T t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; w++)
      t += red[w][threadIdx.x];
    part[(size_t)(r0 + threadIdx.x) * ppr + p] = t;
  }
}

// K0 in the flat form, s_0 = A_0 1 (similarity_transform.cpp:40, the first
// sum_across_rows before the loop's first stop test) for blocks where the
// flat round pays: one short workgroup per (R rows, column piece) writes the
// piece's partial sums, k_parts then sums each row's pieces in a fixed order
// - deterministic and independent of the row partition, as the rounds' row
// sums are.  Read-only and ungated: the loads and walk order of the deferred
// form's read-only round with nothing pending (pt: tiles of pt row groups per
// piece, 0 = row-major), without its scaling.  Replaces the grid-stride
// k_fused launch, which streamed the same bytes at 0.77 / 0.83 of 8 TB/s
// (8192^2 / 32768^2 fp64) where the flat read-only round ran 0.88 / 0.90.
// rev: walk the pieces from the end of the block (an odd round's order,
// flat_reverse<2>): on a cacheable block just written front to back (a
// generator, the drop-in's host copy) the walk starts on what the memory-side
// cache still holds, and leaves the block's start there for round 0.
template <typename T, int W, bool NT, int R, int U, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void
k_flat_sum(const T* __restrict__ a, T* __restrict__ part, uint32_t nrows,
           uint32_t ncols, uint32_t ppr, uint32_t pt, uint32_t gx2, uint32_t rev)
{
  using V = typename vec<T, W>::type;
  constexpr int NW = BLK / 64;
  __shared__ T red[NW][R];
  const uint32_t ng = (nrows + R - 1) / R;
  uint32_t b = blockIdx.x, nb = gridDim.x;
  if (gx2 != 0) { // a 2-D grid (k_flat's gx2): fold blockIdx.y back in
    b += blockIdx.y * gx2;
    nb = ng * ppr;
    if (b >= nb)
      return;
  }
  if (rev)
    b = flat_reverse<2>(b, nb);
  uint32_t rg, p;
  if (pt != 0) { // pt row groups of one piece back to back (k_flat's order)
    const uint32_t tile = b / (pt * ppr), t = b - tile * (pt * ppr);
    const uint32_t left = ng - tile * pt, g = left < pt ? left : pt;
    p = t / g;
    rg = tile * pt + (t - p * g);
  } else {
    rg = b / ppr;
    p = b - rg * ppr;
  }
  const uint32_t c0 = (p * (uint32_t)(BLK * U) + threadIdx.x) * W;
  const uint32_t r0 = rg * R;
  const size_t lda = (size_t)ncols;
  V x[U][R];
#pragma unroll
  for (int j = 0; j < R; j++) {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (c0 + u * BLK * W < ncols && r0 + j < nrows)
        x[u][j] = ld<V, NT>(reinterpret_cast<const V*>(a + (size_t)(r0 + j) * lda + c0 +
                                                       u * BLK * W));
  }
  T acc[R];
#pragma unroll
  for (int j = 0; j < R; j++) {
    acc[j] = (T)0;
#pragma unroll
    for (int u = 0; u < U; u++)
      if (c0 + u * BLK * W < ncols && r0 + j < nrows)
        acc[j] = u == 0 ? hsum<T, W>(x[u][j]) : acc[j] + hsum<T, W>(x[u][j]);
  }
  // the wave sums land in lanes 62 / 63 (k_flat's trees), then the waves'
  // sums in wave order
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j + 1 < R; j += 2) {
    const T t = wave_sum_pair(acc[j], acc[j + 1]);
    if (lane >= 62)
      red[wave][j + (lane - 62)] = t;
  }
  if constexpr (R % 2 == 1) {
    const T t = wave_sum_l63(acc[R - 1]);
    if (lane == 63)
      red[wave][R - 1] = t;
  }
  __syncthreads();
  if (threadIdx.x < R && r0 + threadIdx.x < nrows) {
    T t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < NW; w++)
      t += red[w][threadIdx.x];
    part[(size_t)(r0 + threadIdx.x) * ppr + p] = t;
  }
}

// The solve loops' per-batch look at the state: one wave copies the 64 B
// st_state into the caller's pinned, host-coherent slot with vector stores
// (16 lanes, one word each), in stream order behind the batch's rounds.  It
// replaces a device-to-host copy on the stream, a blit launch whose own
// dispatch gaps cost ~20 us per batch (rocprofv3 trace of the whole solves,
// profiles/r03_state_mirror_*.log).
__global__ __launch_bounds__(64) void
k_state_mirror(const uint32_t* __restrict__ d, uint32_t* h)
{
  const uint32_t i = threadIdx.x;
  if (i < (uint32_t)(sizeof(st_state) / 4))
    __hip_atomic_store(&h[i], d[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The matrix-free round's second launch (after k_flat<..., MF>): one wave
// per row sums its pieces in k_parts' order, s_k[r] = Σ / x[r] with
// x[r] = v_{k-2}[r] s_{k-1}[r] (k_mfree's quotient); the blocks past the
// rows write v_{k-1} = v_{k-2} ∘ (s_{k-1} / m_{k-1}) over ALL n entries
// (every rank of a sharded solve keeps the whole v), m_{k-1} as k_flat's
// first row group published it.  Gated like launch k (end < k).
template <typename T, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void
k_mparts(const T* __restrict__ part, T* __restrict__ s_next, uint32_t nrows,
         uint32_t ppr, uint32_t k, const st_state* state, const T* __restrict__ s_prev,
         const T* __restrict__ v_prev, T* __restrict__ v_cur, uint32_t row0, uint32_t n,
         uint32_t row_blocks)
{
  const uint32_t e = state->end; // plain load: as k_parts
  if (e != 0 && e < k)
    return;
  if (blockIdx.x >= row_blocks) {
    const T m = (T)state->max;
    const uint32_t nb = gridDim.x - row_blocks;
    for (uint32_t i = (blockIdx.x - row_blocks) * BLK + threadIdx.x; i < n; i += nb * BLK)
      v_cur[i] = v_prev[i] * (s_prev[i] / m); // cpp:260
    return;
  }
  const uint32_t r = (blockIdx.x * BLK + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (r >= nrows)
    return; // whole waves leave together
  const T* row = part + (size_t)r * ppr;
  T acc = (T)0;
  for (uint32_t p = lane; p < ppr; p += 64)
    acc += row[p];
  acc = wave_sum(acc);
  if (lane == 0)
    s_next[r] = acc / (v_prev[row0 + r] * s_prev[row0 + r]);
}

// k_parts for rows of at most LPR (16 or 32) partials: 64 / LPR rows per
// wave, LPR lanes each (4x / 2x fewer waves than k_parts).  Bitwise
// k_parts' sums: in k_parts' one-row wave the lanes past ppr hold 0, so its
// rows of 16 (LPR = 16) or half-waves (LPR = 32) past the first carry 0 and
// the tree's later steps add exact zeros - lane 15 after the row_ror steps
// (LPR = 16) / lane 31 after row_bcast 15 (LPR = 32) already holds
// wave_sum's value, bit for bit.  Here those segments hold other rows, and
// the tree stops there.
template <typename T, int LPR, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void
k_parts_seg(const T* __restrict__ part, T* __restrict__ s_next, uint32_t nrows,
            uint32_t ppr /* <= LPR */, uint32_t k, const st_state* state,
            const T* __restrict__ s_cur, T* __restrict__ v, uint32_t row0,
            T* __restrict__ inv_next)
{
  static_assert(LPR == 16 || LPR == 32, "segments of 16 or 32 lanes");
  const uint32_t seg = threadIdx.x % LPR;
  const uint32_t r = (blockIdx.x * BLK + threadIdx.x) / LPR;
  // whole waves stay together (DPP reads neighbours): rows past the block
  // compute on zeros and store nothing
  const bool live = r < nrows;
  const uint32_t e = state != nullptr ? state->end : 0u; // no state: K0, ungated
  T vr = (T)0, sr = (T)1, m = (T)1;
  if (v != nullptr && seg == LPR - 1 && live) {
    vr = v[row0 + r];
    sr = s_cur[row0 + r];
    m = (T)state->max;
  }
  T x = (live && seg < ppr) ? part[(size_t)r * ppr + seg] : (T)0;
  x += dpp_mov<0xB1>(x);       // quad_perm [1,0,3,2]
  x += dpp_mov<0x4E>(x);       // quad_perm [2,3,0,1]
  x += dpp_mov<0x124>(x);      // row_ror 4
  x += dpp_mov<0x128>(x);      // row_ror 8
  if constexpr (LPR == 32)
    x += dpp_mov<0x142, 0xa>(x); // row_bcast 15 (rows 1 and 3)
  if (e != 0 && e <= k)
    return;
  if (seg == LPR - 1 && live) {
    s_next[r] = x;
    if (inv_next != nullptr)
      inv_next[r] = (T)1 / x;
    if (v != nullptr)
      v[row0 + r] = vr * (sr / m); // cpp:260
  }
}

template <typename T, int BLK = kBlock>
__global__ __launch_bounds__(BLK) void
k_parts(const T* __restrict__ part, T* __restrict__ s_next, uint32_t nrows,
        uint32_t ppr /* partials per row */, uint32_t k, const st_state* state,
        const T* __restrict__ s_cur = nullptr, T* __restrict__ v = nullptr,
        uint32_t row0 = 0, const T* __restrict__ part2 = nullptr,
        uint32_t ppr2 = 0, uint32_t skip0 = 0, uint32_t nskip = 0,
        T* __restrict__ inv_next = nullptr)
{
  // [skip0, skip0 + nskip): parts of `part` not written (split round)
  // part2 (split round): the local half's partials, added after part's
  // v != nullptr: also v[r] *= s_k[r] / m_k (cpp:260) with m_k published by
  // k_flat's first row group
  // inv_next != nullptr (deferred writes): also 1 / s_{k+1}[r]
  // Every load is issued before the gate is tested (they are in bounds
  // whatever the gate says; only the stores depend on it), so the launch
  // waits for one memory round trip after its arguments instead of three
  // in a row: the gate, the partials, then m_k / s_k / v.  The gate is a
  // plain (scalar) load, as in k_flat (flat_gated): `end` only changes
  // inside the k_flat launch before this one.
  const uint32_t r = (blockIdx.x * BLK + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  if (r >= nrows)
    return; // whole waves leave together
  const uint32_t e = state != nullptr ? state->end : 0u; // no state: K0, ungated
  T vr = (T)0, sr = (T)1, m = (T)1;
  if (v != nullptr && lane == 0) {
    vr = v[row0 + r];
    sr = s_cur[row0 + r];
    m = (T)state->max;
  }
  const T* row = part + (size_t)r * ppr;
  T acc = (T)0;
  for (uint32_t p = lane; p < ppr; p += 64)
    if (p - skip0 >= nskip)
      acc += row[p];
  acc = wave_sum(acc);
  if (part2 != nullptr) {
    const T* row2 = part2 + (size_t)r * ppr2;
    T acc2 = (T)0;
    for (uint32_t p = lane; p < ppr2; p += 64)
      acc2 += row2[p];
    acc += wave_sum(acc2);
  }
  if (e != 0 && e <= k)
    return;
  if (lane == 0) {
    s_next[r] = acc;
    if (inv_next != nullptr)
      inv_next[r] = (T)1 / acc;
    if (v != nullptr)
      v[row0 + r] = vr * (sr / m); // cpp:260
  }
}

// inv[i] = 1 / s[i] (the reciprocals of s_0 for deferred writes)
template <typename T>
__global__ __launch_bounds__(kBlock) void
k_recip(const T* __restrict__ s, T* __restrict__ inv, uint32_t n)
{
  for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n;
       i += gridDim.x * kBlock)
    inv[i] = (T)1 / s[i];
}

// ---------------------------------------------------------------------------
// matrix-free round: the same iteration without ever
// writing the matrix.  With v the eigenvector accumulator, the transformed
// matrix of round k is A_k = X^-1 A_0 X for X = diag(x), x ∝ Π_{j<k} s_j,
// so its row sums are s_k = (A_0 x) ⊘ x (scale-invariant in x).  Launch k
// (k >= 1; launch 0 is the plain row-sum pass) therefore:
//   * derives m_{k-1}, stop_{k-1} from s_{k-1} (every workgroup, as k_round)
//   * writes v_{k-1} = v_{k-2} * (s_{k-1} / m_{k-1})   (ALL n entries, split
//     over the workgroups: every rank of a sharded solve keeps the full v)
//   * computes s_k[r] = (Σ_c A_0[r][c] x[c]) / x[r] for its rows with
//     x = v_{k-2} ∘ s_{k-1} (∝ v_{k-1}: no division in the sweep)
// and records round k-1 in `state` (end = k when round k-1 stops).  Launch
// j exits at once if end != 0 && end < j.  A_0 is read once per round:
// N^2*b bytes instead of the transform's 2*N^2*b.
// ---------------------------------------------------------------------------
template <typename T, int R, int W, int U, bool NT, int BLK, bool STATS>
__device__ __forceinline__ void
mfree_group(const T* a0, const T* __restrict__ s_prev,
            const T* __restrict__ v_prev, T* __restrict__ s_next,
            uint32_t rbase, uint32_t ncols, uint32_t row0, bool cyclic, T eps,
            T& mx, int& ok, T (*red)[4])
{
  using V = typename vec<T, W>::type;
  const uint32_t nv = ncols / W;
  const V* sv = reinterpret_cast<const V*>(s_prev);
  const V* vv = reinterpret_cast<const V*>(v_prev);
  const V* rows[R];
  T acc[R];
#pragma unroll
  for (int j = 0; j < R; j++) {
    rows[j] = reinterpret_cast<const V*>(a0 + (size_t)(rbase + j) * ncols);
    acc[j] = (T)0;
  }
  auto body = [&](uint32_t c, auto ucount) {
    constexpr int UU = decltype(ucount)::value;
    V x[UU][R];
    V sc[UU], xs[UU];
#pragma unroll
    for (int u = 0; u < UU; u++)
#pragma unroll
      for (int j = 0; j < R; j++)
        x[u][j] = ld<V, NT>(rows[j] + c + u * BLK);
#pragma unroll
    for (int u = 0; u < UU; u++) {
      sc[u] = sv[c + u * BLK];
      xs[u] = vv[c + u * BLK] * sc[u];
    }
    if constexpr (STATS) {
#pragma unroll
      for (int u = 0; u < UU; u++) {
        const uint32_t q = c + u * BLK;
        T e[W + 1];
        if constexpr (W == 1) {
          e[0] = sc[u];
        } else {
#pragma unroll
          for (int i = 0; i < W; i++)
            e[i] = sc[u][i];
        }
        const uint32_t nxt = (q + 1) * W;
        const bool has_next = nxt < ncols || cyclic;
        e[W] = s_prev[nxt < ncols ? nxt : 0];
#pragma unroll
        for (int i = 0; i < W; i++) {
          mx = e[i] > mx ? e[i] : mx;
          if (i < W - 1 || has_next) {
            const T d = e[i] - e[i + 1];
            ok &= (d < (T)0 ? -d : d) < eps ? 1 : 0;
          }
        }
      }
    }
#pragma unroll
    for (int u = 0; u < UU; u++)
#pragma unroll
      for (int j = 0; j < R; j++) {
        if constexpr (W == 1) {
          acc[j] = __builtin_fma(x[u][j], xs[u], acc[j]);
        } else {
#pragma unroll
          for (int i = 0; i < W; i++)
            acc[j] = __builtin_fma(x[u][j][i], xs[u][i], acc[j]);
        }
      }
  };
  uint32_t c = threadIdx.x;
  for (; c + (U - 1) * BLK < nv; c += U * BLK)
    body(c, std::integral_constant<int, U>{});
  sweep_tail<U, BLK>(c, nv, body);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < R; j++) {
    T t = wave_sum(acc[j]);
    if (lane == 0)
      red[wave][j] = t;
  }
  __syncthreads();
  if (threadIdx.x < R) {
    T t = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < BLK / 64; w++)
      t += red[w][threadIdx.x];
    const uint32_t r = row0 + rbase + threadIdx.x;
    s_next[rbase + threadIdx.x] = t / (v_prev[r] * s_prev[r]);
  }
  __syncthreads();
}

template <typename T, int ROWS, int W, int U, bool NT, int BLK = kBlock,
          bool ALT = false>
__global__ __launch_bounds__(BLK) void
k_mfree(const T* a0, const T* __restrict__ s_prev, T* __restrict__ s_next,
        const T* __restrict__ v_prev, T* __restrict__ v_cur, uint32_t ng_main,
        uint32_t nrem, uint32_t ncols, uint32_t row0, T eps, uint32_t k,
        uint32_t max_itr, uint32_t semantics, st_state* state)
{
  static_assert(ROWS <= 4, "red[] holds 4 rows");
  {
    const uint32_t e =
      __hip_atomic_load(&state->end, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e != 0 && e < k)
      return;
  }
  __shared__ T red[BLK / 64][4];
  __shared__ T mx_sh[BLK / 64];
  __shared__ T m_sh;
  const bool cyclic = semantics == ST_SEM_SYCL;
  const uint32_t ngroups = ng_main + nrem;
  T mx = (T)0;
  int ok = 1;
  T dmx = 0;
  int dok = 1;
  const uint32_t cnt = // as k_round
    blockIdx.x < ngroups ? (ngroups - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const bool rev = ALT && (k & 1u);
  for (uint32_t i = 0; i < cnt; i++) {
    const bool first = i == 0;
    const uint32_t g = blockIdx.x + (rev ? cnt - 1 - i : i) * gridDim.x;
    if (g < ng_main) {
      if (first)
        mfree_group<T, ROWS, W, U, NT, BLK, true>(a0, s_prev, v_prev, s_next,
                                                  g * ROWS, ncols, row0,
                                                  cyclic, eps, mx, ok, red);
      else
        mfree_group<T, ROWS, W, U, NT, BLK, false>(a0, s_prev, v_prev, s_next,
                                                   g * ROWS, ncols, row0,
                                                   cyclic, eps, dmx, dok, red);
    } else {
      const uint32_t rb = ng_main * ROWS + (g - ng_main);
      if (first)
        mfree_group<T, 1, W, U, NT, BLK, true>(a0, s_prev, v_prev, s_next, rb,
                                               ncols, row0, cyclic, eps, mx, ok,
                                               red);
      else
        mfree_group<T, 1, W, U, NT, BLK, false>(a0, s_prev, v_prev, s_next, rb,
                                                ncols, row0, cyclic, eps, dmx,
                                                dok, red);
    }
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0)
    mx_sh[threadIdx.x >> 6] = mx;
  const int stop = __syncthreads_and(ok);
  if (threadIdx.x == 0) {
    T m = mx_sh[0];
#pragma unroll
    for (int w = 1; w < BLK / 64; w++)
      m = mx_sh[w] > m ? mx_sh[w] : m;
    m_sh = m;
  }
  __syncthreads();
  const T m = m_sh;
  // v_{k-1} = v_{k-2} * (s_{k-1} / m_{k-1}) over the FULL vector (cpp:260)
  {
    const uint32_t per = (ncols + gridDim.x - 1) / gridDim.x;
    const uint32_t lo = blockIdx.x * per;
    const uint32_t hi = lo + per < ncols ? lo + per : ncols;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += BLK)
      v_cur[i] = v_prev[i] * (s_prev[i] / m);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t rk = k - 1; // the round evaluated by this launch
    state->lambda = (double)s_prev[0];
    state->max = (double)m;
    state->stop = stop ? 1u : 0u;
    state->round = rk;
    if (stop) {
      state->iters = semantics == ST_SEM_SYCL ? rk : rk + 1;
      state->end = k;
      state->done = 1u;
    } else if (k >= max_itr) {
      state->iters = max_itr;
      state->end = k;
      state->done = 1u;
    }
  }
}

// ---------------------------------------------------------------------------
// round epilogue: one workgroup over the full row-sum vector
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(kEpiBlock) void
k_epilogue(const T* __restrict__ s, T* __restrict__ v, uint32_t n, T eps,
           uint32_t max_itr, uint32_t semantics, st_state* __restrict__ state)
{
  if (state->done)
    return;
  __shared__ T red[kEpiBlock / 64];
  __shared__ T m_sh;
  const bool cyclic = semantics == ST_SEM_SYCL;
  const uint32_t last = cyclic ? n : n - 1;

  T mx = (T)0; // find_max starts from 0 (similarity_transform.cpp:185)
  int ok = 1;
  for (uint32_t i = threadIdx.x; i < n; i += kEpiBlock) {
    const T x = s[i];
    mx = x > mx ? x : mx;
    if (i < last) {
      const T d = x - s[i + 1 == n ? 0 : i + 1];
      ok &= (d < (T)0 ? -d : d) < eps ? 1 : 0; // cpp:419-421; NaN fails
    }
  }
  mx = wave_max(mx);
  if ((threadIdx.x & 63) == 0)
    red[threadIdx.x >> 6] = mx;
  const int all_ok = __syncthreads_and(ok);
  if (threadIdx.x == 0) {
    T m = red[0];
    for (int w = 1; w < kEpiBlock / 64; w++)
      m = red[w] > m ? red[w] : m;
    m_sh = m;
  }
  __syncthreads();
  const T m = m_sh;
  if (v != nullptr)
    for (uint32_t i = threadIdx.x; i < n; i += kEpiBlock)
      v[i] = v[i] * (s[i] / m); // similarity_transform.cpp:260

  if (threadIdx.x == 0) {
    const uint32_t i = state->round; // break index if this round stops
    state->lambda = (double)s[0];    // cpp:60-65
    state->max = (double)m;
    state->stop = all_ok ? 1u : 0u;
    if (all_ok) {
      state->iters = semantics == ST_SEM_SYCL ? i : i + 1; // cpp:54 / py:47
      state->done = 1u;
    } else {
      state->round = i + 1;
      if (i + 1 >= max_itr) { // loop exhausted (cpp:39,54)
        state->iters = max_itr;
        state->done = 1u;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// generators and fill
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t
splitmix(uint64_t seed, uint64_t idx)
{
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

template <typename T>
__device__ __forceinline__ T
uniform01(uint64_t z);
template <>
__device__ __forceinline__ double
uniform01<double>(uint64_t z)
{
  return (double)((z >> 11) + 1) * 0x1.0p-53;
}
template <>
__device__ __forceinline__ float
uniform01<float>(uint64_t z)
{
  return (float)((z >> 40) + 1) * 0x1.0p-24f;
}

enum GenKind
{
  kHilbert = 0,
  kRandom = 1,
  kIdentity = 2
};

template <typename T, int KIND>
__global__ __launch_bounds__(kBlock) void
k_generate(T* __restrict__ a, uint32_t nrows, uint32_t ncols, uint32_t row0,
           uint64_t seed)
{
  for (uint32_t r = blockIdx.x; r < nrows; r += gridDim.x) {
    const uint64_t gr = (uint64_t)row0 + r;
    T* row = a + (size_t)r * ncols;
    for (uint32_t c = threadIdx.x; c < ncols; c += kBlock) {
      T x;
      if constexpr (KIND == kHilbert)
        x = (T)1 / (T)(gr + c + 1); // utils.cpp:150
      else if constexpr (KIND == kRandom)
        x = uniform01<T>(splitmix(seed, gr * ncols + c));
      else
        x = (gr == c) ? (T)1 : (T)0; // utils.cpp:5-27
      row[c] = x;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void
k_fill(T* __restrict__ x, uint64_t count, T value)
{
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < count;
       i += (uint64_t)gridDim.x * kBlock)
    x[i] = value;
}

// ---------------------------------------------------------------------------
// the whole solve in ONE workgroup, for matrices that fit its registers
// (N <= 64*W: 128 fp64, 256 fp32; N % W == 0)
//
// A small solve is launch-bound: ~10 rounds of a few microseconds of work,
// each a launch plus the host's batch checks.  Here 16 waves keep the
// matrix in VGPRs for the whole iteration (row r on wave r % 16, lane l
// holding its 16-byte chunk l; at most 16 fp64 or 64 fp32 values per lane),
// s and v in LDS, and run every round back to back with workgroup barriers
// only.  Each round computes exactly what k_round computes, bit for bit:
//   row sums   hsum of the lane's chunk, then wave_sum over the 64 lanes
//              (k_round / k_fused: a single chunk per lane at these sizes,
//              the other waves' zeros add nothing)
//   m_k, stop  max from 0 and the (cyclic) pair test over s_k
//   v          v[r] * (s_k[r] / m_k)
//   transform  x * ((1/s_r) * s_c)  (or ((1/s_r) * x) * s_c, main.py)
// and, like k_round, the stopping (or last) round still transforms and
// sums, so the final matrix equals the per-round loop's.  The matrix, v and
// the state are written back at the end; s_k is not.
// ---------------------------------------------------------------------------
constexpr int kSmallBlock = 1024; // 16 waves
constexpr int kSmallWaves = kSmallBlock / 64;

template <typename T>
constexpr uint32_t
small_solve_max_n()
{
  return 64u * (16u / sizeof(T));
}

template <typename T, int ORDER, int RPW>
__global__ __launch_bounds__(kSmallBlock) void
k_solve_small(T* a, T* __restrict__ v_out, uint32_t n, T eps, uint32_t max_itr,
              uint32_t semantics, st_state* state)
{
  // RPW: rows per wave, the power of two >= ceil(n / 16) (the launcher
  // picks the instantiation; rows r = wave + 16 i past n are zeros)
  constexpr int W = 16 / sizeof(T);
  constexpr uint32_t NMAX = small_solve_max_n<T>();
  static_assert(RPW * kSmallWaves <= (int)NMAX, "rows per wave");
  using V = typename vec<T, W>::type;
  __shared__ V s_sh[2][NMAX / W];
  __shared__ T v_sh[NMAX];
  __shared__ T inv_sh[NMAX]; // 1 / s_k[r], once per row instead of per lane
  __shared__ T mx_sh[kSmallWaves];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nv = n / W; // chunks per row
  const bool has = lane < nv;
  const bool cyclic = semantics == ST_SEM_SYCL;
  T* s0 = reinterpret_cast<T*>(s_sh[0]);
  T* s1 = reinterpret_cast<T*>(s_sh[1]);

  V x[RPW];
  T t[RPW];
#pragma unroll
  for (int i = 0; i < RPW; i++) {
    const uint32_t r = wave + kSmallWaves * i;
    if (has && r < n)
      x[i] = *reinterpret_cast<const V*>(a + (size_t)r * n + lane * W);
    else
      x[i] = (V)(T)0;
  }
  // K0: s_0 = rowsum(A_0)
#pragma unroll
  for (int i = 0; i < RPW; i++)
    t[i] = has ? hsum<T, W>(x[i]) : (T)0;
  wave_sum_rows<T, RPW>(t);
  if (lane == 63) {
#pragma unroll
    for (int i = 0; i < RPW; i++)
      if (wave + kSmallWaves * i < n)
        s0[wave + kSmallWaves * i] = t[i];
  }
  if (threadIdx.x < n)
    v_sh[threadIdx.x] = (T)1; // initialise_eigen_vector (cpp:34)

  T* sc_ = s0;
  T* sn_ = s1;
  uint32_t k = 0;
  for (;; k++) {
    __syncthreads(); // s_k complete
    // m_k and stop_k (find_max starts from 0, cpp:185; cpp:413-421)
    T mx = (T)0;
    int ok = 1;
    if (threadIdx.x < n) {
      const T e0 = sc_[threadIdx.x];
      inv_sh[threadIdx.x] = (T)1 / e0;
      mx = e0 > mx ? e0 : mx;
      const uint32_t nx = threadIdx.x + 1;
      if (nx < n || cyclic) {
        const T d = e0 - sc_[nx < n ? nx : 0];
        ok = (d < (T)0 ? -d : d) < eps ? 1 : 0;
      }
    }
    mx = wave_max(mx);
    if (lane == 0)
      mx_sh[wave] = mx;
    const int stop = __syncthreads_and(ok);
    T m = mx_sh[0];
#pragma unroll
    for (int w = 1; w < kSmallWaves; w++)
      m = mx_sh[w] > m ? mx_sh[w] : m;
    if (threadIdx.x < n) // cpp:260
      v_sh[threadIdx.x] = v_sh[threadIdx.x] * (sc_[threadIdx.x] / m);
    const bool last = stop || k + 1 >= max_itr;
    if (last && threadIdx.x == 0) {
      state->lambda = (double)sc_[0]; // cpp:60-65
      state->max = (double)m;
      state->stop = stop ? 1u : 0u;
      state->round = k;
      state->iters = stop ? (semantics == ST_SEM_SYCL ? k : k + 1) : max_itr;
      state->end = k + 1;
      state->done = 1u;
    }
    // A_{k+1} = D_k^-1 A_k D_k and s_{k+1} (as k_round, also in the last round)
    const V sc = has ? reinterpret_cast<const V*>(sc_)[lane] : (V)(T)1;
#pragma unroll
    for (int i = 0; i < RPW; i++) {
      const uint32_t r = wave + kSmallWaves * i;
      const T inv = r < n ? inv_sh[r] : (T)1;
      if constexpr (ORDER == 0)
        x[i] = x[i] * (inv * sc); // cpp:324-325
      else
        x[i] = (inv * x[i]) * sc; // main.py:13-16
      t[i] = has ? hsum<T, W>(x[i]) : (T)0;
    }
    wave_sum_rows<T, RPW>(t);
    if (lane == 63) {
#pragma unroll
      for (int i = 0; i < RPW; i++)
        if (wave + kSmallWaves * i < n)
          sn_[wave + kSmallWaves * i] = t[i];
    }
    T* tmp = sc_;
    sc_ = sn_;
    sn_ = tmp;
    if (last)
      break;
  }
  // write back: the transformed matrix and v
#pragma unroll
  for (int i = 0; i < RPW; i++) {
    const uint32_t r = wave + kSmallWaves * i;
    if (has && r < n)
      *reinterpret_cast<V*>(a + (size_t)r * n + lane * W) = x[i];
  }
  __syncthreads();
  if (threadIdx.x < n)
    v_out[threadIdx.x] = v_sh[threadIdx.x];
}

} // namespace dev
} // namespace st
