// st_kernels.hip — launchers for the gfx950 kernels in st_device.h and the
// step-level C-ABI (similarity_transform.h layer 4).
//
// Launch shapes:
//   fused scale+rowsum / rowsum : 256-thread workgroups, ROWS rows each,
//                                 16-byte accesses, U chunks in flight;
//                                 remainder rows (nrows % ROWS) in a second
//                                 launch with ROWS = 1
//   epilogue                    : one 1024-thread workgroup
//   generators / fill           : grid-stride, 256-thread workgroups

#include <hip/hip_runtime.h>

#include <cstring>
#include <stdint.h>

#include <atomic>

#include "st_device.h"
#include "st_internal.h"

#ifndef ST_TUNING_ABI
#define ST_TUNING_ABI 0
#endif
#if ST_TUNING_ABI
#include "st_tuning.h"
#endif

// A/B probe switches of the launch shapes (st_device.h has those of the
// kernel code: ST_DPP_NOINIT, ST_ROW_VLOAD, ST_FLAT_UNMASKED,
// ST_DEFER_STORE_NT).  A probe build of the library (`make probe
// PROBE="-DST_FLAT_ALT=0"`, eigen_value_amd/lib/variants/) passes
// -DST_PROBES=1 with other values; a library build with any other value
// fails here, and st_version() names the switches a probe build was made with.
#ifndef ST_EVERY_CACHED_R1 // 0 = round 2's 2 rows, row-major
#define ST_EVERY_CACHED_R1 1
#endif
#ifndef ST_DEFER_R0_CACHED // rows of the cached fp64 NP = 0 round (1, 2, 4)
#define ST_DEFER_R0_CACHED 1
#endif
#ifndef ST_DEFER_PT0_CACHED // its piece tile (0 = row-major)
#define ST_DEFER_PT0_CACHED 4u
#endif
#ifndef ST_DEFER_STORE_R8_CACHED // 8 rows for the cached fp64 5-pending store
#define ST_DEFER_STORE_R8_CACHED 1
#endif
#ifndef ST_DEFER_TS5_CACHED // its piece tile (row groups; 0 = row-major)
#define ST_DEFER_TS5_CACHED 16u
#endif
#ifndef ST_FLAT_ALT // the flat launches' odd-round order (2 = reversed per XCD, 0 = none)
#define ST_FLAT_ALT 2
#endif
#define ST_PROBES_DEFAULT                                                      \
  (ST_DPP_NOINIT == 1 && ST_ROW_VLOAD == 0 && ST_FLAT_UNMASKED == 1 &&         \
   ST_DEFER_STORE_NT == 0 && ST_EVERY_CACHED_R1 == 1 &&                        \
   ST_DEFER_R0_CACHED == 1 && ST_DEFER_PT0_CACHED == 4 &&                      \
   ST_DEFER_STORE_R8_CACHED == 1 && ST_DEFER_TS5_CACHED == 16 && ST_FLAT_ALT == 2)
#ifndef ST_PROBES
static_assert(ST_PROBES_DEFAULT,
              "A/B probe switch set in a library build (use -DST_PROBES=1)");
#endif
static_assert(ST_FLAT_ALT == 0 || ST_FLAT_ALT == 2, "ST_FLAT_ALT: 0 or 2");
static_assert(ST_DEFER_R0_CACHED == 1 || ST_DEFER_R0_CACHED == 2 ||
                ST_DEFER_R0_CACHED == 4,
              "ST_DEFER_R0_CACHED: 1, 2 or 4 rows");
#define ST_STR2(x) #x
#define ST_STR(x) ST_STR2(x)

namespace st {
namespace {

using dev::kBlock;
using dev::kEpiBlock;

inline bool
aligned16(const void* p)
{
  return ((uintptr_t)p & 15u) == 0;
}

int
check_launch(const char* what)
{
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch failed: %s", what, hipGetErrorString(e));
    return -1;
  }
  return 0;
}

// Tuned shapes (the sweeps tune_fused.hip / sweep_dir.hip (git history),
// tools/stream_bench.hip; profiles/README.md).  One 256-thread workgroup
// streams a group of rows, 2 column chunks of 16 B per lane per row in
// flight; the grid strides over the row groups.  What pays depends on the
// size of the (local) matrix relative to the caches — 4 MB L2 per XCD, the
// 256 MB memory-side cache (MALL) — so the shape is picked per launch:
//   * matrices that outgrow the MALL (k_round >= 1 GiB, k_mfree >= 512 MiB,
//     k_flat >= 2 GiB)
//     use non-temporal loads/stores; below that, cached accesses let the
//     MALL serve part of the next round;
//   * every workgroup keeps the same row groups each round (same XCD, same
//     L2) and walks them backwards on odd rounds (ALT in st_device.h), so a
//     round starts on the rows the previous round touched last;
//   * k_round: 4 rows per group while rows are short (<= 96 KiB streamed,
//     <= 12288 columns cached), 2 above; one workgroup per CU; 2 rows and
//     2 (<= 128 MiB) or 4 (<= 32 MiB) workgroups per CU on small matrices;
//     1 row per group below 1024 rows.  (The solve loops hand blocks of
//     144 MiB and more to the flat round below; st_round_* keeps these
//     shapes at every size.)
//   * k_mfree: 4 rows per group, 2 workgroups per CU (2 rows between 64
//     and 512 MiB).
constexpr int kRows = 2; // k_fused (K0 row sums and the step API)
constexpr int kUnroll = 2;
constexpr uint32_t kGridCap = 512;
constexpr int kMfUnroll = 2;
// the fp32 element-wide path (W = 1) keeps 4x the chunks in flight per
// lane (as many bytes as the 16-byte vector path): 9-28 % faster k_mfree
// and up to 3 % k_round on ragged fp32 sizes; fp64 is 1-7 % slower with
// 2x, so it keeps kUnroll (a lane's columns are summed in column order
// whatever the chunking, so results do not change;
// profiles/r01_ragged_probe.log)
template <typename T, int W, int U>
constexpr int kChunks = (W == 1 && sizeof(T) == 4) ? 4 * U : U;

struct Shape
{
  int rows;      // rows per group: 1, 2 or 4
  bool nt;       // non-temporal matrix loads/stores
  uint32_t grid; // workgroup cap
};

inline size_t
block_bytes(uint32_t nrows, uint32_t ncols, size_t elem)
{
  return (size_t)nrows * ncols * elem;
}

inline Shape
round_shape(uint32_t nrows, uint32_t ncols, size_t elem)
{
  const size_t b = block_bytes(nrows, ncols, elem);
  if (nrows < 2 * kGridCap)
    return { 1, false, 512u };
  if (b <= ((size_t)32 << 20)) // L2-sized: one group per workgroup
    return { 2, false, 1024u };
  if (b < ((size_t)128 << 20))
    return { 2, false, 512u };
  if (b < ((size_t)1 << 30)) // 4 rows per group only while rows are short
    return { ncols <= 12288u ? 4 : 2, false, 256u };
  return { (size_t)ncols * elem <= ((size_t)96 << 10) ? 4 : 2, true, 256u };
}

// tools: st_set_mfree_shape (0 = the table below; 1 / 2 = cached, 2 / 4 rows;
// 3 = non-temporal, 4 rows; grid 512)
// The table: cached loads below 512 MiB, 4 rows per group up to 64 MiB and
// again from 280 MiB (tools/defer_profile.py --mfree-ab, fresh A_0 per pass,
// profiles/r03_mfab_*.json, ms per round, 2 rows vs 4): 6144^2 fp64 0.0462 vs
// 0.0453, 7168^2 0.0674 vs 0.0637, 10240^2 fp32 0.0686 vs 0.0650, the P = 8
// block 2880 x 23040 0.0928 vs 0.0867; below 280 MiB 2 rows (4608^2 fp64
// 0.0255 vs 0.0264, 8192^2 fp32 0.0387 vs 0.0397); from 512 MiB
// non-temporal 4 rows (8192^2 fp64 0.0810 against 0.0846 cached).
std::atomic<uint32_t> g_mfree_shape{ 0u };

inline Shape
mfree_shape(uint32_t nrows, uint32_t ncols, size_t elem)
{
  const size_t b = block_bytes(nrows, ncols, elem);
  const uint32_t ov = g_mfree_shape.load(std::memory_order_relaxed);
  if (ov != 0 && nrows >= 2 * kGridCap)
    return { ov == 1 ? 2 : 4, ov == 3, 512u };
  if (nrows < 2 * kGridCap)
    return { 1, false, 1024u };
  if (b <= ((size_t)64 << 20))
    return { 4, false, 512u };
  if (b < ((size_t)512 << 20))
    return { b >= ((size_t)280 << 20) ? 4 : 2, false, 512u };
  return { 4, true, 512u };
}

// the flat round (k_flat + k_parts) for blocks of >= 144 MiB, with cached
// accesses and alternating piece order below 2 GiB (the memory-side cache
// then serves the start of each round; odd rounds reverse the pieces in
// steps of 8 workgroups so that every piece stays on its XCD and L2,
// flat_reverse<2>) and non-temporal ones above:
// sweep_dir.hip (round 1, git history) SWEEP_FLAT=1 / SWEEP_XCD=1,
// profiles/r01_sweep_flat_cached.log, r01_sweep_xcd{,_round}.log
// (32768^2 fp64 2.68 ms vs 3.06 for k_round; 16384^2 0.67 vs 0.76; 8192^2
// fp64 0.160 vs 0.168, fp32 0.079 vs 0.080; the 2880x23040 block 0.165 vs
// 0.182; 6144^2 fp32 (144 MiB) 0.0472 vs 0.0478; at 128 MiB and below
// k_round stays ahead: 4096^2 fp64 0.0412 vs 0.0426)
constexpr int kFlatRows = 2; // rows per workgroup sharing a column piece
constexpr int kFlatAlt = ST_FLAT_ALT; // odd rounds: pieces reversed per XCD (flat_reverse)
// m_k / stop_k in k_flat's first row group (two launches per round) rather
// than in a k_stats launch of their own (three)
constexpr bool kFlatFusedStats = true;

// A dispatch counts at most 2^32 - 1 work-items per grid dimension, so a
// flat launch of more than kFlatGridX workgroups (fp64 from 131072^2, fp32
// from ~185000^2) goes 2-D; k_flat folds blockIdx.y back in.  A multiple of
// 8, so a workgroup's XCD (linear id % 8) stays the same.
// st_set_flat_grid_limit lowers it (tests: the 2-D form at small sizes).
constexpr uint32_t kFlatGridX = (0xffffffffu / kBlock) & ~7u;
std::atomic<uint32_t> g_flat_grid_x{ kFlatGridX };

struct FlatGrid
{
  dim3 grid;
  uint32_t gx2; // k_flat's gx2 argument: the row width of a 2-D grid, else 0
};

inline FlatGrid
flat_grid(uint32_t nb)
{
  const uint32_t gmax = g_flat_grid_x.load(std::memory_order_relaxed);
  if (nb <= gmax)
    return { dim3(nb), 0u };
  // as few rows as fit, as narrow as they can be: < 8 padding workgroups
  // per row (they exit at once)
  const uint32_t gy = (nb + gmax - 1) / gmax;
  const uint32_t gx = ((nb + gy - 1) / gy + 7u) & ~7u;
  return { dim3(gx, gy), gx };
}

inline bool
flat_round_pays(uint32_t nrows, uint32_t ncols, size_t elem)
{
  return block_bytes(nrows, ncols, elem) >= ((size_t)144 << 20);
}

// dynamic LDS that leaves room for `cap` workgroups per CU (160 KB of LDS
// per CU on gfx950, k_flat's own few hundred bytes included)
inline uint32_t
defer_cap_lds(uint32_t cap)
{
  return cap < 2 ? 0u : (160u << 10) / cap - 2048u;
}

inline bool
flat_round_nt(uint32_t nrows, uint32_t ncols, size_t elem)
{
  return block_bytes(nrows, ncols, elem) >= ((size_t)2 << 30);
}

// chunks of kBlock * W columns per flat piece: 4 KB of a row per piece,
// 8 KB for cached fp64 blocks (below 2 GiB: 1 % faster at 8192^2, 4-6 % on
// the long-row P = 8 block 2880 x 23040; non-temporal blocks and fp32 lose
// 1-7 %, profiles/r01_sweep_rbu.log); the element-wide path (W = 1) takes
// 16 / sizeof(T) chunks so that its pieces hold as many bytes
// (profiles/r01_ragged_probe.log).  Every flat launcher of a block takes
// the same U, so the row sums' order is that of the block's pieces.
template <typename T, int W, bool NT>
constexpr int kFlatU =
  (W == 1 ? (int)(16 / sizeof(T)) : 1) * ((sizeof(T) == 8 && !NT) ? 2 : 1);

// Shape of the every-round flat launch (flat_map_sweep (round 2, git history) FMS_EVERY=1,
// profiles/r02_flat_map_every_*.log, two repeats each):
//   non-temporal blocks  2 rows per workgroup, pieces walked in tiles of 4
//                        row groups (32768^2 fp64 2.625 vs 2.688 ms, fp32
//                        1.301 vs 1.336, 16384 / 8192 x 65536 -1.8 / -1.0 %)
//   cached fp64 blocks   1 row (8 KB pieces), tiles of 8 rows from 384 MiB
//                        and of 4 below: 8192^2 0.1536 / 0.1528 vs 0.1545 /
//                        0.1539 ms (2 rows, row-major), 12288^2 -0.5 %,
//                        6144^2 -1 % (tiles of 4; 8 lose 2 % there); the
//                        whole round on the weak-scaled rank blocks, k_parts
//                        included (tools/split_cost.py,
//                        profiles/r02_every_cached_ab_split_cost.log):
//                        5824 x 11648 0.162 vs 0.171 ms, 4096 x 16384 0.156
//                        vs 0.159, 2880 x 23040 0.155 vs 0.159
//   cached fp32 blocks   2 rows, row-major (1 row or tiles lose 0-3 %)
// Which rows a workgroup takes, and in what order, changes no result.
template <typename T, bool NT>
constexpr int kFlatEveryRows =
  (sizeof(T) == 8 && !NT && ST_EVERY_CACHED_R1) ? 1 : kFlatRows;

// tools: the every-round launch's piece tile per size class
// (every_cache_class; 0 = the table below, 1 = row-major, t = tiles of t row
// groups), st_set_every_tile
constexpr int kEveryTileClasses = 4;
std::atomic<uint32_t> g_every_tile[kEveryTileClasses] = { 0u, 0u, 0u, 0u };

inline uint32_t every_cache_class(size_t bytes);

template <typename T, bool NT>
inline uint32_t
flat_every_tile(uint32_t nrows, uint32_t ncols)
{
  const uint32_t ov =
    g_every_tile[every_cache_class(block_bytes(nrows, ncols, sizeof(T)))].load(
      std::memory_order_relaxed);
  if (ov != 0)
    return ov == 1 ? 0u : ov;
  if (NT)
    return 4u;
  if (sizeof(T) == 4 || !ST_EVERY_CACHED_R1)
    return 0u;
  return block_bytes(nrows, ncols, sizeof(T)) >= ((size_t)384 << 20) ? 8u : 4u;
}

// Cache policy of the every-round flat launch, by block size class
// (every_cache_class: below 384 MiB, below 640 MiB, below 2 GiB - the cached
// form - and from 2 GiB - the non-temporal form): bit 0 turns the matrix
// loads' policy over (cached <-> non-temporal), bit 1 the stores'; the
// shapes, piece size and piece order stay the form's.  Set per class for
// tools by st_set_every_cache; results do not depend on it.  The bench's
// timed step (tools/defer_profile.py --every-ab, 5 - 10 interleaved passes
// of 100 rounds, two boxes, profiles/r03_everyab_*.json), ms per round:
//   policy         0 (form's)   1 (nt loads)   2 (nt stores)  3 (both)
//   8192^2 fp64    0.1555/0.1558   0.1625        0.1533/0.1528   0.1747
//   2880 x 23040   0.1470/0.1469   0.1678        0.1467/0.1462   0.1776
//   5824 x 11648   0.1560/0.1564   0.1790        0.1557/0.1554   0.1840
//   4096 x 16384   0.1469/0.1472   0.1573        0.1462/0.1462   0.1734
//   6144^2 fp64    0.0878/0.0882   0.1011        0.0876/0.0882   0.1020
//   8192^2 fp32    0.0764/0.0764   0.0833        0.0759/0.0760   0.0878
//   12288^2 fp32   0.1760/0.1760   0.1920        0.1755/0.1752   0.1978
//   10240^2 fp64   0.2594/0.2595   0.2760        0.2605/0.2603   0.2755
//   12288^2 fp64   0.3845/0.3848   0.4026        0.3858/0.3853   0.3947
//   16384^2 fp32   0.3262/0.3257   0.3474        0.3260/0.3253   0.3370
//   (non-temporal form: 1 = cached loads, 2 = cached stores, 3 = both)
//   32768^2 fp64   2.643           3.180          2.944          3.226
//   8192 x 65536   1.349           1.632          1.464          1.635
//   32768^2 fp32   1.308           1.426          1.466          1.425
// Streaming the stores past the caches pays while the block is at most
// about twice the 256 MB memory-side cache (8192^2 fp64 -1.9 %), not above;
// loads stay cached there (the next round's first pieces are read from the
// cache), and the non-temporal form keeps both non-temporal.
constexpr int kEveryCacheClasses = 4;
std::atomic<uint32_t> g_every_cache[kEveryCacheClasses] = { 2u, 2u, 0u, 0u };
// workgroups per CU of the every-round launch per size class (0 = as many
// as the registers allow; dynamic LDS the kernel does not use, as for the
// deferred launches: defer_cap_lds), st_set_every_caps
std::atomic<uint32_t> g_every_caps[kEveryCacheClasses] = { 0u, 0u, 0u, 0u };

inline uint32_t
every_cache_class(size_t bytes)
{
  return bytes < ((size_t)384 << 20)   ? 0u
         : bytes < ((size_t)640 << 20) ? 1u
         : bytes < ((size_t)2 << 30)   ? 2u
                                       : 3u;
}

// k_parts of an unsplit flat round: rows of <= 16 / 32 partials take 4 / 2
// rows per wave (k_parts_seg, bitwise k_parts' sums), longer ones a wave
// each (k_parts)
template <typename T>
void
launch_parts(const T* part, T* s_next, uint32_t nrows, uint32_t ppr, uint32_t k,
             const st_state* st, const T* s_cur, T* v, uint32_t row0, T* inv_next,
             hipStream_t stream)
{
  if (ppr <= 16) {
    const uint32_t g = (nrows + kBlock / 16 - 1) / (kBlock / 16);
    hipLaunchKernelGGL((dev::k_parts_seg<T, 16>), dim3(g), dim3(kBlock), 0, stream, part,
                       s_next, nrows, ppr, k, st, s_cur, v, row0, inv_next);
  } else if (ppr <= 32) {
    const uint32_t g = (nrows + kBlock / 32 - 1) / (kBlock / 32);
    hipLaunchKernelGGL((dev::k_parts_seg<T, 32>), dim3(g), dim3(kBlock), 0, stream, part,
                       s_next, nrows, ppr, k, st, s_cur, v, row0, inv_next);
  } else {
    const uint32_t g = (nrows + dev::kWaves - 1) / dev::kWaves;
    hipLaunchKernelGGL((dev::k_parts<T>), dim3(g), dim3(kBlock), 0, stream, part, s_next,
                       nrows, ppr, k, st, s_cur, v, row0, nullptr, 0u, 0u, 0u, inv_next);
  }
}

// partial sums per row (one per piece) and the scratch they need
inline uint32_t
flat_pieces(uint32_t ncols, int w)
{
  return (ncols + (uint32_t)(kBlock * w) - 1) / (uint32_t)(kBlock * w);
}

inline size_t
flat_scratch_elems(uint32_t nrows, uint32_t ncols)
{
  return (size_t)nrows * flat_pieces(ncols, 1); // enough for any vector width
}

inline bool
fused_nt(uint32_t nrows, uint32_t ncols, size_t elem)
{
  // k_fused is the read-mostly K0 row-sum pass: the k_mfree threshold
  return block_bytes(nrows, ncols, elem) >= ((size_t)512 << 20);
}

template <typename T, int ROWS, int W, int U, bool SCALE, bool SUM, int ORDER>
void
launch_cfg(T* a, const T* s_cur, T* s_next, uint32_t row_begin,
           uint32_t nblocks, uint32_t ncols, uint32_t row0, bool nt,
           const st_state* st, hipStream_t stream)
{
  if (nblocks == 0)
    return;
  const uint32_t grid = nblocks < kGridCap ? nblocks : kGridCap;
  if (nt)
    hipLaunchKernelGGL((dev::k_fused<T, ROWS, W, U, SCALE, SUM, ORDER, true>),
                       dim3(grid), dim3(kBlock), 0, stream, a, a, s_cur, s_next,
                       row_begin, nblocks, ncols, row0, st);
  else
    hipLaunchKernelGGL((dev::k_fused<T, ROWS, W, U, SCALE, SUM, ORDER, false>),
                       dim3(grid), dim3(kBlock), 0, stream, a, a, s_cur, s_next,
                       row_begin, nblocks, ncols, row0, st);
}

template <typename T, int W, bool SCALE, bool SUM, int ORDER>
void
launch_rows(T* a, const T* s_cur, T* s_next, uint32_t nrows, uint32_t ncols,
            uint32_t row0, const st_state* st, hipStream_t stream)
{
  const bool nt = fused_nt(nrows, ncols, sizeof(T));
  // small matrices: one row per workgroup keeps >= 256 workgroups busy
  if (nrows < 2 * kGridCap) {
    launch_cfg<T, 1, W, kChunks<T, W, kUnroll>, SCALE, SUM, ORDER>(a, s_cur, s_next, 0, nrows,
                                                    ncols, row0, nt, st, stream);
    return;
  }
  // the pure row-sum pass streams like k_mfree: 4 rows per group once the
  // matrix outgrows the MALL
  constexpr int R4 = SCALE ? kRows : 4;
  const int rows = nt ? R4 : kRows;
  const uint32_t full = nrows / rows;
  if (rows == 4)
    launch_cfg<T, R4, W, kChunks<T, W, kUnroll>, SCALE, SUM, ORDER>(
      a, s_cur, s_next, 0, full, ncols, row0, nt, st, stream);
  else
    launch_cfg<T, kRows, W, kChunks<T, W, kUnroll>, SCALE, SUM, ORDER>(
      a, s_cur, s_next, 0, full, ncols, row0, nt, st, stream);
  launch_cfg<T, 1, W, kChunks<T, W, kUnroll>, SCALE, SUM, ORDER>(
    a, s_cur, s_next, full * rows, nrows - full * rows, ncols, row0, nt, st,
    stream);
}

template <typename T, bool SCALE, bool SUM, int ORDER>
void
launch_vec(T* a, const T* s_cur, T* s_next, uint32_t nrows, uint32_t ncols,
           uint32_t row0, const st_state* st, hipStream_t stream)
{
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok =
    (ncols % W) == 0 && aligned16(a) && (!SCALE || aligned16(s_cur));
  if (vec_ok)
    launch_rows<T, W, SCALE, SUM, ORDER>(a, s_cur, s_next, nrows, ncols, row0,
                                         st, stream);
  else
    launch_rows<T, 1, SCALE, SUM, ORDER>(a, s_cur, s_next, nrows, ncols, row0,
                                         st, stream);
}

template <typename T, int ROWS, int W, int ORDER, int NT>
void
launch_round_cfg(T* a, const T* s_cur, T* s_next, T* v, uint32_t nrows,
                 uint32_t ncols, uint32_t row0, T eps, uint32_t k,
                 uint32_t max_itr, uint32_t semantics, st_state* st,
                 uint32_t cap, hipStream_t stream)
{
  const uint32_t ng_main = nrows / ROWS, nrem = nrows % ROWS;
  const uint32_t ng = ng_main + nrem;
  const uint32_t grid = ng < cap ? ng : cap;
  hipLaunchKernelGGL(
    (dev::k_round<T, ROWS, W, kChunks<T, W, kUnroll>, ORDER, NT, kBlock, true>),
    dim3(grid),
    dim3(kBlock), 0, stream, a, s_cur, s_next, v, ng_main, nrem, ncols, row0,
    eps, k, max_itr, semantics, st);
}

template <typename T, int W, int ORDER>
void
launch_round_rows(T* a, const T* s_cur, T* s_next, T* v, uint32_t nrows,
                  uint32_t ncols, uint32_t row0, T eps, uint32_t k,
                  uint32_t max_itr, uint32_t semantics, st_state* st,
                  hipStream_t stream)
{
  const Shape sh = round_shape(nrows, ncols, sizeof(T));
#define ST_ROUND_CFG(R, N)                                                     \
  launch_round_cfg<T, R, W, ORDER, N>(a, s_cur, s_next, v, nrows, ncols, row0, \
                                      eps, k, max_itr, semantics, st, sh.grid, \
                                      stream)
  using dev::kCached;
  using dev::kNtBoth;
  if (sh.rows == 1)
    ST_ROUND_CFG(1, kCached);
  else if (sh.rows == 2)
    sh.nt ? ST_ROUND_CFG(2, kNtBoth) : ST_ROUND_CFG(2, kCached);
  else
    sh.nt ? ST_ROUND_CFG(4, kNtBoth) : ST_ROUND_CFG(4, kCached);
#undef ST_ROUND_CFG
}

template <typename T, int ROWS, int W, int ORDER, int NT, int SPAN>
void
launch_split_cfg(T* a, const T* s_cur, T* s_next, T* part, T* v,
                 uint32_t nrows, uint32_t ncols, uint32_t row0, uint32_t q0,
                 uint32_t q1, T eps, uint32_t k, uint32_t max_itr,
                 uint32_t semantics, st_state* st, uint32_t cap,
                 hipStream_t stream)
{
  const uint32_t ng_main = nrows / ROWS, nrem = nrows % ROWS;
  const uint32_t ng = ng_main + nrem;
  const uint32_t grid = ng < cap ? ng : cap;
  hipLaunchKernelGGL((dev::k_round_split<T, ROWS, W, kChunks<T, W, kUnroll>, ORDER, NT,
                                          SPAN>),
                     dim3(grid), dim3(kBlock), 0, stream, a, s_cur, s_next,
                     part, v, ng_main, nrem, ncols, row0, q0, q1, eps, k,
                     max_itr, semantics, st);
}

template <typename T, int W, int ORDER, int SPAN>
void
launch_split_rows(T* a, const T* s_cur, T* s_next, T* part, T* v,
                  uint32_t nrows, uint32_t ncols, uint32_t row0, uint32_t q0,
                  uint32_t q1, T eps, uint32_t k, uint32_t max_itr,
                  uint32_t semantics, st_state* st, hipStream_t stream)
{
  // the shape of the whole round (both halves stream the same rows); the
  // local half streams non-temporally so that it does not evict what the
  // remote half re-reads from the memory-side cache round after round
  // (sweep_dir.hip (round 1, git history) SWEEP_SPLIT=1: at the P = 8 block the pair then
  // costs 4 us over one k_round launch instead of 25 us)
  const Shape sh = round_shape(nrows, ncols, sizeof(T));
#define ST_SPLIT_CFG(R, N)                                                     \
  launch_split_cfg<T, R, W, ORDER,                                             \
                   SPAN == dev::kSpanLocal ? dev::kNtBoth : (N), SPAN>(        \
    a, s_cur, s_next, part, v, nrows, ncols, row0, q0, q1, eps, k, max_itr,    \
    semantics, st, sh.grid, stream)
  using dev::kCached;
  using dev::kNtBoth;
  // 4 rows per group whenever rows are grouped: each half sweeps only part
  // of a row, so more rows amortise the per-group reduction (6 % at P = 8)
  if (sh.rows == 1)
    ST_SPLIT_CFG(1, kCached);
  else
    sh.nt ? ST_SPLIT_CFG(4, kNtBoth) : ST_SPLIT_CFG(4, kCached);
#undef ST_SPLIT_CFG
}

template <typename T, int W, int SPAN>
void
launch_split_order(T* a, const T* s_cur, T* s_next, T* part, T* v,
                   uint32_t nrows, uint32_t ncols, uint32_t row0, uint32_t q0,
                   uint32_t q1, T eps, uint32_t k, uint32_t max_itr,
                   uint32_t semantics, st_state* st, hipStream_t stream)
{
  if (semantics == ST_SEM_MAINPY)
    launch_split_rows<T, W, 1, SPAN>(a, s_cur, s_next, part, v, nrows, ncols,
                                     row0, q0, q1, eps, k, max_itr, semantics,
                                     st, stream);
  else
    launch_split_rows<T, W, 0, SPAN>(a, s_cur, s_next, part, v, nrows, ncols,
                                     row0, q0, q1, eps, k, max_itr, semantics,
                                     st, stream);
}

template <typename T, int ROWS, int W, bool NT>
void
launch_mfree_cfg(const T* a0, const T* s_prev, T* s_next, const T* v_prev,
                 T* v_cur, uint32_t nrows, uint32_t ncols, uint32_t row0,
                 T eps, uint32_t k, uint32_t max_itr, uint32_t semantics,
                 st_state* st, uint32_t cap, hipStream_t stream)
{
  const uint32_t ng_main = nrows / ROWS, nrem = nrows % ROWS;
  const uint32_t ng = ng_main + nrem;
  const uint32_t grid = ng < cap ? ng : cap;
  hipLaunchKernelGGL(
    (dev::k_mfree<T, ROWS, W, kChunks<T, W, kMfUnroll>, NT, kBlock, true>),
    dim3(grid),
    dim3(kBlock), 0, stream, a0, s_prev, s_next, v_prev, v_cur, ng_main, nrem,
    ncols, row0, eps, k, max_itr, semantics, st);
}

template <typename T, int W>
void
launch_mfree_rows(const T* a0, const T* s_prev, T* s_next, const T* v_prev,
                  T* v_cur, uint32_t nrows, uint32_t ncols, uint32_t row0,
                  T eps, uint32_t k, uint32_t max_itr, uint32_t semantics,
                  st_state* st, hipStream_t stream)
{
  const Shape sh = mfree_shape(nrows, ncols, sizeof(T));
#define ST_MFREE_CFG(R, N)                                                     \
  launch_mfree_cfg<T, R, W, N>(a0, s_prev, s_next, v_prev, v_cur, nrows,       \
                               ncols, row0, eps, k, max_itr, semantics, st,    \
                               sh.grid, stream)
  if (sh.rows == 1)
    ST_MFREE_CFG(1, false);
  else if (sh.rows == 2)
    sh.nt ? ST_MFREE_CFG(2, true) : ST_MFREE_CFG(2, false);
  else
    sh.nt ? ST_MFREE_CFG(4, true) : ST_MFREE_CFG(4, false);
#undef ST_MFREE_CFG
}

} // namespace

template <typename T>
int
launch_mfree(const T* a0, const T* s_prev, T* s_next, const T* v_prev,
             T* v_cur, uint32_t nrows, uint32_t ncols, uint32_t row0, T eps,
             uint32_t k, uint32_t max_itr, uint32_t semantics, st_state* st,
             hipStream_t stream)
{
  ST_REQUIRE(a0 && s_prev && s_next && v_prev && v_cur && st,
             "mfree: null pointer");
  ST_REQUIRE(nrows > 0 && ncols > 0, "mfree: empty block");
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "mfree: bad semantics %u", semantics);
  ST_REQUIRE(k >= 1 && max_itr > 0, "mfree: launch index k must be >= 1");
  ST_REQUIRE(v_prev != v_cur, "mfree: v_prev and v_cur must differ");
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && aligned16(a0) && aligned16(s_prev) &&
                      aligned16(v_prev);
  if (vec_ok)
    launch_mfree_rows<T, W>(a0, s_prev, s_next, v_prev, v_cur, nrows, ncols,
                            row0, eps, k, max_itr, semantics, st, stream);
  else
    launch_mfree_rows<T, 1>(a0, s_prev, s_next, v_prev, v_cur, nrows, ncols,
                            row0, eps, k, max_itr, semantics, st, stream);
  return check_launch("mfree");
}

// ---- the matrix-free round, flat -------------------------------------------
// k_flat<..., MF> over one 4 / 8 KB piece of R rows per workgroup, the first
// row group folding round k-1's stats, then k_mparts (s_k of the rows,
// v_{k-1} of all n).  Same row sums up to association as k_mfree (pieces
// summed apart).  Shapes (store_probe (round 3, git history) SP_MF=1,
// profiles/r03_mf_shapes_{nt,cached}.log; a flat launch + k_mparts against
// one k_mfree launch): every lane's x = v ∘ s vector serves R rows, so 4 - 8
// rows pay where the read-only deferred rounds take 1 - 2, and they want a
// workgroup cap like the deferred rounds' (dynamic LDS): cached fp64 8 rows
// in tiles of 8 row groups, 4 per CU (8192^2 0.0798 vs 0.0848 ms for
// k_mfree); non-temporal 4 rows in tiles of 8, 5 per CU (32768^2 fp64 1.205
// vs 1.216, 8192 x 65536 0.642 vs 0.644).
template <typename T, int W, bool NT>
void
launch_mfree_flat_cfg(const T* a0, const T* s_prev, T* s_next, const T* v_prev, T* v_cur,
                      T* part, uint32_t nrows, uint32_t ncols, uint32_t row0, T eps,
                      uint32_t k, uint32_t max_itr, uint32_t semantics, st_state* st,
                      hipStream_t stream)
{
  constexpr int U = kFlatU<T, W, NT>;
  constexpr int R = NT ? 4 : 8;
  const uint32_t ppr = flat_pieces(ncols, W * U);
  const FlatGrid fg = flat_grid((nrows + R - 1) / R * ppr);
  dev::FlatPending<T, -1> pe{};
  pe.pt = 8u;
  const uint32_t lds = defer_cap_lds(NT ? 5u : 4u);
  hipLaunchKernelGGL((dev::k_flat<T, W, 0, NT, R, true, kFlatAlt, 0, -1, U, -1, true>),
                     fg.grid, dim3(kBlock), lds, stream, const_cast<T*>(a0), s_prev, part,
                     const_cast<T*>(v_prev), nrows, ncols, ppr, row0, k, st, eps, max_itr,
                     semantics, 0u, 0u, 0u, pe, fg.gx2);
  const uint32_t rb = (nrows + dev::kWaves - 1) / dev::kWaves;
  const uint32_t vb = (ncols + kBlock - 1) / kBlock < 256u ? (ncols + kBlock - 1) / kBlock
                                                            : 256u;
  hipLaunchKernelGGL((dev::k_mparts<T>), dim3(rb + vb), dim3(kBlock), 0, stream, part,
                     s_next, nrows, ppr, k, st, s_prev, v_prev, v_cur, row0, ncols, rb);
}

template <typename T>
int
launch_mfree_flat(const T* a0, const T* s_prev, T* s_next, const T* v_prev, T* v_cur,
                  T* part, uint32_t nrows, uint32_t ncols, uint32_t row0, T eps,
                  uint32_t k, uint32_t max_itr, uint32_t semantics, st_state* st,
                  hipStream_t stream)
{
  ST_REQUIRE(a0 && s_prev && s_next && v_prev && v_cur && part && st,
             "mfree_flat: null pointer");
  ST_REQUIRE(nrows > 0 && ncols > 0 && row0 + (uint64_t)nrows <= ncols,
             "mfree_flat: bad block");
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "mfree_flat: bad semantics %u", semantics);
  ST_REQUIRE(k >= 1 && max_itr > 0, "mfree_flat: launch index k must be >= 1");
  ST_REQUIRE(v_prev != v_cur, "mfree_flat: v_prev and v_cur must differ");
  ST_REQUIRE((uint64_t)((nrows + kFlatRows - 1) / kFlatRows) * flat_pieces(ncols, 1) <
               (1ull << 31),
             "mfree_flat: %u x %u is too large for one launch", nrows, ncols);
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && aligned16(a0) && aligned16(s_prev) &&
                      aligned16(v_prev);
  const bool nt = flat_round_nt(nrows, ncols, sizeof(T));
#define ST_MFF(WW, NN)                                                         \
  launch_mfree_flat_cfg<T, WW, NN>(a0, s_prev, s_next, v_prev, v_cur, part, nrows, \
                                   ncols, row0, eps, k, max_itr, semantics, st,   \
                                   stream)
  if (vec_ok)
    nt ? ST_MFF(W, true) : ST_MFF(W, false);
  else
    nt ? ST_MFF(1, true) : ST_MFF(1, false);
#undef ST_MFF
  return check_launch("mfree_flat");
}

template int launch_mfree_flat<float>(const float*, const float*, float*, const float*,
                                      float*, float*, uint32_t, uint32_t, uint32_t, float,
                                      uint32_t, uint32_t, uint32_t, st_state*, hipStream_t);
template int launch_mfree_flat<double>(const double*, const double*, double*, const double*,
                                       double*, double*, uint32_t, uint32_t, uint32_t,
                                       double, uint32_t, uint32_t, uint32_t, st_state*,
                                       hipStream_t);

template <typename T>
int
launch_round(T* a, const T* s_cur, T* s_next, T* v, uint32_t nrows,
             uint32_t ncols, uint32_t row0, T eps, uint32_t k,
             uint32_t max_itr, uint32_t semantics, st_state* st,
             hipStream_t stream)
{
  ST_REQUIRE(s_cur && v && st, "round: null pointer");
  ST_REQUIRE(a && s_next, "round: null pointer");
  ST_REQUIRE(ncols > 0, "round: ncols must be > 0");
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "round: bad semantics %u", semantics);
  ST_REQUIRE(max_itr > 0, "round: max_itr must be > 0");
  // every launch must own >= 1 row: the stop test and m_k are derived from
  // the sweep of a row group (the sharded driver rejects empty row blocks)
  ST_REQUIRE(nrows > 0, "round: nrows must be > 0");
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && aligned16(a) && aligned16(s_cur);
  const bool order1 = semantics == ST_SEM_MAINPY;
  if (vec_ok) {
    if (order1)
      launch_round_rows<T, W, 1>(a, s_cur, s_next, v, nrows, ncols, row0, eps,
                                 k, max_itr, semantics, st, stream);
    else
      launch_round_rows<T, W, 0>(a, s_cur, s_next, v, nrows, ncols, row0, eps,
                                 k, max_itr, semantics, st, stream);
  } else {
    if (order1)
      launch_round_rows<T, 1, 1>(a, s_cur, s_next, v, nrows, ncols, row0, eps,
                                 k, max_itr, semantics, st, stream);
    else
      launch_round_rows<T, 1, 0>(a, s_cur, s_next, v, nrows, ncols, row0, eps,
                                 k, max_itr, semantics, st, stream);
  }
  return check_launch("round");
}

template <typename T>
int
launch_round_split(int span, T* a, const T* s_cur, T* s_next, T* part, T* v,
                   uint32_t nrows, uint32_t ncols, uint32_t row0,
                   uint32_t col0, uint32_t col1, T eps, uint32_t k,
                   uint32_t max_itr, uint32_t semantics, st_state* st,
                   hipStream_t stream)
{
  ST_REQUIRE(a && s_cur && part && st, "round_split: null pointer");
  ST_REQUIRE(span == 1 || span == 2, "round_split: span must be 1 (local) "
                                     "or 2 (remote), not %d", span);
  ST_REQUIRE(span == 1 || (s_next && v), "round_split: null pointer");
  ST_REQUIRE(ncols > 0 && nrows > 0, "round_split: empty block");
  ST_REQUIRE(col0 <= col1 && col1 <= ncols,
             "round_split: bad local column range [%u, %u) of %u", col0, col1,
             ncols);
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "round_split: bad semantics %u",
             semantics);
  ST_REQUIRE(max_itr > 0, "round_split: max_itr must be > 0");
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && (col0 % W) == 0 && (col1 % W) == 0 &&
                      aligned16(a) && aligned16(s_cur);
  const uint32_t w = vec_ok ? W : 1;
  const uint32_t q0 = col0 / w, q1 = col1 / w;
#define ST_SPLIT(WW, SP)                                                       \
  launch_split_order<T, WW, SP>(a, s_cur, s_next, part, v, nrows, ncols, row0, \
                                q0, q1, eps, k, max_itr, semantics, st, stream)
  if (vec_ok)
    span == 1 ? ST_SPLIT(W, dev::kSpanLocal) : ST_SPLIT(W, dev::kSpanRemote);
  else
    span == 1 ? ST_SPLIT(1, dev::kSpanLocal) : ST_SPLIT(1, dev::kSpanRemote);
#undef ST_SPLIT
  return check_launch("round_split");
}

template <typename T, int W, int ORDER, bool NT>
void
launch_flat_parts(T* a, const T* s_cur, T* s_next, T* part, T* v,
                  uint32_t nrows, uint32_t ncols, uint32_t row0, T eps,
                  uint32_t k, uint32_t max_itr, uint32_t semantics,
                  st_state* st, hipStream_t stream)
{
  constexpr int U = kFlatU<T, W, NT>;
  // rows per workgroup: 2, one on cached fp64 blocks (below)
  constexpr int R = kFlatEveryRows<T, NT>;
  const uint32_t ppr = flat_pieces(ncols, W * U);
  const uint32_t grid = (nrows + R - 1) / R * ppr;
  const uint32_t pgrid = (nrows + dev::kWaves - 1) / dev::kWaves;
  const FlatGrid fg = flat_grid(grid);
  dev::FlatPending<T, -1> pe{};
  pe.pt = flat_every_tile<T, NT>(nrows, ncols);
  if constexpr (kFlatFusedStats) {
    // two launches: m_k / stop_k folded into k_flat's first row group, the
    // v update into k_parts; the cache policy of the matrix loads / stores
    // per g_every_cache (vector path only)
    const uint32_t pol =
      W == 1 ? 0u
             : g_every_cache[every_cache_class(block_bytes(nrows, ncols, sizeof(T)))]
                 .load(std::memory_order_relaxed);
    const uint32_t lds = defer_cap_lds(
      g_every_caps[every_cache_class(block_bytes(nrows, ncols, sizeof(T)))].load(
        std::memory_order_relaxed));
#define ST_EVERY(FL)                                                           \
  hipLaunchKernelGGL(                                                          \
    (dev::k_flat<T, W, ORDER, NT, R, true, kFlatAlt, 0, -1, U, -1, false,      \
                 FL>),                                                         \
    fg.grid, dim3(kBlock), lds, stream, a, s_cur, part, v, nrows, ncols, ppr,  \
    row0, k, st, eps, max_itr, semantics, 0u, 0u, 0u, pe, fg.gx2)
    constexpr int kV = W > 1 ? 1 : 0;
    switch (pol) {
      case 1u: ST_EVERY(kV); break;
      case 2u: ST_EVERY(2 * kV); break;
      case 3u: ST_EVERY(3 * kV); break;
      default: ST_EVERY(0); break;
    }
#undef ST_EVERY
    launch_parts<T>(part, s_next, nrows, ppr, k, st, s_cur, v, row0, nullptr, stream);
  } else {
    const uint32_t sgrid =
      (ncols + kBlock - 1) / kBlock < 256u ? (ncols + kBlock - 1) / kBlock : 256u;
    hipLaunchKernelGGL((dev::k_stats<T>), dim3(sgrid), dim3(kBlock), 0, stream,
                       s_cur, ncols, eps, k, max_itr, semantics, st);
    hipLaunchKernelGGL(
      (dev::k_flat<T, W, ORDER, NT, R, false, kFlatAlt, 0, -1, U>),
      fg.grid, dim3(kBlock), 0, stream, a, s_cur, part, v, nrows, ncols, ppr,
      row0, k, st, eps, max_itr, semantics, 0u, 0u, 0u, pe, fg.gx2);
    hipLaunchKernelGGL((dev::k_parts<T>), dim3(pgrid), dim3(kBlock), 0, stream,
                       part, s_next, nrows, ppr, k, st, nullptr, nullptr, 0u);
  }
}

template <typename T>
int
launch_round_flat(T* a, const T* s_cur, T* s_next, T* part, T* v,
                  uint32_t nrows, uint32_t ncols, uint32_t row0, T eps,
                  uint32_t k, uint32_t max_itr, uint32_t semantics,
                  st_state* st, hipStream_t stream)
{
  ST_REQUIRE(a && s_cur && s_next && part && v && st,
             "round_flat: null pointer");
  ST_REQUIRE(ncols > 0 && nrows > 0, "round_flat: empty block");
  ST_REQUIRE(row0 + (uint64_t)nrows <= ncols,
             "round_flat: rows [%u, %u) outside the %u-long row-sum vector",
             row0, row0 + nrows, ncols);
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "round_flat: bad semantics %u",
             semantics);
  ST_REQUIRE(max_itr > 0, "round_flat: max_itr must be > 0");
  ST_REQUIRE((uint64_t)((nrows + kFlatRows - 1) / kFlatRows) *
                 flat_pieces(ncols, 1) <
               (1ull << 31),
             "round_flat: %u x %u is too large for one launch", nrows, ncols);
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && aligned16(a) && aligned16(s_cur);
  const bool order1 = semantics == ST_SEM_MAINPY;
  const bool nt = flat_round_nt(nrows, ncols, sizeof(T));
#define ST_FLAT(WW, OO, NN)                                                    \
  launch_flat_parts<T, WW, OO, NN>(a, s_cur, s_next, part, v, nrows, ncols,    \
                                   row0, eps, k, max_itr, semantics, st,       \
                                   stream)
  if (vec_ok) {
    if (order1)
      nt ? ST_FLAT(W, 1, true) : ST_FLAT(W, 1, false);
    else
      nt ? ST_FLAT(W, 0, true) : ST_FLAT(W, 0, false);
  } else {
    if (order1)
      nt ? ST_FLAT(1, 1, true) : ST_FLAT(1, 1, false);
    else
      nt ? ST_FLAT(1, 0, true) : ST_FLAT(1, 0, false);
  }
#undef ST_FLAT
  return check_launch("round_flat");
}

// ---- the flat round with deferred writes ----------------------------------
// (FlatPending in st_device.h): A is stored every defer_rounds() rounds;
// the rounds in between re-apply the pending scalings from
// the last stored matrix, bit-identical to storing every round.
// sweep_dir.hip (round 1, git history) SWEEP_DEFER=1 [SWEEP_DEFER_RING=1],
// profiles/r01_sweep_defer{,_ring}.log, with s and 1/s in a ring of distinct
// vectors as the solve keeps them: per round 32768^2 fp64 1.85 ms (every
// 3rd round stored, 2 rows per workgroup) vs 2.70 storing every round,
// 8192^2 fp64 0.125 vs 0.158; fp32 (every 4th, 4 rows) 0.821 vs 1.350 and
// 0.053 vs 0.078.  Longer groups lose: the pending scales' loads and
// registers outgrow the bytes saved.
template <typename T, int W, int ORDER, bool NT, int NP, int R, bool STORE,
          int FL = 0>
void
launch_flat_deferred_np(T* a, const T* s_cur, const T* inv_cur, T* s_next,
                        T* inv_next, T* part, T* v, uint32_t nrows,
                        uint32_t ncols, uint32_t row0, T eps, uint32_t k,
                        uint32_t max_itr, uint32_t semantics, st_state* st,
                        const T* const* pend_s, const T* const* pend_inv,
                        bool flush, uint32_t pt, uint32_t lds, hipStream_t stream)
{
  constexpr int U = kFlatU<T, W, NT>;
  const uint32_t ppr = flat_pieces(ncols, W * U);
  const uint32_t grid = (nrows + R - 1) / R * ppr;
  dev::FlatPending<T, NP> pd{};
  for (int i = 0; i < NP; i++) {
    pd.s[i] = pend_s[i];
    pd.inv[i] = pend_inv[i];
  }
  pd.inv_cur = inv_cur;
  pd.pt = pt;
  const FlatGrid fg = flat_grid(grid);
  // lds: dynamic LDS the kernel does not use, reserved only to cap the
  // workgroups per CU (see launch_flat_deferred)
  hipLaunchKernelGGL((dev::k_flat<T, W, ORDER, NT, R, true, kFlatAlt, 0, NP, U,
                                  STORE ? 1 : 0, false, FL>),
                     fg.grid, dim3(kBlock), lds, stream, a, s_cur, part, v,
                     nrows, ncols, ppr, row0, k, st, eps, max_itr, semantics,
                     0u, 0u, 0u, pd, fg.gx2);
  if (!flush) // a flush only stores the matrix: s, v and the state stand
    launch_parts<T>(part, s_next, nrows, ppr, k, st, s_cur, v, row0, inv_next, stream);
}

// Workgroups per CU of the deferred rounds' launches (0 = as many as the
// registers allow).  A launch that keeps R = 4 or 8 rows x 16 B per lane in
// flight oversubscribes the memory system at full occupancy (5-6
// workgroups, up to 192 KB of loads per CU): capping it - with dynamic LDS
// the kernel does not use, the only hard cap on workgroups per CU - is
// faster: single launches (store_probe (round 3, git history) SP_CAPS=1,
// profiles/r03_store_probe_caps_*.log) the non-temporal storing round 2.85
// -> 2.78 ms at 3 per CU (32768^2 fp64), NP = 3 1.205 -> 1.183 at 4; the
// R = 2 launches (every-round, NP = 0) only lose.  The solve loop over whole
// store cycles (tools/defer_profile.py --caps-ab, 5 interleaved passes,
// profiles/r03_capsab_*.json) picks the table: 32768^2 fp64 1.483 vs 1.510
// ms per round, the P = 8 rank block of configs[3] 0.767 vs 0.782, 32768^2
// fp32 0.733 vs 0.744, 8192^2 fp64 0.1008 vs 0.1024; cached fp32 blocks lose
// with any cap (8192^2 0.0486 uncapped, 0.050 - 0.055 capped).  A second
// A/B of the table against its neighbours (profiles/r03_capsab2_*.json):
// P = 8 rank block 0.759 vs 0.777 uncapped, 8192^2 fp64 0.0995 (NP = 3 at 3
// per CU) vs 0.1013; 32768^2 fp64 within the box's noise that run (min
// 1.485 vs 1.503 uncapped).  Indexed
// [fp64][non-temporal][slot], slot = the pending count of a read-only round
// (0 ... 4) or kCapStore for a storing one (5 unused).
constexpr int kCapStore = 6;
std::atomic<uint32_t> g_defer_caps[2][2][7] = {
  // fp32: cached, non-temporal
  { { 0, 0, 0, 0, 0, 0, 0 }, { 0, 6, 5, 4, 5, 0, 3 } },
  // fp64: cached, non-temporal (the cached storing round uncapped since
  // round 4: caps 0 / 3 / 4 tie within 0.1 % on 8192^2 and the three
  // weak-scaled rank blocks once it is tiled by 16, 2 loses 1-2 %,
  // profiles/r04_storeab.json, runs *_s5t16)
  { { 0, 4, 4, 3, 3, 0, 0 }, { 0, 5, 4, 4, 4, 0, 3 } },
};


// Non-temporal matrix loads in the deferred rounds of cached fp64 blocks
// (below 2 GiB; the launch shapes, piece size and stores stay the cached
// form's): bit NP (0 ... 4) of a read-only round with NP pending, bit
// kCapStore of a storing one, by block size class (defer_ntload_class).
// The solve loop over whole store cycles (tools/defer_profile.py
// --ntload-ab, 5 interleaved passes, profiles/r03_ntab_*.json), ms per round
// with the mask shipped vs cached loads throughout:
//   4096 x 8192 (256 MiB, the 256 MB MALL holds most of it)  0.0474, NT 0x1
//                                       0.0483 - every NT mask loses
//   8192^2 (512 MiB)     0x41  0.0954 vs 0.0997 (0x1 0.0955, 0x5f 0.0969)
//   2880 x 23040 (506 MiB, the P = 8 block)  0x41  0.0982 vs 0.1093
//   10240^2 (800 MiB)    0x5f  0.1499 vs 0.1586 (0x41 0.1536)
//   8192 x 16384, 12288^2, 14336^2 (1 - 1.5 GiB)  0x5f  0.1989 / 0.2146 /
//                        0.3022 vs 0.2071 / 0.2253 / 0.3182
// The post-store round (NP = 0) reads a matrix the storing round just
// wrote through the cache; once the block outgrows the MALL those lines
// only evict each other, and on the larger blocks every read-only round
// does better streaming past it.
// Generalised (tools/defer_profile.py --defer-cache-ab, 5 interleaved
// passes, two boxes, profiles/r03_dcab_*.json): per dtype and size class of
// every_cache_class (3 = the non-temporal form, from 2 GiB), bit NP / bit
// kCapStore turns the matrix loads' policy over (cached <-> non-temporal) in
// that round, bit 7 the storing round's stores'.  Cached fp32 blocks from
// 384 MiB gain like fp64 from non-temporal loads in the post-store and
// storing rounds (0x41): 10240^2 0.0764 vs 0.0792 ms per round, 12288^2
// 0.1091 / 0.1094 vs 0.1141 / 0.1146, 16384^2 0.1900 vs 0.1942, 20480^2
// 0.3103 vs 0.3182; below (8192^2 fp32, the 5824 x 11648 block) every mask
// loses.  On the non-temporal form every cached variant loses or ties
// (32768^2 fp64 0x1 / 0x3 / 0x1f 1.499 / 1.523 / 1.617 vs 1.481 ms, 0x40 /
// 0x80 1.478 / 1.485; fp32 0.739 - 0.758 vs 0.729; the P = 8 block 0.769 /
// 0.827 vs 0.760), so it keeps both non-temporal.
[[maybe_unused]] constexpr int kNtLoadClasses = 3; // st_set_defer_ntload: fp64, cached
constexpr int kDeferFlipClasses = 4;
std::atomic<uint32_t> g_defer_flip[2][kDeferFlipClasses] = {
  { 0u, 0x41u, 0x41u, 0u },      // fp32
  { 0u, 0x41u, 0x5fu, 0u },      // fp64
};
// bit 7: the storing round's stores turned over too
constexpr uint32_t kNtStoreBit = 7u;
[[maybe_unused]] constexpr uint32_t kNtLoadMask = 0xdfu;

// below 384 MiB, below 640 MiB, above (the cached fp64 classes of
// st_set_defer_ntload)
inline uint32_t
defer_ntload_class(size_t bytes)
{
  return bytes < ((size_t)384 << 20) ? 0u : bytes < ((size_t)640 << 20) ? 1u : 2u;
}

template <typename T>
inline uint32_t
defer_flip(uint32_t nrows, uint32_t ncols)
{
  return g_defer_flip[sizeof(T) == 8]
                     [every_cache_class(block_bytes(nrows, ncols, sizeof(T)))]
                       .load(std::memory_order_relaxed);
}

template <typename T, bool NT>
inline uint32_t
defer_lds(uint32_t slot)
{
  return defer_cap_lds(
    g_defer_caps[sizeof(T) == 8][NT][slot].load(std::memory_order_relaxed));
}

// Launch shape of the deferred rounds by pending count NP
// (flat_map_sweep (round 2, git history), profiles/r02_flat_map_shape_*.log and
// r02_flat_map_np5_*.log: 32768^2, 32768 / 16384 / 8192 x 65536 fp64
// non-temporal, 8192^2 / 12288^2 / 2880 x 23040 fp64 cached, 32768^2 and
// 8192^2 fp32):
//   NP = 0            2 rows per workgroup; non-temporal blocks in the
//                     piece-tiled order of 8 row groups (5-6 % at 32768^2)
//   NP = 1, 2         4 rows (the pending rounds' column scales then serve
//                     4 rows: 10-23 % at NP = 2; NP = 2 on non-temporal
//                     blocks 8 rows, 1-2 %), piece-tiled by 32 row groups
//                     on non-temporal blocks, 16 on cached ones
//   NP = 3, 4         8 rows (the column scales of 3 - 4 pending rounds then
//                     serve 8 rows: 3-10 % over 4 rows, NP = 4 at 32768^2
//                     fp64 1.230 vs 1.351 ms, profiles/r02_flat_map_r8_*.log),
//                     tiled by 16: on non-temporal blocks the row-major
//                     order's time depends on the allocation (32768^2 fp64
//                     NP = 3 1.25 or 1.33 ms from one allocation to the
//                     next, tiles of 16 1.20-1.22 in both;
//                     profiles/r02_rowload_merge_ab*.log)
//   storing rounds    row-major; 4 rows (10-16 % over 2), 8 on non-temporal
//                     blocks when rounds are pending (3 %: 32768^2 fp64
//                     2.852 vs 2.931 ms, 8192 x 65536 1.434 vs 1.481)
// (the every-round flat round has its own shapes: kFlatEveryRows /
// flat_every_tile above)
// rows per workgroup and piece tile (row groups, 0 = row-major) of a
// deferred round, by pending count and store: the table above, in one place
// for the launcher (template arguments) and st_launch_policy (tests and the
// pinned map, tests/golden/launch_policy.json)
template <typename T, bool NT>
constexpr int
defer_rows(int np, bool store)
{
  // NP = 0 on cached fp64 blocks: 1 row, tiles of 4 (the solve loop 0.3 -
  // 0.7 % faster per round at 8192^2 / 10240^2 / 12288^2,
  // profiles/r02_defer_cycle_ab_np0_cached.log); fp32 keeps 2 rows,
  // row-major (1 row: 18 % slower at 8192^2 fp32,
  // profiles/r02_flat_map_r1_f32_cached.log)
  // stores with pending rounds: 8 rows on non-temporal blocks, 4 cached
  // (8192^2 fp32 and the P = 8 block lose 3-5 % with 8 there); the cached
  // fp64 store with 5 pending: 8 (below)
  constexpr bool kF64C = !NT && sizeof(T) == 8;
  if (store)
    return np == 0 ? 4
           : np < 5 ? (NT ? 8 : 4)
                    : ((kF64C && ST_DEFER_STORE_R8_CACHED) ? 8 : (NT ? 8 : 4));
  return np == 0 ? (NT ? 2 : kF64C ? ST_DEFER_R0_CACHED : 2)
         : np == 1 ? 4
         : np == 2 ? (NT ? 8 : 4) // NP = 2: 1-2 % with 8 rows, non-temporal only
                   : 8;
}

template <typename T, bool NT>
constexpr uint32_t
defer_tile(int np, bool store)
{
  constexpr bool kF64C = !NT && sizeof(T) == 8;
  // storing rounds row-major, but the cached fp64 one with 5 pending (on
  // non-temporal blocks tiles of 4 ... 32 lose 0.3 - 6 %,
  // profiles/r04_ntstore.json)
  if (store)
    return (np >= 5 && kF64C && ST_DEFER_STORE_R8_CACHED) ? (uint32_t)ST_DEFER_TS5_CACHED
                                                           : 0u;
  return np == 0 ? (NT ? 8u : kF64C ? (uint32_t)ST_DEFER_PT0_CACHED : 0u)
         : np <= 2 ? (NT ? 32u : 16u)
                   : 16u;
}

template <typename T, int W, int ORDER, bool NT>
void
launch_flat_deferred(T* a, const T* s_cur, const T* inv_cur, T* s_next,
                     T* inv_next, T* part, T* v, uint32_t nrows,
                     uint32_t ncols, uint32_t row0, T eps, uint32_t k,
                     uint32_t max_itr, uint32_t semantics, st_state* st,
                     const T* const* pend_s, const T* const* pend_inv,
                     uint32_t npend, bool store, bool flush,
                     hipStream_t stream)
{
  // the matrix loads' / stores' cache policy turned over where
  // g_defer_flip says so (vector path only)
  constexpr int kV = W > 1 ? 1 : 0;
  const uint32_t fl = kV ? defer_flip<T>(nrows, ncols) : 0u;
#define ST_NPL(NPV, RV, STV, FLV, PTV, LDS)                                    \
  launch_flat_deferred_np<T, W, ORDER, NT, NPV, RV, STV, (FLV) * kV>(          \
    a, s_cur, inv_cur, s_next, inv_next, part, v, nrows, ncols, row0, eps, k,  \
    max_itr, semantics, st, pend_s, pend_inv, flush, PTV, LDS, stream)
#define ST_NP(NPV, LDS)                                                        \
  (((fl >> (NPV)) & 1u)                                                        \
     ? ST_NPL(NPV, (defer_rows<T, NT>(NPV, false)), false, 1,                  \
              (defer_tile<T, NT>(NPV, false)), LDS)                            \
     : ST_NPL(NPV, (defer_rows<T, NT>(NPV, false)), false, 0,                  \
              (defer_tile<T, NT>(NPV, false)), LDS))
#define ST_NPS1(NPV, FLV, LDS)                                                 \
  ST_NPL(NPV, (defer_rows<T, NT>(NPV, true)), true, FLV,                       \
         (defer_tile<T, NT>(NPV, true)), LDS)
#define ST_NPS(NPV, LDS)                                                       \
  (((fl >> kNtStoreBit) & 1u)                                                  \
     ? (((fl >> kCapStore) & 1u) ? ST_NPS1(NPV, 3, LDS) : ST_NPS1(NPV, 2, LDS)) \
     : (((fl >> kCapStore) & 1u) ? ST_NPS1(NPV, 1, LDS) : ST_NPS1(NPV, 0, LDS)))
  static_assert(kDeferRoundsMax == 6, "one case per pending count below");
  // shapes: defer_rows / defer_tile; caps: g_defer_caps
  if (store) {
    const uint32_t lds = defer_lds<T, NT>(kCapStore);
    switch (npend) {
    case 0: ST_NPS(0, lds); break;
    case 1: ST_NPS(1, lds); break;
    case 2: ST_NPS(2, lds); break;
    case 3: ST_NPS(3, lds); break;
    case 4: ST_NPS(4, lds); break;
    default: ST_NPS(5, lds); break;
    }
  } else {
    const uint32_t lds = defer_lds<T, NT>(npend < 5 ? npend : 4);
    switch (npend) {
    case 0: ST_NP(0, lds); break;
    case 1: ST_NP(1, lds); break;
    case 2: ST_NP(2, lds); break;
    case 3: ST_NP(3, lds); break;
    default: ST_NP(4, lds); break;
    }
  }
#undef ST_NPS1
#undef ST_NP
#undef ST_NPS
#undef ST_NPL
}

template <typename T>
int
launch_round_flat_deferred(T* a, const T* s_cur, const T* inv_cur, T* s_next,
                           T* inv_next, T* part, T* v, uint32_t nrows,
                           uint32_t ncols, uint32_t row0, T eps, uint32_t k,
                           uint32_t max_itr, uint32_t semantics, st_state* st,
                           const T* const* pend_s, const T* const* pend_inv,
                           uint32_t npend, bool store, bool flush,
                           hipStream_t stream)
{
  ST_REQUIRE(a && s_cur && inv_cur && part && v && st,
             "round_flat_deferred: null pointer");
  ST_REQUIRE(flush || (s_next && inv_next), "round_flat_deferred: null pointer");
  ST_REQUIRE(npend < defer_rounds(nrows, ncols, sizeof(T)),
             "round_flat_deferred: %u pending rounds", npend);
  // the m-th round of a group (m - 1 pending) is the storing one: a round
  // that does not store re-applies at most m - 2 (launch_flat_deferred has
  // no read-only kernel for m - 1)
  ST_REQUIRE(store || npend + 1 < defer_rounds(nrows, ncols, sizeof(T)),
             "round_flat_deferred: %u pending rounds without a store (the "
             "round with %u pending stores)",
             npend, defer_rounds(nrows, ncols, sizeof(T)) - 1);
  ST_REQUIRE(!flush || store, "round_flat_deferred: a flush stores");
  ST_REQUIRE(ncols > 0 && nrows > 0 && row0 + (uint64_t)nrows <= ncols,
             "round_flat_deferred: bad block");
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "round_flat_deferred: bad semantics");
  constexpr int W = 16 / sizeof(T);
  bool vec_ok = (ncols % W) == 0 && aligned16(a) && aligned16(s_cur);
  for (uint32_t i = 0; i < npend; i++)
    vec_ok = vec_ok && aligned16(pend_s[i]);
  const bool order1 = semantics == ST_SEM_MAINPY;
  const bool nt = flat_round_nt(nrows, ncols, sizeof(T));
#define ST_DEF(WW, OO, NN)                                                     \
  launch_flat_deferred<T, WW, OO, NN>(a, s_cur, inv_cur, s_next, inv_next,     \
                                      part, v, nrows, ncols, row0, eps, k,     \
                                      max_itr, semantics, st, pend_s,          \
                                      pend_inv, npend, store, flush, stream)
  if (vec_ok) {
    if (order1)
      nt ? ST_DEF(W, 1, true) : ST_DEF(W, 1, false);
    else
      nt ? ST_DEF(W, 0, true) : ST_DEF(W, 0, false);
  } else {
    if (order1)
      nt ? ST_DEF(1, 1, true) : ST_DEF(1, 1, false);
    else
      nt ? ST_DEF(1, 0, true) : ST_DEF(1, 0, false);
  }
#undef ST_DEF
  return check_launch("round_flat_deferred");
}

uint32_t
defer_rounds(uint32_t nrows, uint32_t ncols, size_t elem)
{
  // 6 everywhere: with the shapes above a read-only round with 1 ... 4
  // pending scalings costs 0-10 % more than the first one, so the group
  // that spreads one store over 6 rounds is 3-5 % faster per round than 4
  // (32768^2 fp64 1.55 vs 1.62 ms, 8192 x 65536 0.818 vs 0.842, 32768^2
  // fp32 0.762 vs 0.798; profiles/r02_flat_map_np5_*.log), and even on
  // cached fp64 blocks, where round 1 took 3
  (void)nrows;
  (void)ncols;
  (void)elem;
  return kDeferRoundsMax;
}

template <typename T>
int
launch_recip(const T* s, T* inv, uint32_t n, hipStream_t stream)
{
  ST_REQUIRE(s && inv, "recip: null pointer");
  const uint32_t grid = (n + kBlock - 1) / kBlock < 1024u ? (n + kBlock - 1) / kBlock
                                                          : 1024u;
  hipLaunchKernelGGL((dev::k_recip<T>), dim3(grid), dim3(kBlock), 0, stream, s,
                     inv, n);
  return check_launch("recip");
}

template int launch_round_flat_deferred<float>(
  float*, const float*, const float*, float*, float*, float*, float*, uint32_t,
  uint32_t, uint32_t, float, uint32_t, uint32_t, uint32_t, st_state*,
  const float* const*, const float* const*, uint32_t, bool, bool, hipStream_t);
template int launch_round_flat_deferred<double>(
  double*, const double*, const double*, double*, double*, double*, double*,
  uint32_t, uint32_t, uint32_t, double, uint32_t, uint32_t, uint32_t,
  st_state*, const double* const*, const double* const*, uint32_t, bool, bool,
  hipStream_t);
template int launch_recip<float>(const float*, float*, uint32_t, hipStream_t);
template int launch_recip<double>(const double*, double*, uint32_t,
                                  hipStream_t);

// ---- the flat round split in two for the overlapped exchange ------------
// span 1 (local): k_flat over the pieces holding [col0, col1), lanes masked
// to those columns, partials to the local region of `part`; span 2
// (remote): k_flat over every piece with the other columns and the fused
// stats, then k_parts sums remote-then-local partials (fixed order: the
// result does not depend on how the two launches interleave with the
// all-gather) and updates v.  `part` holds split_flat_scratch() elements:
// [nrows x flat_pieces(ncols, 1)] remote, then the local region.
inline size_t
split_flat_local_off(uint32_t nrows, uint32_t ncols)
{
  return flat_scratch_elems(nrows, ncols);
}

inline size_t
split_flat_scratch_elems(uint32_t nrows, uint32_t ncols, uint32_t col0,
                         uint32_t col1)
{
  return split_flat_local_off(nrows, ncols) +
         (size_t)nrows * (flat_pieces(col1 - col0, 1) + 1);
}

template <typename T, int W, int ORDER, bool NT>
void
launch_split_flat_cfg(int span, T* a, const T* s_cur, T* s_next, T* part,
                      T* v, uint32_t nrows, uint32_t ncols, uint32_t row0,
                      uint32_t col0, uint32_t col1, T eps, uint32_t k,
                      uint32_t max_itr, uint32_t semantics, st_state* st,
                      hipStream_t stream)
{
  constexpr int U = kFlatU<T, W, NT>;
  constexpr uint32_t PW = kBlock * W * U;
  const uint32_t ppr = flat_pieces(ncols, W * U);
  const uint32_t p_lo = col0 / PW;
  const uint32_t npl = col1 > col0 ? (col1 + PW - 1) / PW - p_lo : 0u;
  const uint32_t ngroups = (nrows + kFlatRows - 1) / kFlatRows;
  T* part_local = part + split_flat_local_off(nrows, ncols);
  if (span == 1) {
    if (npl == 0)
      return;
    const FlatGrid fl = flat_grid(ngroups * npl);
    // a local half short of the whole row streams non-temporally at every
    // size: cached, it would evict from the MALL what the remote half is
    // about to re-read (profiles/r01_split_cost.log)
    if (NT || col1 - col0 < ncols)
      hipLaunchKernelGGL(
        (dev::k_flat<T, W, ORDER, true, kFlatRows, false, kFlatAlt, 1, -1, U>),
        fl.grid, dim3(kBlock), 0, stream, a, s_cur, part_local, v, nrows, ncols,
        npl, row0, k, st, eps, max_itr, semantics, p_lo, col0, col1,
        dev::FlatPending<T, -1>{}, fl.gx2);
    else
      hipLaunchKernelGGL(
        (dev::k_flat<T, W, ORDER, false, kFlatRows, false, kFlatAlt, 1, -1, U>),
        fl.grid, dim3(kBlock), 0, stream, a, s_cur, part_local, v, nrows, ncols,
        npl, row0, k, st, eps, max_itr, semantics, p_lo, col0, col1,
        dev::FlatPending<T, -1>{}, fl.gx2);
    return;
  }
  // row group 0 over every piece (it takes the stats), the other row
  // groups only over pieces holding remote columns
  uint32_t pa, nfull;
  dev::split_full_pieces<PW>(ncols, ppr, col0, col1, pa, nfull);
  const FlatGrid fr = flat_grid(ppr + (ngroups - 1) * (ppr - nfull));
  hipLaunchKernelGGL(
    (dev::k_flat<T, W, ORDER, NT, kFlatRows, true, kFlatAlt, 2, -1, U>),
    fr.grid, dim3(kBlock), 0, stream, a, s_cur, part, v, nrows, ncols, ppr,
    row0, k, st, eps, max_itr, semantics, 0u, col0, col1,
    dev::FlatPending<T, -1>{}, fr.gx2);
  const uint32_t pgrid = (nrows + dev::kWaves - 1) / dev::kWaves;
  hipLaunchKernelGGL((dev::k_parts<T>), dim3(pgrid), dim3(kBlock), 0, stream,
                     part, s_next, nrows, ppr, k, st, s_cur, v, row0,
                     (const T*)part_local, npl, pa, nfull);
}

template <typename T>
int
launch_round_split_flat(int span, T* a, const T* s_cur, T* s_next, T* part,
                        T* v, uint32_t nrows, uint32_t ncols, uint32_t row0,
                        uint32_t col0, uint32_t col1, T eps, uint32_t k,
                        uint32_t max_itr, uint32_t semantics, st_state* st,
                        hipStream_t stream)
{
  ST_REQUIRE(a && s_cur && part && st, "round_split_flat: null pointer");
  ST_REQUIRE(span == 1 || span == 2, "round_split_flat: span must be 1 "
                                     "(local) or 2 (remote), not %d", span);
  ST_REQUIRE(span == 1 || (s_next && v), "round_split_flat: null pointer");
  ST_REQUIRE(ncols > 0 && nrows > 0, "round_split_flat: empty block");
  ST_REQUIRE(row0 + (uint64_t)nrows <= ncols,
             "round_split_flat: rows [%u, %u) outside the %u-long row-sum "
             "vector", row0, row0 + nrows, ncols);
  ST_REQUIRE(col0 <= col1 && col1 <= ncols,
             "round_split_flat: bad local column range [%u, %u) of %u", col0,
             col1, ncols);
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "round_split_flat: bad semantics %u",
             semantics);
  ST_REQUIRE(max_itr > 0, "round_split_flat: max_itr must be > 0");
  ST_REQUIRE((uint64_t)((nrows + kFlatRows - 1) / kFlatRows) *
                 flat_pieces(ncols, 1) <
               (1ull << 31),
             "round_split_flat: %u x %u is too large for one launch", nrows,
             ncols);
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && (col0 % W) == 0 && (col1 % W) == 0 &&
                      aligned16(a) && aligned16(s_cur);
  const bool order1 = semantics == ST_SEM_MAINPY;
  const bool nt = flat_round_nt(nrows, ncols, sizeof(T));
#define ST_SFLAT(WW, OO, NN)                                                   \
  launch_split_flat_cfg<T, WW, OO, NN>(span, a, s_cur, s_next, part, v, nrows, \
                                       ncols, row0, col0, col1, eps, k,        \
                                       max_itr, semantics, st, stream)
  if (vec_ok) {
    if (order1)
      nt ? ST_SFLAT(W, 1, true) : ST_SFLAT(W, 1, false);
    else
      nt ? ST_SFLAT(W, 0, true) : ST_SFLAT(W, 0, false);
  } else {
    if (order1)
      nt ? ST_SFLAT(1, 1, true) : ST_SFLAT(1, 1, false);
    else
      nt ? ST_SFLAT(1, 0, true) : ST_SFLAT(1, 0, false);
  }
#undef ST_SFLAT
  return check_launch("round_split_flat");
}

size_t
round_flat_scratch(uint32_t nrows, uint32_t ncols)
{
  return flat_scratch_elems(nrows, ncols);
}

bool
round_flat_pays(uint32_t nrows, uint32_t ncols, size_t elem)
{
  return flat_round_pays(nrows, ncols, elem);
}

template <typename T>
int
launch_rowsum(const T* a, T* s, uint32_t nrows, uint32_t ncols,
              hipStream_t stream)
{
  ST_REQUIRE(a && s, "rowsum: null pointer");
  if (nrows == 0)
    return 0;
  ST_REQUIRE(ncols > 0, "rowsum: ncols must be > 0");
  launch_vec<T, false, true, 0>(const_cast<T*>(a), nullptr, s, nrows, ncols, 0,
                                nullptr, stream);
  return check_launch("rowsum");
}

// K0's walk order (k_flat_sum's rev): -1 = reversed where the loads go
// through the caches (the block is memory-side-cacheable), 0 = front to back
// (the default), 1 = reversed; st_set_k0_reverse (tuning build)
std::atomic<int> g_k0_rev{ 0 };

// K0 in the flat form (k_flat_sum + k_parts) for blocks where the flat round
// pays: the pieces (kFlatU), rows per workgroup and walk order (defer_rows /
// defer_tile), workgroups-per-CU cap and load policy (g_defer_flip bit 0) of
// the deferred form's read-only round with nothing pending, which streams
// the same bytes - a matrix just written, like A_0 after its generator or
// copy - without the scaling.  k_parts runs ungated (no state).
template <typename T, int W, bool NT>
void
launch_rowsum_flat_cfg(const T* a, T* s, T* part, uint32_t nrows, uint32_t ncols,
                       hipStream_t stream)
{
  constexpr int U = kFlatU<T, W, NT>;
  constexpr int R = defer_rows<T, NT>(0, false);
  const uint32_t ppr = flat_pieces(ncols, W * U);
  const uint32_t pt = defer_tile<T, NT>(0, false);
  const uint32_t lds = defer_lds<T, NT>(0);
  const FlatGrid fg = flat_grid((nrows + R - 1) / R * ppr);
  const bool flip = W > 1 && (defer_flip<T>(nrows, ncols) & 1u) != 0;
  const int rv = g_k0_rev.load(std::memory_order_relaxed);
  const uint32_t rev = rv < 0 ? (NT == flip ? 1u : 0u) : (uint32_t)rv;
  if (NT != flip)
    hipLaunchKernelGGL((dev::k_flat_sum<T, W, true, R, U>), fg.grid, dim3(kBlock), lds,
                       stream, a, part, nrows, ncols, ppr, pt, fg.gx2, rev);
  else
    hipLaunchKernelGGL((dev::k_flat_sum<T, W, false, R, U>), fg.grid, dim3(kBlock), lds,
                       stream, a, part, nrows, ncols, ppr, pt, fg.gx2, rev);
  launch_parts<T>(part, s, nrows, ppr, 0u, nullptr, nullptr, nullptr, 0u, nullptr, stream);
}

template <typename T>
int
launch_rowsum_flat(const T* a, T* s, T* part, uint32_t nrows, uint32_t ncols,
                   hipStream_t stream)
{
  ST_REQUIRE(a && s && part, "rowsum_flat: null pointer");
  if (nrows == 0)
    return 0;
  ST_REQUIRE(ncols > 0, "rowsum_flat: ncols must be > 0");
  constexpr int W = 16 / sizeof(T);
  const bool vec_ok = (ncols % W) == 0 && aligned16(a);
  const bool nt = flat_round_nt(nrows, ncols, sizeof(T));
  if (vec_ok)
    nt ? launch_rowsum_flat_cfg<T, W, true>(a, s, part, nrows, ncols, stream)
       : launch_rowsum_flat_cfg<T, W, false>(a, s, part, nrows, ncols, stream);
  else
    nt ? launch_rowsum_flat_cfg<T, 1, true>(a, s, part, nrows, ncols, stream)
       : launch_rowsum_flat_cfg<T, 1, false>(a, s, part, nrows, ncols, stream);
  return check_launch("rowsum_flat");
}

template int launch_rowsum_flat<float>(const float*, float*, float*, uint32_t, uint32_t,
                                       hipStream_t);
template int launch_rowsum_flat<double>(const double*, double*, double*, uint32_t,
                                        uint32_t, hipStream_t);

template <typename T>
int
launch_scale_rowsum(T* a, const T* s_cur, T* s_next, uint32_t nrows,
                    uint32_t ncols, uint32_t row0, uint32_t semantics,
                    const st_state* st, hipStream_t stream)
{
  ST_REQUIRE(a && s_cur, "scale_rowsum: null pointer");
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "scale_rowsum: bad semantics %u",
             semantics);
  if (nrows == 0)
    return 0;
  ST_REQUIRE(ncols > 0, "scale_rowsum: ncols must be > 0");
  const bool order1 = semantics == ST_SEM_MAINPY;
  if (s_next) {
    if (order1)
      launch_vec<T, true, true, 1>(a, s_cur, s_next, nrows, ncols, row0, st,
                                   stream);
    else
      launch_vec<T, true, true, 0>(a, s_cur, s_next, nrows, ncols, row0, st,
                                   stream);
  } else {
    if (order1)
      launch_vec<T, true, false, 1>(a, s_cur, nullptr, nrows, ncols, row0, st,
                                    stream);
    else
      launch_vec<T, true, false, 0>(a, s_cur, nullptr, nrows, ncols, row0, st,
                                    stream);
  }
  return check_launch("scale_rowsum");
}

template <typename T>
int
launch_epilogue(const T* s, T* v, uint32_t n, T eps, uint32_t max_itr,
                uint32_t semantics, st_state* st, hipStream_t stream)
{
  ST_REQUIRE(s && st, "epilogue: null pointer");
  ST_REQUIRE(n > 0, "epilogue: n must be > 0");
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "epilogue: bad semantics %u",
             semantics);
  hipLaunchKernelGGL(dev::k_epilogue<T>, dim3(1), dim3(kEpiBlock), 0, stream,
                     s, v, n, eps, max_itr, semantics, st);
  return check_launch("epilogue");
}

int
launch_state_mirror(const st_state* d_state, st_state* h_state, hipStream_t stream)
{
  ST_REQUIRE(d_state && h_state, "state_mirror: null pointer");
  hipLaunchKernelGGL(dev::k_state_mirror, dim3(1), dim3(64), 0, stream,
                     reinterpret_cast<const uint32_t*>(d_state),
                     reinterpret_cast<uint32_t*>(h_state));
  return check_launch("state_mirror");
}

template <typename T>
int
launch_fill(T* x, uint64_t count, T value, hipStream_t stream)
{
  ST_REQUIRE(x || count == 0, "fill: null pointer");
  if (count == 0)
    return 0;
  uint64_t blocks = (count + kBlock - 1) / kBlock;
  const uint32_t grid = (uint32_t)(blocks < 8192 ? blocks : 8192);
  hipLaunchKernelGGL(dev::k_fill<T>, dim3(grid), dim3(kBlock), 0, stream, x,
                     count, value);
  return check_launch("fill");
}

template <typename T, int KIND>
int
launch_generate(T* a, uint32_t nrows, uint32_t ncols, uint32_t row0,
                uint64_t seed, hipStream_t stream)
{
  ST_REQUIRE(a || nrows == 0 || ncols == 0, "generate: null pointer");
  if (nrows == 0 || ncols == 0)
    return 0;
  const uint32_t grid = nrows < 65536 ? nrows : 65536;
  hipLaunchKernelGGL((dev::k_generate<T, KIND>), dim3(grid), dim3(kBlock), 0,
                     stream, a, nrows, ncols, row0, seed);
  return check_launch("generate");
}

template <typename T>
bool
solve_small_fits(const T* a, uint32_t n)
{
  constexpr uint32_t W = 16 / sizeof(T);
  return n > 0 && n <= dev::small_solve_max_n<T>() && n % W == 0 &&
         aligned16(a);
}

template <typename T>
int
launch_solve_small(T* a, T* v, uint32_t n, T eps, uint32_t max_itr,
                   uint32_t semantics, st_state* st, hipStream_t stream)
{
  ST_REQUIRE(a && v && st, "solve_small: null pointer");
  ST_REQUIRE(solve_small_fits<T>(a, n),
             "solve_small: n = %u does not fit one workgroup", n);
  ST_REQUIRE(semantics <= ST_SEM_MAINPY, "solve_small: bad semantics %u",
             semantics);
  ST_REQUIRE(max_itr > 0, "solve_small: max_itr must be > 0");
  // rows per wave: the power of two >= ceil(n / 16)
  const uint32_t rows = (n + dev::kSmallWaves - 1) / dev::kSmallWaves;
  auto go = [&](auto order, auto rpw) {
    hipLaunchKernelGGL(
      (dev::k_solve_small<T, decltype(order)::value, decltype(rpw)::value>),
      dim3(1), dim3(dev::kSmallBlock), 0, stream, a, v, n, eps, max_itr,
      semantics, st);
  };
  auto by_rows = [&](auto order) {
    if (rows <= 1)
      go(order, std::integral_constant<int, 1>{});
    else if (rows <= 2)
      go(order, std::integral_constant<int, 2>{});
    else if (rows <= 4)
      go(order, std::integral_constant<int, 4>{});
    else if constexpr (sizeof(T) == 8)
      go(order, std::integral_constant<int, 8>{});
    else if (rows <= 8)
      go(order, std::integral_constant<int, 8>{});
    else
      go(order, std::integral_constant<int, 16>{});
  };
  if (semantics == ST_SEM_MAINPY)
    by_rows(std::integral_constant<int, 1>{});
  else
    by_rows(std::integral_constant<int, 0>{});
  return check_launch("solve_small");
}

template bool solve_small_fits<float>(const float*, uint32_t);
template bool solve_small_fits<double>(const double*, uint32_t);
template int launch_solve_small<float>(float*, float*, uint32_t, float,
                                       uint32_t, uint32_t, st_state*,
                                       hipStream_t);
template int launch_solve_small<double>(double*, double*, uint32_t, double,
                                        uint32_t, uint32_t, st_state*,
                                        hipStream_t);
template int launch_rowsum<float>(const float*, float*, uint32_t, uint32_t,
                                  hipStream_t);
template int launch_rowsum<double>(const double*, double*, uint32_t, uint32_t,
                                   hipStream_t);
template int launch_scale_rowsum<float>(float*, const float*, float*, uint32_t,
                                        uint32_t, uint32_t, uint32_t,
                                        const st_state*, hipStream_t);
template int launch_scale_rowsum<double>(double*, const double*, double*,
                                         uint32_t, uint32_t, uint32_t,
                                         uint32_t, const st_state*,
                                         hipStream_t);
template int launch_epilogue<float>(const float*, float*, uint32_t, float,
                                    uint32_t, uint32_t, st_state*,
                                    hipStream_t);
template int launch_epilogue<double>(const double*, double*, uint32_t, double,
                                     uint32_t, uint32_t, st_state*,
                                     hipStream_t);
template int launch_round<float>(float*, const float*, float*, float*,
                                 uint32_t, uint32_t, uint32_t, float, uint32_t,
                                 uint32_t, uint32_t, st_state*, hipStream_t);
template int launch_round<double>(double*, const double*, double*, double*,
                                  uint32_t, uint32_t, uint32_t, double,
                                  uint32_t, uint32_t, uint32_t, st_state*,
                                  hipStream_t);
template int launch_round_flat<float>(float*, const float*, float*, float*,
                                     float*, uint32_t, uint32_t, uint32_t,
                                     float, uint32_t, uint32_t, uint32_t,
                                     st_state*, hipStream_t);
template int launch_round_flat<double>(double*, const double*, double*,
                                      double*, double*, uint32_t, uint32_t,
                                      uint32_t, double, uint32_t, uint32_t,
                                      uint32_t, st_state*, hipStream_t);
template int launch_mfree<float>(const float*, const float*, float*,
                                 const float*, float*, uint32_t, uint32_t,
                                 uint32_t, float, uint32_t, uint32_t, uint32_t,
                                 st_state*, hipStream_t);
template int launch_mfree<double>(const double*, const double*, double*,
                                  const double*, double*, uint32_t, uint32_t,
                                  uint32_t, double, uint32_t, uint32_t,
                                  uint32_t, st_state*, hipStream_t);
template int launch_fill<float>(float*, uint64_t, float, hipStream_t);
template int launch_fill<double>(double*, uint64_t, double, hipStream_t);

// ---- the launch policy, as one map (st_launch_policy) ---------------------
// What the solve loops launch for a block, read from the same functions and
// tables the launchers above use (round_shape / mfree_shape, kFlatEveryRows
// / flat_every_tile / g_every_cache / g_every_caps, defer_rows / defer_tile
// / g_defer_flip / g_defer_caps), so the pinned map
// (tests/golden/launch_policy.json, tools/launch_policy_table.py) changes
// whenever a launch does.  Vector path (ncols a multiple of 16 / b).
namespace {
template <typename T, bool NT>
int
policy_flat(uint32_t nrows, uint32_t ncols, int form, uint32_t np,
            st_launch_policy* o)
{
  constexpr int W = 16 / sizeof(T);
  o->piece_bytes = (uint32_t)(kBlock * W * kFlatU<T, W, NT> * sizeof(T));
  o->grid = 0;
  o->alt = kFlatAlt != 0;
  const uint32_t cls = every_cache_class(block_bytes(nrows, ncols, sizeof(T)));
  if (form == ST_FORM_ROUND) {
    const uint32_t pol = g_every_cache[cls].load(std::memory_order_relaxed);
    o->kernel = ST_KERNEL_FLAT;
    o->rows = kFlatEveryRows<T, NT>;
    o->tile = flat_every_tile<T, NT>(nrows, ncols);
    o->cap = g_every_caps[cls].load(std::memory_order_relaxed);
    o->load_nt = NT != ((pol & 1u) != 0);
    o->store_nt = NT != ((pol & 2u) != 0);
    return 0;
  }
  if (form == ST_FORM_ROWSUM) { // K0: launch_rowsum_flat_cfg
    o->kernel = ST_KERNEL_FLAT_SUM;
    o->rows = defer_rows<T, NT>(0, false);
    o->tile = defer_tile<T, NT>(0, false);
    o->cap = g_defer_caps[sizeof(T) == 8][NT][0].load(std::memory_order_relaxed);
    o->load_nt = NT != ((defer_flip<T>(nrows, ncols) & 1u) != 0);
    o->store_nt = -1;
    const int rv = g_k0_rev.load(std::memory_order_relaxed);
    o->alt = rv < 0 ? (o->load_nt ? 0 : 1) : rv; // launch_rowsum_flat_cfg's rev
    return 0;
  }
  const bool store = form == ST_FORM_DEFER_STORE;
  ST_REQUIRE(np < kDeferRoundsMax && (store || np + 1 < kDeferRoundsMax),
             "st_launch_policy: %u pending rounds %s", np,
             store ? "(at most 5)" : "without a store (at most 4)");
  const uint32_t fl = defer_flip<T>(nrows, ncols);
  o->kernel = ST_KERNEL_FLAT_DEFERRED;
  o->rows = defer_rows<T, NT>((int)np, store);
  o->tile = defer_tile<T, NT>((int)np, store);
  o->cap = g_defer_caps[sizeof(T) == 8][NT][store ? kCapStore : (np < 5 ? np : 4)].load(
    std::memory_order_relaxed);
  o->load_nt = NT != (((fl >> (store ? (uint32_t)kCapStore : np)) & 1u) != 0);
  o->store_nt = store ? (int)((NT || ST_DEFER_STORE_NT) != (((fl >> kNtStoreBit) & 1u) != 0))
                      : -1;
  return 0;
}

template <typename T>
int
policy(uint32_t nrows, uint32_t ncols, int form, uint32_t np, st_launch_policy* o)
{
  std::memset(o, 0, sizeof(*o));
  if (form == ST_FORM_MFREE) {
    const Shape sh = mfree_shape(nrows, ncols, sizeof(T));
    o->kernel = ST_KERNEL_MFREE;
    o->rows = sh.rows;
    o->grid = sh.grid;
    o->load_nt = sh.nt;
    o->store_nt = -1;
    o->alt = 1;
    return 0;
  }
  if (form == ST_FORM_ROWSUM && !round_flat_pays(nrows, ncols, sizeof(T))) {
    // K0 below the flat round: k_fused (launch_rows)
    const bool nt = fused_nt(nrows, ncols, sizeof(T));
    o->kernel = ST_KERNEL_FUSED;
    o->rows = nrows < 2 * kGridCap ? 1 : nt ? 4 : kRows;
    o->grid = kGridCap;
    o->load_nt = nt;
    o->store_nt = -1;
    return 0;
  }
  if (!round_flat_pays(nrows, ncols, sizeof(T))) {
    ST_REQUIRE(form == ST_FORM_ROUND,
               "st_launch_policy: deferred writes need the flat round (>= 144 MiB)");
    const Shape sh = round_shape(nrows, ncols, sizeof(T));
    o->kernel = ST_KERNEL_ROUND;
    o->rows = sh.rows;
    o->grid = sh.grid;
    o->load_nt = o->store_nt = sh.nt;
    o->alt = 1;
    return 0;
  }
  return flat_round_nt(nrows, ncols, sizeof(T))
           ? policy_flat<T, true>(nrows, ncols, form, np, o)
           : policy_flat<T, false>(nrows, ncols, form, np, o);
}
} // namespace

} // namespace st

// ---------------------------------------------------------------------------
// step-level C-ABI (similarity_transform.h, layer 4)
// ---------------------------------------------------------------------------
#define ST_STREAM(p) (reinterpret_cast<hipStream_t>(p))

extern "C" {

int
st_state_reset(st_state* d_state, void* stream)
{
  st::clear_error();
  ST_REQUIRE(d_state, "st_state_reset: null state");
  ST_CHECK(hipMemsetAsync(d_state, 0, sizeof(st_state), ST_STREAM(stream)));
  return 0;
}

#define ST_STEP_EXPORTS(T, SFX)                                                \
  int st_generate_hilbert_##SFX(T* d_mat, unsigned int nrows,                  \
                                unsigned int ncols, unsigned int row0,         \
                                void* stream)                                  \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_generate<T, st::dev::kHilbert>(d_mat, nrows, ncols,      \
                                                     row0, 0,                  \
                                                     ST_STREAM(stream));       \
  }                                                                            \
  int st_generate_random_##SFX(T* d_mat, unsigned int nrows,                   \
                               unsigned int ncols, unsigned int row0,          \
                               uint64_t seed, void* stream)                    \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_generate<T, st::dev::kRandom>(d_mat, nrows, ncols, row0, \
                                                    seed, ST_STREAM(stream));  \
  }                                                                            \
  int st_generate_identity_##SFX(T* d_mat, unsigned int nrows,                 \
                                 unsigned int ncols, unsigned int row0,        \
                                 void* stream)                                 \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_generate<T, st::dev::kIdentity>(                         \
      d_mat, nrows, ncols, row0, 0, ST_STREAM(stream));                        \
  }                                                                            \
  int st_fill_##SFX(T* d_x, uint64_t count, T value, void* stream)             \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_fill<T>(d_x, count, value, ST_STREAM(stream));           \
  }                                                                            \
  int st_rowsum_##SFX(const T* d_mat, T* d_s, unsigned int nrows,              \
                      unsigned int ncols, void* stream)                        \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_rowsum<T>(d_mat, d_s, nrows, ncols, ST_STREAM(stream)); \
  }                                                                            \
  int st_rowsum_flat_##SFX(const T* d_mat, T* d_s, T* d_part,                  \
                           unsigned int nrows, unsigned int ncols,             \
                           void* stream)                                       \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_rowsum_flat<T>(d_mat, d_s, d_part, nrows, ncols,         \
                                     ST_STREAM(stream));                       \
  }                                                                            \
  int st_scale_rowsum_##SFX(T* d_mat, const T* d_s_cur, T* d_s_next,           \
                            unsigned int nrows, unsigned int ncols,            \
                            unsigned int row0, unsigned int semantics,         \
                            const st_state* d_state, void* stream)             \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_scale_rowsum<T>(d_mat, d_s_cur, d_s_next, nrows, ncols,  \
                                      row0, semantics, d_state,                \
                                      ST_STREAM(stream));                      \
  }                                                                            \
  int st_round_##SFX(T* d_mat, const T* d_s_cur, T* d_s_next, T* d_v,          \
                     unsigned int nrows, unsigned int ncols,                   \
                     unsigned int row0, T eps, unsigned int k,                 \
                     unsigned int max_itr, unsigned int semantics,             \
                     st_state* d_state, void* stream)                          \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_round<T>(d_mat, d_s_cur, d_s_next, d_v, nrows, ncols,    \
                               row0, eps, k, max_itr, semantics, d_state,      \
                               ST_STREAM(stream));                             \
  }                                                                            \
  int st_round_flat_##SFX(T* d_mat, const T* d_s_cur, T* d_s_next,            \
                          T* d_part, T* d_v, unsigned int nrows,               \
                          unsigned int ncols, unsigned int row0, T eps,        \
                          unsigned int k, unsigned int max_itr,                \
                          unsigned int semantics, st_state* d_state,           \
                          void* stream)                                        \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_round_flat<T>(d_mat, d_s_cur, d_s_next, d_part, d_v,     \
                                    nrows, ncols, row0, eps, k, max_itr,       \
                                    semantics, d_state, ST_STREAM(stream));    \
  }                                                                            \
  int st_round_split_##SFX(T* d_mat, const T* d_s_cur, T* d_s_next,           \
                           T* d_part, T* d_v, unsigned int nrows,              \
                           unsigned int ncols, unsigned int row0,              \
                           unsigned int col0, unsigned int col1, T eps,        \
                           unsigned int k, unsigned int max_itr,               \
                           unsigned int semantics, int span,                   \
                           st_state* d_state, void* stream)                    \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_round_split<T>(span, d_mat, d_s_cur, d_s_next, d_part,   \
                                     d_v, nrows, ncols, row0, col0, col1, eps, \
                                     k, max_itr, semantics, d_state,           \
                                     ST_STREAM(stream));                       \
  }                                                                            \
  int st_round_split_flat_##SFX(T* d_mat, const T* d_s_cur, T* d_s_next,      \
                                T* d_part, T* d_v, unsigned int nrows,         \
                                unsigned int ncols, unsigned int row0,         \
                                unsigned int col0, unsigned int col1, T eps,   \
                                unsigned int k, unsigned int max_itr,          \
                                unsigned int semantics, int span,              \
                                st_state* d_state, void* stream)               \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_round_split_flat<T>(                                     \
      span, d_mat, d_s_cur, d_s_next, d_part, d_v, nrows, ncols, row0, col0,   \
      col1, eps, k, max_itr, semantics, d_state, ST_STREAM(stream));           \
  }                                                                            \
  int st_mfree_round_##SFX(const T* d_mat0, const T* d_s_prev, T* d_s_next,    \
                           const T* d_v_prev, T* d_v_cur, unsigned int nrows,  \
                           unsigned int ncols, unsigned int row0, T eps,       \
                           unsigned int k, unsigned int max_itr,               \
                           unsigned int semantics, st_state* d_state,          \
                           void* stream)                                       \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_mfree<T>(d_mat0, d_s_prev, d_s_next, d_v_prev, d_v_cur,  \
                               nrows, ncols, row0, eps, k, max_itr, semantics, \
                               d_state, ST_STREAM(stream));                    \
  }                                                                            \
  int st_mfree_round_flat_##SFX(const T* d_mat0, const T* d_s_prev,            \
                                T* d_s_next, const T* d_v_prev, T* d_v_cur,    \
                                T* d_part, unsigned int nrows,                 \
                                unsigned int ncols, unsigned int row0, T eps,  \
                                unsigned int k, unsigned int max_itr,          \
                                unsigned int semantics, st_state* d_state,     \
                                void* stream)                                  \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_mfree_flat<T>(d_mat0, d_s_prev, d_s_next, d_v_prev,      \
                                    d_v_cur, d_part, nrows, ncols, row0, eps,  \
                                    k, max_itr, semantics, d_state,            \
                                    ST_STREAM(stream));                        \
  }                                                                            \
  int st_epilogue_##SFX(const T* d_s, T* d_v, unsigned int n, T eps,           \
                        unsigned int max_itr, unsigned int semantics,          \
                        st_state* d_state, void* stream)                       \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_epilogue<T>(d_s, d_v, n, eps, max_itr, semantics,        \
                                  d_state, ST_STREAM(stream));                 \
  }

ST_STEP_EXPORTS(float, f32)
ST_STEP_EXPORTS(double, f64)

#define ST_DEFER_EXPORTS(T, SFX)                                               \
  int st_round_flat_deferred_##SFX(                                            \
    T* d_mat, const T* d_s_cur, const T* d_inv_cur, T* d_s_next,               \
    T* d_inv_next, T* d_part, T* d_v, unsigned int nrows, unsigned int ncols,  \
    unsigned int row0, T eps, unsigned int k, unsigned int max_itr,            \
    unsigned int semantics, const T* const* d_pend_s,                          \
    const T* const* d_pend_inv, unsigned int npend, int store, int flush,      \
    st_state* d_state, void* stream)                                           \
  {                                                                            \
    st::clear_error();                                                         \
    if (npend > 0 && (!d_pend_s || !d_pend_inv)) {                             \
      st::set_error("round_flat_deferred: null pending list");                \
      return -1;                                                               \
    }                                                                          \
    return st::launch_round_flat_deferred<T>(                                  \
      d_mat, d_s_cur, d_inv_cur, d_s_next, d_inv_next, d_part, d_v, nrows,     \
      ncols, row0, eps, k, max_itr, semantics, d_state, d_pend_s, d_pend_inv,  \
      npend, store != 0, flush != 0, ST_STREAM(stream));                       \
  }                                                                            \
  int st_recip_##SFX(const T* d_s, T* d_inv, unsigned int n, void* stream)     \
  {                                                                            \
    st::clear_error();                                                         \
    return st::launch_recip<T>(d_s, d_inv, n, ST_STREAM(stream));              \
  }

ST_DEFER_EXPORTS(float, f32)
ST_DEFER_EXPORTS(double, f64)

const char*
st_probe_switches(void)
{
  return ST_PROBES_DEFAULT
           ? "defaults"
           : "ST_DPP_NOINIT=" ST_STR(ST_DPP_NOINIT) " ST_ROW_VLOAD=" ST_STR(
               ST_ROW_VLOAD) " ST_FLAT_UNMASKED=" ST_STR(ST_FLAT_UNMASKED)
               " ST_DEFER_STORE_NT=" ST_STR(ST_DEFER_STORE_NT)
                 " ST_EVERY_CACHED_R1=" ST_STR(ST_EVERY_CACHED_R1)
                   " ST_DEFER_R0_CACHED=" ST_STR(ST_DEFER_R0_CACHED)
                     " ST_DEFER_PT0_CACHED=" ST_STR(ST_DEFER_PT0_CACHED)
                       " ST_DEFER_STORE_R8_CACHED=" ST_STR(
                         ST_DEFER_STORE_R8_CACHED) " ST_DEFER_TS5_CACHED=" ST_STR(
                           ST_DEFER_TS5_CACHED) " ST_FLAT_ALT=" ST_STR(ST_FLAT_ALT);
}

unsigned int
st_defer_rounds(unsigned int nrows, unsigned int ncols, int dtype)
{
  return st::defer_rounds(nrows, ncols, dtype == 1 ? 8 : 4);
}

uint64_t
st_round_flat_scratch(unsigned int nrows, unsigned int ncols)
{
  return st::round_flat_scratch(nrows, ncols);
}

uint64_t
st_round_split_flat_scratch(unsigned int nrows, unsigned int ncols,
                            unsigned int col0, unsigned int col1)
{
  if (col1 < col0)
    return 0;
  return st::split_flat_scratch_elems(nrows, ncols, col0, col1);
}

int
st_launch_policy_query(int dtype, unsigned int nrows, unsigned int ncols, int form,
                       unsigned int npend, st_launch_policy* out)
{
  st::clear_error();
  ST_REQUIRE(out, "st_launch_policy: null output");
  ST_REQUIRE(dtype == 0 || dtype == 1, "st_launch_policy: dtype 0 (fp32) or 1 (fp64)");
  ST_REQUIRE(nrows > 0 && ncols > 0 && ncols % (dtype == 1 ? 2u : 4u) == 0,
             "st_launch_policy: a block of whole 16-byte chunks per row");
  ST_REQUIRE(form >= ST_FORM_ROUND && form <= ST_FORM_ROWSUM, "st_launch_policy: form 0..4");
  return dtype == 1 ? st::policy<double>(nrows, ncols, form, npend, out)
                    : st::policy<float>(nrows, ncols, form, npend, out);
}

int
st_round_flat_pays(unsigned int nrows, unsigned int ncols, int dtype)
{
  return st::round_flat_pays(nrows, ncols, dtype == 1 ? 8 : 4) ? 1 : 0;
}

// ---- tuning setters (include/st_tuning.h): the tuning build only -------
// (libsimilarity_transform_tuning.so, -DST_TUNING_ABI=1; the library the
// drop-in callers load exports none of them)
#if ST_TUNING_ABI
int
st_set_defer_caps(int dtype, int nontemporal, unsigned int slot,
                  unsigned int wg_per_cu)
{
  st::clear_error();
  if ((dtype != 0 && dtype != 1) || slot > (unsigned)st::kCapStore ||
      (wg_per_cu == 1 || wg_per_cu > 32)) {
    st::set_error("st_set_defer_caps: dtype 0/1, slot 0..6, cap 0 or 2..32");
    return -1;
  }
  return (int)st::g_defer_caps[dtype][nontemporal != 0][slot].exchange(
    wg_per_cu, std::memory_order_relaxed);
}

int
st_set_defer_ntload(unsigned int size_class, unsigned int mask)
{
  st::clear_error();
  if (size_class >= (unsigned)st::kNtLoadClasses ||
      (mask & ~st::kNtLoadMask) != 0) {
    st::set_error("st_set_defer_ntload: size class 0..2, mask of bits 0..4, 6 and 7");
    return -1;
  }
  return (int)st::g_defer_flip[1][size_class].exchange(mask,
                                                       std::memory_order_relaxed);
}

int
st_set_defer_cache(int dtype, unsigned int size_class, unsigned int mask)
{
  st::clear_error();
  if ((dtype != 0 && dtype != 1) || size_class >= (unsigned)st::kDeferFlipClasses ||
      (mask & ~st::kNtLoadMask) != 0) {
    st::set_error("st_set_defer_cache: dtype 0/1, size class 0..3, mask of bits "
                  "0..4, 6 and 7");
    return -1;
  }
  return (int)st::g_defer_flip[dtype][size_class].exchange(mask,
                                                           std::memory_order_relaxed);
}

int
st_defer_ntload_class(unsigned int nrows, unsigned int ncols, int dtype)
{
  st::clear_error();
  if (dtype != 0 && dtype != 1) {
    st::set_error("st_defer_ntload_class: dtype 0/1");
    return -1;
  }
  return (int)st::defer_ntload_class(
    st::block_bytes(nrows, ncols, dtype == 1 ? 8 : 4));
}

int
st_set_every_cache(unsigned int size_class, unsigned int policy)
{
  st::clear_error();
  if (size_class >= (unsigned)st::kEveryCacheClasses || policy > 3u) {
    st::set_error("st_set_every_cache: size class 0..3, policy 0..3");
    return -1;
  }
  return (int)st::g_every_cache[size_class].exchange(policy,
                                                     std::memory_order_relaxed);
}

int
st_set_every_caps(unsigned int size_class, unsigned int wg_per_cu)
{
  st::clear_error();
  if (size_class >= (unsigned)st::kEveryCacheClasses || wg_per_cu == 1u ||
      wg_per_cu > 32u) {
    st::set_error("st_set_every_caps: size class 0..3, 0 (uncapped) or 2..32 "
                  "workgroups per CU");
    return -1;
  }
  return (int)st::g_every_caps[size_class].exchange(wg_per_cu,
                                                    std::memory_order_relaxed);
}

int
st_set_every_tile(unsigned int size_class, unsigned int tile)
{
  st::clear_error();
  if (size_class >= (unsigned)st::kEveryTileClasses || tile > 4096u) {
    st::set_error("st_set_every_tile: size class 0..3, tile 0..4096");
    return -1;
  }
  return (int)st::g_every_tile[size_class].exchange(tile, std::memory_order_relaxed);
}

int
st_set_mfree_shape(unsigned int shape)
{
  st::clear_error();
  if (shape > 3u) {
    st::set_error("st_set_mfree_shape: shape 0..3");
    return -1;
  }
  return (int)st::g_mfree_shape.exchange(shape, std::memory_order_relaxed);
}

int
st_every_cache_class(unsigned int nrows, unsigned int ncols, int dtype)
{
  st::clear_error();
  if (dtype != 0 && dtype != 1) {
    st::set_error("st_every_cache_class: dtype 0/1");
    return -1;
  }
  return (int)st::every_cache_class(
    st::block_bytes(nrows, ncols, dtype == 1 ? 8 : 4));
}

int
st_set_k0_reverse(int mode)
{
  return st::g_k0_rev.exchange(mode < 0 ? -1 : (mode ? 1 : 0), std::memory_order_relaxed);
}

unsigned int
st_set_flat_grid_limit(unsigned int max_x)
{
  const uint32_t gx = (max_x == 0 || max_x > st::kFlatGridX) ? st::kFlatGridX
                      : (max_x < 8u ? 8u : (max_x & ~7u));
  st::g_flat_grid_x.store(gx, std::memory_order_relaxed);
  return gx;
}

#endif // ST_TUNING_ABI

} // extern "C"
