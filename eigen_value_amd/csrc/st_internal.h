// Internal helpers shared by the HIP translation units of
// libsimilarity_transform.so (not part of the public C-ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "similarity_transform.h"

namespace st {

// thread-local last-error message (eigen_last_error)
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

#define ST_CHECK(expr)                                                         \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess) {                                                    \
      ::st::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,       \
                      hipGetErrorString(e_));                                  \
      return -1;                                                               \
    }                                                                          \
  } while (0)

#define ST_REQUIRE(cond, ...)                                                  \
  do {                                                                         \
    if (!(cond)) {                                                             \
      ::st::set_error(__VA_ARGS__);                                            \
      return -1;                                                               \
    }                                                                          \
  } while (0)

// "RCCL X.Y.Z (path of the library that holds the bound ncclAllGather)"
// (st_multi.hip; st_version, st_rccl_version)
std::string rccl_desc();

// Restores the caller's current HIP device when a C entry point returns
// (by any path): contexts, shards and communicators switch devices
// internally, and the caller's thread must not see that.
struct DeviceGuard
{
  int prev = -1;
  DeviceGuard()
  {
    if (hipGetDevice(&prev) != hipSuccess)
      prev = -1;
  }
  ~DeviceGuard()
  {
    if (prev >= 0)
      (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// kernel launchers (st_kernels.hip); all asynchronous on `stream`
template <typename T>
int launch_rowsum(const T* a, T* s, uint32_t nrows, uint32_t ncols,
                  hipStream_t stream);
// K0 in the flat form (k_flat_sum + k_parts) for blocks where the flat round
// pays; `part` holds round_flat_scratch(nrows, ncols) elements
template <typename T>
int launch_rowsum_flat(const T* a, T* s, T* part, uint32_t nrows,
                       uint32_t ncols, hipStream_t stream);
template <typename T>
int launch_scale_rowsum(T* a, const T* s_cur, T* s_next, uint32_t nrows,
                        uint32_t ncols, uint32_t row0, uint32_t semantics,
                        const st_state* st, hipStream_t stream);
template <typename T>
int launch_round(T* a, const T* s_cur, T* s_next, T* v, uint32_t nrows,
                 uint32_t ncols, uint32_t row0, T eps, uint32_t k,
                 uint32_t max_itr, uint32_t semantics, st_state* st,
                 hipStream_t stream);
// the flat round for large blocks (k_flat + k_parts); `part`
// holds round_flat_scratch(nrows, ncols) elements
template <typename T>
int launch_round_flat(T* a, const T* s_cur, T* s_next, T* part, T* v,
                      uint32_t nrows, uint32_t ncols, uint32_t row0, T eps,
                      uint32_t k, uint32_t max_itr, uint32_t semantics,
                      st_state* st, hipStream_t stream);
size_t round_flat_scratch(uint32_t nrows, uint32_t ncols);
bool round_flat_pays(uint32_t nrows, uint32_t ncols, size_t elem);
// the flat round with deferred writes (A stored every defer_rounds(...)
// rounds, bit-identical results; FlatPending in st_device.h): npend pending
// rounds' s and 1/s (oldest first), inv_cur = 1/s_cur, inv_next <- 1/s_{k+1};
// flush = store the matrix only (after the loop; no row sums, no v)
// rounds per store for a block: 6 (launch_flat_deferred's shapes,
// profiles/r02_flat_map_np5_*.log)
uint32_t defer_rounds(uint32_t nrows, uint32_t ncols, size_t elem);
constexpr uint32_t kDeferRoundsMax = 6;
template <typename T>
int launch_round_flat_deferred(T* a, const T* s_cur, const T* inv_cur,
                               T* s_next, T* inv_next, T* part, T* v,
                               uint32_t nrows, uint32_t ncols, uint32_t row0,
                               T eps, uint32_t k, uint32_t max_itr,
                               uint32_t semantics, st_state* st,
                               const T* const* pend_s,
                               const T* const* pend_inv, uint32_t npend,
                               bool store, bool flush, hipStream_t stream);
template <typename T>
int launch_recip(const T* s, T* inv, uint32_t n, hipStream_t stream);
template <typename T>
int launch_mfree(const T* a0, const T* s_prev, T* s_next, const T* v_prev,
                 T* v_cur, uint32_t nrows, uint32_t ncols, uint32_t row0,
                 T eps, uint32_t k, uint32_t max_itr, uint32_t semantics,
                 st_state* st, hipStream_t stream);
// the matrix-free round in the flat form (k_flat<MF> + k_mparts); `part`
// holds round_flat_scratch(nrows, ncols) elements
template <typename T>
int launch_mfree_flat(const T* a0, const T* s_prev, T* s_next, const T* v_prev,
                      T* v_cur, T* part, uint32_t nrows, uint32_t ncols,
                      uint32_t row0, T eps, uint32_t k, uint32_t max_itr,
                      uint32_t semantics, st_state* st, hipStream_t stream);
template <typename T>
int launch_epilogue(const T* s, T* v, uint32_t n, T eps, uint32_t max_itr,
                    uint32_t semantics, st_state* st, hipStream_t stream);
// st_state -> pinned host-coherent memory, in stream order (the solve loops'
// per-batch flag read)
int launch_state_mirror(const st_state* d_state, st_state* h_state,
                        hipStream_t stream);

template <typename T>
int launch_fill(T* x, uint64_t count, T value, hipStream_t stream);
// the whole solve in one workgroup (k_solve_small): v = 1, s_0, every round,
// the final state; for n <= 128 (fp64) / 256 (fp32), n % (16/sizeof(T)) == 0
template <typename T>
bool solve_small_fits(const T* a, uint32_t n);
template <typename T>
int launch_solve_small(T* a, T* v, uint32_t n, T eps, uint32_t max_itr,
                       uint32_t semantics, st_state* st, hipStream_t stream);

} // namespace st
