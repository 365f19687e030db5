// st_solve.hip — host orchestration of the similarity-transform round loop
// and the drop-in C-ABI (similarity_transform.h layers 1-3).
//
// Replaces, in the reference (itzmeanjan/eigen_value):
//   wrapper/similarity_transform.cpp:3-37   make_queue / max_eigen_value
//   similarity_transform.cpp:5-75           similarity_transform() host loop
//
// Round loop (one device stream, no per-round host sync):
//   K0  s_0 = rowsum(A_0)                                  N^2 b read, once
//       (k_flat_sum + k_parts where the flat round pays, else k_fused)
//   per round k, ONE launch (k_round, st_device.h; matrices of >= 144 MiB
//   take the flat round, k_flat + k_parts, instead, storing the matrix
//   every defer_rounds() rounds; N <= 128 fp64 / 256 fp32 run the whole
//   loop in one k_solve_small launch):
//     from s_k: max, v *= s/m, stop test, lambda = s_k[0] (every workgroup
//     derives m_k/stop_k from its own sweep of s_k; workgroup 0 records)
//     A_{k+1} = D_k^-1 A_k D_k in place, s_{k+1} = rowsum(A_{k+1})
//     (launches after the stop round return at once)
// The reference blocks on a host_accessor every round
// (similarity_transform.cpp:45-50).  Here rounds are enqueued in batches;
// the host checks the device `done` flag of batch b while batch b+1 is
// already queued, and rounds after convergence are device-gated no-ops, so
// the observable results (lambda, v, iter_count) are exactly those of the
// sequential loop.

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "st_internal.h"

namespace st {

static thread_local char g_err[512];

void
set_error(const char* fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void
clear_error()
{
  g_err[0] = '\0';
}

namespace {

constexpr uint32_t kDefaultBatch = 8;
constexpr uint32_t kFlatBatch = 2;

struct Context
{
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr; // own_stream or a caller stream
  // cached device workspaces (grown on demand, freed by destroy_queue)
  void* d_mat = nullptr;
  size_t mat_bytes = 0;
  // [s0 | s1 | v | v' | s ring (kDeferRoundsMax + 1) | 1/s ring (same)],
  // each vec_bytes
  void* d_vec = nullptr;
  size_t vec_bytes = 0;
  void* d_part = nullptr; // flat-round partial sums (large matrices)
  size_t part_bytes = 0;
  st_state* d_state = nullptr;
  st_state* h_state = nullptr; // pinned, 2 slots
  std::vector<float> round_ms; // per-round kernel time of the last timed solve
  // ST_FLAG_TRACE_SUMS: the row sums s_k every round of the last traced
  // solve evaluated (device staging, then the host copy st_last_round_sums
  // returns)
  void* d_trace = nullptr;
  size_t trace_cap = 0;
  std::vector<unsigned char> trace;
  uint32_t trace_rounds = 0;
  hipEvent_t ev_flag[2] = { nullptr, nullptr };
};

double
ms_since(std::chrono::steady_clock::time_point t0)
{
  return std::chrono::duration<double, std::milli>(
           std::chrono::steady_clock::now() - t0)
    .count();
}

int
ensure_device(Context* c)
{
  ST_CHECK(hipSetDevice(c->device));
  return 0;
}

int
ensure_vectors(Context* c, size_t vec_bytes)
{
  vec_bytes = (vec_bytes + 255) & ~(size_t)255;
  if (c->d_vec && c->vec_bytes >= vec_bytes)
    return 0;
  if (c->d_vec) {
    ST_CHECK(hipStreamSynchronize(c->stream));
    ST_CHECK(hipFree(c->d_vec));
    c->d_vec = nullptr;
  }
  ST_CHECK(hipMalloc(&c->d_vec, (4 + 2 * (kDeferRoundsMax + 1)) * vec_bytes));
  c->vec_bytes = vec_bytes;
  return 0;
}

int
ensure_part(Context* c, size_t bytes)
{
  if (c->d_part && c->part_bytes >= bytes)
    return 0;
  if (c->d_part) {
    ST_CHECK(hipStreamSynchronize(c->stream));
    ST_CHECK(hipFree(c->d_part));
    c->d_part = nullptr;
    c->part_bytes = 0;
  }
  ST_CHECK(hipMalloc(&c->d_part, bytes));
  c->part_bytes = bytes;
  return 0;
}

int
ensure_matrix(Context* c, size_t bytes)
{
  if (c->d_mat && c->mat_bytes >= bytes)
    return 0;
  if (c->d_mat) {
    ST_CHECK(hipStreamSynchronize(c->stream));
    ST_CHECK(hipFree(c->d_mat));
    c->d_mat = nullptr;
    c->mat_bytes = 0;
  }
  ST_CHECK(hipMalloc(&c->d_mat, bytes));
  c->mat_bytes = bytes;
  return 0;
}

// a traced solve records every evaluated round's n row sums: at most
// kTraceMaxBytes of them (tests and diagnostics, not a production mode)
constexpr size_t kTraceMaxBytes = (size_t)1 << 30;

int
ensure_trace(Context* c, size_t bytes)
{
  if (c->d_trace && c->trace_cap >= bytes)
    return 0;
  if (c->d_trace) {
    ST_CHECK(hipStreamSynchronize(c->stream));
    ST_CHECK(hipFree(c->d_trace));
    c->d_trace = nullptr;
    c->trace_cap = 0;
  }
  ST_CHECK(hipMalloc(&c->d_trace, bytes));
  c->trace_cap = bytes;
  return 0;
}

template <typename T>
T
default_eps();
template <>
float
default_eps<float>()
{
  return ST_EPS_F32; // include/similarity_transform.hpp:4 (float)
}
template <>
double
default_eps<double>()
{
  return ST_EPS_F64; // main.py:6
}

struct Resolved
{
  double eps;
  uint32_t max_itr, semantics, batch, flags;
};

template <typename T>
int
resolve(const st_options* opt, Resolved* r)
{
  r->eps = (opt && opt->eps >= 0.0) ? opt->eps : (double)default_eps<T>();
  r->max_itr = (opt && opt->max_itr) ? opt->max_itr : ST_MAX_ITR;
  r->semantics = opt ? opt->semantics : ST_SEM_SYCL;
  r->batch = (opt && opt->batch) ? opt->batch : 0; // 0: per round form
  r->flags = opt ? opt->flags : 0u;
  ST_REQUIRE(r->semantics <= ST_SEM_MAINPY, "unknown semantics %u",
             r->semantics);
  return 0;
}

// The round loop on a device-resident matrix (transformed in place).
// flush_matrix: leave the matrix as the every-round loop would (the caller
// sees it); a private copy (solve_host) skips the deferred loop's last store
template <typename T>
int64_t
solve_device(Context* c, T* d_mat, uint32_t n, T* d_v_out, T* v_host,
             T* eigen_val, uint32_t* iter_cnt, const st_options* opt,
             st_stats* stats, bool flush_matrix = true)
{
  ST_REQUIRE(c, "null queue");
  ST_REQUIRE(d_mat, "null matrix");
  ST_REQUIRE(n > 0, "dim must be > 0");
  ST_REQUIRE(eigen_val && iter_cnt, "null output pointer");
  ST_REQUIRE(d_v_out || v_host, "need a device or host eigenvector output");
  Resolved o;
  if (resolve<T>(opt, &o))
    return -1;
  if (ensure_device(c) || ensure_vectors(c, sizeof(T) * (size_t)n))
    return -1;
  hipStream_t s = c->stream;
  T* s_buf[2] = { reinterpret_cast<T*>(c->d_vec),
                  reinterpret_cast<T*>((char*)c->d_vec + c->vec_bytes) };
  T* d_v = d_v_out ? d_v_out
                   : reinterpret_cast<T*>((char*)c->d_vec + 2 * c->vec_bytes);
  // matrix-free ping-pong partner of d_v
  T* d_v2 = reinterpret_cast<T*>((char*)c->d_vec + 3 * c->vec_bytes);
  T* vb[2] = { d_v, d_v2 };
  const bool timed = (o.flags & ST_FLAG_TIME_KERNELS) != 0;
  const bool traced = (o.flags & ST_FLAG_TRACE_SUMS) != 0;
  const size_t row_bytes = sizeof(T) * (size_t)n;
  c->trace.clear();
  c->trace_rounds = 0;
  if (traced) {
    ST_REQUIRE(row_bytes * o.max_itr <= kTraceMaxBytes,
               "ST_FLAG_TRACE_SUMS: %u rounds x %u row sums exceed the %zu MiB "
               "trace; lower max_itr", o.max_itr, n, kTraceMaxBytes >> 20);
    if (ensure_trace(c, row_bytes * o.max_itr))
      return -1;
  }
  const bool mfree = (o.flags & ST_FLAG_MATRIX_FREE) != 0;
  // large matrices: the flat round (k_flat + k_parts)
  const bool flat = !mfree && round_flat_pays(n, n, sizeof(T));
  // the flat round stores the matrix every kDefer rounds (bit-identical
  // results; ST_FLAG_WRITE_EVERY_ROUND stores every round)
  const bool defer = flat && (o.flags & ST_FLAG_WRITE_EVERY_ROUND) == 0;
  const uint32_t kDefer = defer_rounds(n, n, sizeof(T));
  const uint32_t kR = kDefer + 1; // ring slots: pending + s_k + s_{k+1}
  T* ring_s[kDeferRoundsMax + 1];
  T* ring_inv[kDeferRoundsMax + 1];
  for (uint32_t i = 0; i < kR; i++) {
    ring_s[i] = reinterpret_cast<T*>((char*)c->d_vec + (4 + i) * c->vec_bytes);
    ring_inv[i] = reinterpret_cast<T*>((char*)c->d_vec +
                                       (4 + kDeferRoundsMax + 1 + i) * c->vec_bytes);
  }
  // K0 takes the flat form wherever the flat round pays (the matrix-free
  // loop's too)
  const bool flat_k0 = round_flat_pays(n, n, sizeof(T));
  if (flat_k0 && ensure_part(c, sizeof(T) * round_flat_scratch(n, n)))
    return -1;
  T* d_part = reinterpret_cast<T*>(c->d_part);
  // rounds per host flag check: the launches queued behind the stopping
  // round still run as gated no-ops, and a gated flat round is two launches
  // of up to millions of workgroups (~10 us each), so the flat form checks
  // every 2 rounds (>= 0.16 ms of work each) and the one-launch form every 8
  if (o.batch == 0)
    o.batch = flat ? kFlatBatch : kDefaultBatch;
  // timing events [rowsum_a, rowsum_b, (round_a, round_b)*], destroyed on
  // every exit path
  struct Events
  {
    std::vector<hipEvent_t> e;
    ~Events()
    {
      for (hipEvent_t x : e)
        if (x)
          (void)hipEventDestroy(x);
    }
  } events;
  std::vector<hipEvent_t>& ev = events.e;
  auto mk = [&](hipEvent_t* e) -> int {
    ST_CHECK(hipEventCreate(e));
    return 0;
  };
  int rc = 0;

  // a matrix that fits one workgroup's registers runs the whole solve in a
  // single launch, bit-identical to the round loop below; per-round timing,
  // tracing and ST_FLAG_ROUND_LOOP keep the loop
  const bool single = !mfree && !timed && !traced && (o.flags & ST_FLAG_ROUND_LOOP) == 0 &&
                      solve_small_fits<T>(d_mat, n);
  const auto t0 = std::chrono::steady_clock::now();
  ST_CHECK(hipMemsetAsync(c->d_state, 0, sizeof(st_state), s));
  if (!single && launch_fill<T>(d_v, n, (T)1, s)) // initialise_eigen_vector, cpp:34
    return -1;
  if (timed) { // (never single: k_solve_small does v = 1 and s_0 itself)
    ev.resize(2, nullptr);
    if (mk(&ev[0]) || mk(&ev[1]))
      return -1;
    (void)hipEventRecord(ev[0], s);
  }
  T* const s0 = defer ? ring_s[0] : s_buf[0];
  if (!single && (flat_k0 ? launch_rowsum_flat<T>(d_mat, s0, d_part, n, n, s)
                          : launch_rowsum<T>(d_mat, s0, n, n, s))) // K0
    return -1;
  if (defer && launch_recip<T>(ring_s[0], ring_inv[0], n, s))
    return -1;
  if (timed)
    (void)hipEventRecord(ev[1], s);

  const T eps = (T)o.eps;
  uint32_t enqueued = 0, cur = 0, batch_no = 0;
  bool done = false;
  if (single) { // the whole loop in one launch (k_solve_small)
    if (launch_solve_small<T>(d_mat, d_v, n, eps, o.max_itr, o.semantics,
                              c->d_state, s))
      return -1;
    done = true;
  }
  while (!done && enqueued < o.max_itr) {
    const uint32_t b = (o.max_itr - enqueued) < o.batch ? (o.max_itr - enqueued)
                                                        : o.batch;
    for (uint32_t j = 0; j < b; j++) {
      const uint32_t k = enqueued + j;
      hipEvent_t ea = nullptr, eb = nullptr;
      if (traced) // s_k, the row sums round k evaluates (no-op copies past the stop)
        rc |= hipMemcpyAsync((char*)c->d_trace + (size_t)k * row_bytes,
                             defer ? ring_s[k % kR] : s_buf[cur], row_bytes,
                             hipMemcpyDeviceToDevice, s) != hipSuccess;
      if (timed) {
        rc |= mk(&ea) | mk(&eb);
        ev.push_back(ea);
        ev.push_back(eb);
        (void)hipEventRecord(ea, s);
      }
      if (mfree) // launch k+1 evaluates round k
        rc |= launch_mfree<T>(d_mat, s_buf[cur], s_buf[cur ^ 1], vb[k & 1],
                              vb[(k + 1) & 1], n, n, 0, eps, k + 1, o.max_itr,
                              o.semantics, c->d_state, s);
      else if (defer) {
        // stored: A_j, j = the last multiple of kDefer <= k
        const uint32_t j0 = k - k % kDefer, np = k - j0;
        const T* ps[kDeferRoundsMax];
        const T* pi[kDeferRoundsMax];
        for (uint32_t i = 0; i < np; i++) {
          ps[i] = ring_s[(j0 + i) % kR];
          pi[i] = ring_inv[(j0 + i) % kR];
        }
        rc |= launch_round_flat_deferred<T>(
          d_mat, ring_s[k % kR], ring_inv[k % kR], ring_s[(k + 1) % kR],
          ring_inv[(k + 1) % kR], d_part, d_v, n, n, 0, eps, k, o.max_itr,
          o.semantics, c->d_state, ps, pi, np, np + 1 == kDefer, false, s);
      } else if (flat)
        rc |= launch_round_flat<T>(d_mat, s_buf[cur], s_buf[cur ^ 1], d_part,
                                   d_v, n, n, 0, eps, k, o.max_itr,
                                   o.semantics, c->d_state, s);
      else
        rc |= launch_round<T>(d_mat, s_buf[cur], s_buf[cur ^ 1], d_v, n, n, 0,
                              eps, k, o.max_itr, o.semantics, c->d_state, s);
      if (timed)
        (void)hipEventRecord(eb, s);
      cur ^= 1;
      if (rc)
        return -1;
    }
    enqueued += b;
    const int slot = batch_no & 1;
    if (launch_state_mirror(c->d_state, &c->h_state[slot], s))
      return -1;
    ST_CHECK(hipEventRecord(c->ev_flag[slot], s));
    // wait for the previous batch's flag while this batch runs
    if (batch_no > 0) {
      ST_CHECK(hipEventSynchronize(c->ev_flag[slot ^ 1]));
      done = c->h_state[slot ^ 1].done != 0;
    }
    batch_no++;
  }
  ST_CHECK(hipStreamSynchronize(s));
  st_state fin;
  ST_CHECK(hipMemcpy(&fin, c->d_state, sizeof(st_state), hipMemcpyDeviceToHost));
  ST_REQUIRE(fin.done, "internal: loop ended without done flag");
  if (defer && flush_matrix && fin.end % kDefer != 0) {
    // the matrix stands at A_J (J = the last store); apply rounds J .. end-1
    // and store A_end, exactly what storing every round leaves
    const uint32_t kl = fin.end - 1, j0 = kl - kl % kDefer, np = kl - j0;
    const T* ps[kDeferRoundsMax];
    const T* pi[kDeferRoundsMax];
    for (uint32_t i = 0; i < np; i++) {
      ps[i] = ring_s[(j0 + i) % kR];
      pi[i] = ring_inv[(j0 + i) % kR];
    }
    if (launch_round_flat_deferred<T>(
          d_mat, ring_s[kl % kR], ring_inv[kl % kR], nullptr, nullptr, d_part,
          d_v, n, n, 0, eps, kl, o.max_itr, o.semantics, c->d_state, ps, pi,
          np, true, true, s))
      return -1;
    ST_CHECK(hipStreamSynchronize(s));
  }
  if (mfree && (fin.end & 1u)) { // the final v_{end-1} landed in the partner
    ST_CHECK(hipMemcpyAsync(d_v, d_v2, sizeof(T) * (size_t)n,
                            hipMemcpyDeviceToDevice, s));
    ST_CHECK(hipStreamSynchronize(s));
  }
  const double loop_ms = ms_since(t0);

  const auto t1 = std::chrono::steady_clock::now();
  *eigen_val = (T)fin.lambda;
  *iter_cnt = fin.iters;
  if (v_host)
    ST_CHECK(hipMemcpy(v_host, d_v, sizeof(T) * (size_t)n,
                       hipMemcpyDeviceToHost));
  const double d2h_ms = ms_since(t1);
  if (traced) { // rounds 0 .. end-1 were evaluated
    c->trace.resize(row_bytes * fin.end);
    ST_CHECK(hipMemcpy(c->trace.data(), c->d_trace, c->trace.size(),
                       hipMemcpyDeviceToHost));
    c->trace_rounds = fin.end;
  }

  // per-round kernel times (rounds 0 .. end-1 did work; the stop round's
  // launch also streams the matrix), kept for st_last_round_times
  c->round_ms.clear();
  float rowsum_ms = 0.f;
  double tot = 0.0;
  if (timed) {
    (void)hipEventElapsedTime(&rowsum_ms, ev[0], ev[1]);
    for (uint32_t k = 0; k < fin.end && 2 + 2 * k + 1 < ev.size(); k++) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, ev[2 + 2 * k], ev[2 + 2 * k + 1]);
      c->round_ms.push_back(ms);
      tot += ms;
    }
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->loop_ms = loop_ms;
    stats->d2h_ms = d2h_ms;
    stats->rounds = fin.end;
    stats->converged = fin.stop;
    if (timed) {
      stats->rowsum_ms = rowsum_ms;
      stats->fused_ms_total = tot;
      stats->fused_launches = (uint32_t)c->round_ms.size();
    }
  }
  return (int64_t)loop_ms;
}

template <typename T>
int64_t
solve_host(Context* c, const T* mat, uint32_t n, T* eigen_val, T* eigen_vec,
           uint32_t* iter_cnt, const st_options* opt, st_stats* stats)
{
  ST_REQUIRE(c, "null queue");
  ST_REQUIRE(mat && eigen_val && eigen_vec && iter_cnt, "null pointer");
  ST_REQUIRE(n > 0, "dim must be > 0");
  if (ensure_device(c))
    return -1;
  const size_t bytes = sizeof(T) * (size_t)n * n;
  if (ensure_matrix(c, bytes))
    return -1;
  // the reference's timed region starts before the first kernel, which
  // performs the lazy host->device copy (similarity_transform.cpp:36-40)
  const auto t0 = std::chrono::steady_clock::now();
  ST_CHECK(hipMemcpyAsync(c->d_mat, mat, bytes, hipMemcpyHostToDevice,
                          c->stream));
  ST_CHECK(hipStreamSynchronize(c->stream));
  const double h2d = ms_since(t0);
  st_stats local{};
  if (solve_device<T>(c, reinterpret_cast<T*>(c->d_mat), n, nullptr,
                      eigen_vec, eigen_val, iter_cnt, opt, &local,
                      false) < 0)
    return -1;
  local.h2d_ms = h2d;
  if (stats)
    *stats = local;
  return (int64_t)(h2d + local.loop_ms);
}

Context*
as_ctx(void* wq)
{
  return reinterpret_cast<Context*>(wq);
}

} // namespace
} // namespace st

using st::Context;

extern "C" {

const char*
eigen_last_error(void)
{
  return st::g_err;
}

const char*
st_version(void)
{
  // the A/B probe switches the kernels were built with (st_kernels.hip):
  // "defaults" in every library build, the values in a probe build
  static const std::string v =
    std::string("eigen_value_amd 0.5.0 (gfx950; probe switches: ") +
    st_probe_switches() + "; " + st::rccl_desc() + ")";
  return v.c_str();
}

int
st_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess)
    return 0;
  return n;
}

void
make_queue(void** wq)
{
  st::clear_error();
  st::DeviceGuard guard;
  if (!wq)
    return;
  *wq = nullptr;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    st::set_error("make_queue: no HIP device");
    return;
  }
  if (const char* e = std::getenv("EIGEN_VALUE_DEVICE"))
    dev = std::atoi(e);
  Context* c = new (std::nothrow) Context();
  if (!c) {
    st::set_error("make_queue: out of host memory");
    return;
  }
  c->device = dev;
  bool ok = hipSetDevice(dev) == hipSuccess &&
            hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) ==
              hipSuccess &&
            hipMalloc(&c->d_state, sizeof(st_state)) == hipSuccess &&
            hipHostMalloc(&c->h_state, 2 * sizeof(st_state),
                          hipHostMallocCoherent | hipHostMallocMapped) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_flag[0], hipEventDisableTiming) ==
              hipSuccess &&
            hipEventCreateWithFlags(&c->ev_flag[1], hipEventDisableTiming) ==
              hipSuccess;
  if (!ok) {
    st::set_error("make_queue: HIP initialisation failed: %s",
                  hipGetErrorString(hipGetLastError()));
    destroy_queue(c);
    return;
  }
  c->stream = c->own_stream;
  *wq = c;
}

void
destroy_queue(void* wq)
{
  st::DeviceGuard guard;
  Context* c = st::as_ctx(wq);
  if (!c)
    return;
  (void)hipSetDevice(c->device);
  if (c->stream)
    (void)hipStreamSynchronize(c->stream);
  if (c->d_mat)
    (void)hipFree(c->d_mat);
  if (c->d_vec)
    (void)hipFree(c->d_vec);
  if (c->d_part)
    (void)hipFree(c->d_part);
  if (c->d_trace)
    (void)hipFree(c->d_trace);
  if (c->d_state)
    (void)hipFree(c->d_state);
  if (c->h_state)
    (void)hipHostFree(c->h_state);
  for (hipEvent_t e : c->ev_flag)
    if (e)
      (void)hipEventDestroy(e);
  if (c->own_stream)
    (void)hipStreamDestroy(c->own_stream);
  delete c;
}

int
st_last_round_times(void* wq, float* ms, unsigned int cap)
{
  st::clear_error();
  Context* c = st::as_ctx(wq);
  ST_REQUIRE(c, "st_last_round_times: null queue");
  ST_REQUIRE(ms || cap == 0, "st_last_round_times: null buffer");
  const size_t n = c->round_ms.size();
  for (size_t i = 0; i < n && i < cap; i++)
    ms[i] = c->round_ms[i];
  return (int)n;
}

int
st_last_round_sums(void* wq, void* sums, unsigned int cap_rounds)
{
  st::clear_error();
  Context* c = st::as_ctx(wq);
  ST_REQUIRE(c, "st_last_round_sums: null queue");
  ST_REQUIRE(sums || cap_rounds == 0, "st_last_round_sums: null buffer");
  const uint32_t r = c->trace_rounds;
  if (r && cap_rounds) {
    const size_t row = c->trace.size() / r;
    std::memcpy(sums, c->trace.data(), row * (cap_rounds < r ? cap_rounds : r));
  }
  return (int)r;
}

int
st_set_stream(void* wq, void* stream)
{
  st::clear_error();
  Context* c = st::as_ctx(wq);
  ST_REQUIRE(c, "st_set_stream: null queue");
  // NULL is HIP's null stream (torch's default stream handle is 0), not
  // "no stream": the context must order itself after the caller's work
  c->stream = reinterpret_cast<hipStream_t>(stream);
  return 0;
}

int
st_use_own_stream(void* wq)
{
  st::clear_error();
  Context* c = st::as_ctx(wq);
  ST_REQUIRE(c, "st_use_own_stream: null queue");
  c->stream = c->own_stream;
  return 0;
}

int64_t
max_eigen_value(void* wq, float* mat, float* eigen_val, float* eigen_vec,
                unsigned int dim, unsigned int* iter_cnt)
{
  st::clear_error();
  st::DeviceGuard guard;
  return st::solve_host<float>(st::as_ctx(wq), mat, dim, eigen_val, eigen_vec,
                               iter_cnt, nullptr, nullptr);
}

int64_t
max_eigen_value_f64(void* wq, double* mat, double* eigen_val,
                    double* eigen_vec, unsigned int dim,
                    unsigned int* iter_cnt)
{
  st::clear_error();
  st::DeviceGuard guard;
  return st::solve_host<double>(st::as_ctx(wq), mat, dim, eigen_val,
                                eigen_vec, iter_cnt, nullptr, nullptr);
}

int64_t
max_eigen_value_ex(void* wq, int dtype, const void* mat, void* eigen_val,
                   void* eigen_vec, unsigned int dim, unsigned int* iter_cnt,
                   const st_options* opt, st_stats* stats)
{
  st::clear_error();
  st::DeviceGuard guard;
  if (dtype == 0)
    return st::solve_host<float>(st::as_ctx(wq), (const float*)mat, dim,
                                 (float*)eigen_val, (float*)eigen_vec,
                                 iter_cnt, opt, stats);
  if (dtype == 1)
    return st::solve_host<double>(st::as_ctx(wq), (const double*)mat, dim,
                                  (double*)eigen_val, (double*)eigen_vec,
                                  iter_cnt, opt, stats);
  st::set_error("max_eigen_value_ex: dtype must be 0 (f32) or 1 (f64)");
  return -1;
}

int64_t
st_solve_device_f32(void* wq, float* d_mat, unsigned int dim,
                    float* d_eigen_vec, float* eigen_vec_host,
                    float* eigen_val, unsigned int* iter_cnt,
                    const st_options* opt, st_stats* stats)
{
  st::clear_error();
  st::DeviceGuard guard;
  return st::solve_device<float>(st::as_ctx(wq), d_mat, dim, d_eigen_vec,
                                 eigen_vec_host, eigen_val, iter_cnt, opt,
                                 stats);
}

int64_t
st_solve_device_f64(void* wq, double* d_mat, unsigned int dim,
                    double* d_eigen_vec, double* eigen_vec_host,
                    double* eigen_val, unsigned int* iter_cnt,
                    const st_options* opt, st_stats* stats)
{
  st::clear_error();
  st::DeviceGuard guard;
  return st::solve_device<double>(st::as_ctx(wq), d_mat, dim, d_eigen_vec,
                                  eigen_vec_host, eigen_val, iter_cnt, opt,
                                  stats);
}

} // extern "C"
