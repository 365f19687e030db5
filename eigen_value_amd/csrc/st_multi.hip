// st_multi.hip — native multi-GPU solve: one process, P devices, row-block
// sharding with ONE RCCL all-gather of the N-length row-sum vector per round
// (SURVEY.md §8e), driven from one host thread with ncclGroupStart/End.
//
// Device d owns rows [d*chunk, d*chunk + rows_d), chunk = ceil(N/P), and
// keeps: its row block of A (transformed in place, or read only in the
// matrix-free form), a ring of padded P*chunk row-sum vectors (two slots,
// or defer_rounds() + 1 when its block takes the flat round with deferred
// writes, with their reciprocals), the eigenvector accumulator(s) and an
// st_state.  Round k on every device:
//   k_round / the flat round (deferred writes: A stored every
//   defer_rounds() rounds, st_solve.hip) / k_mfree (launch k+1) on its stream
//   ncclAllGather(slot_d, s_next, chunk, type, comm_d, stream_d)
// Every device derives m_k / stop_k from the identical gathered vector, so
// the states agree without a further collective; the host polls device 0's
// flag per batch, as in the single-GPU loop (st_solve.hip).  At the end the
// eigenvector rows come back from each device's own slice (transform form)
// or from device 0's full copy (matrix-free form).
//
// This is the C-ABI counterpart of eigen_value_amd/sharded.py (one process
// per GPU over torch.distributed); both run the same kernels.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "st_internal.h"
#include "st_rendezvous.h"

namespace st {
namespace {

#define ST_NCCL(expr)                                                          \
  do {                                                                         \
    ncclResult_t r_ = (expr);                                                  \
    if (r_ != ncclSuccess) {                                                   \
      ::st::set_error("%s:%d: %s failed: %s", __FILE__, __LINE__, #expr,       \
                      ncclGetErrorString(r_));                                 \
      return -1;                                                               \
    }                                                                          \
  } while (0)

// ---------------------------------------------------------------------------
// deadline on every RCCL step that waits for peers (comm_timeout_s).
// Communicators are non-blocking (ncclConfig_t.blocking = 0): a collective
// whose connection setup is still running returns ncclInProgress and this
// thread polls ncclCommGetAsyncError until it is enqueued or the deadline
// passes (comm_wait / comm_settle); past it the communicators are aborted
// (a completed init, so abort is safe) and the call returns -1 naming the
// stalled rank and device.  Creation runs on a helper thread under the same
// deadline (init_with_deadline), and st_comm_init first checks that every
// rank is present (st_rendezvous.hip), so a missing peer is reported before
// any rank enters ncclCommInitRankConfig.
// ---------------------------------------------------------------------------
std::atomic<double> g_comm_timeout_s{ -1.0 }; // < 0: ST_COMM_TIMEOUT_S or 120 s

double
comm_timeout_s()
{
  const double set = g_comm_timeout_s.load(std::memory_order_relaxed);
  if (set >= 0.0)
    return set;
  const char* e = std::getenv("ST_COMM_TIMEOUT_S");
  const double v = e ? std::atof(e) : 0.0;
  return v > 0.0 ? v : 120.0;
}

ncclConfig_t
comm_config()
{
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  return cfg;
}

// Wait until none of comms[0..n) is in progress.  ranks / devs name them
// in the message.  Returns 0, or -1 (error set) on an asynchronous error or
// when the deadline passes; on -1 the caller aborts the communicators.
int
comm_wait(const ncclComm_t* comms, int n, const int* ranks, const int* devs,
          const char* what)
{
  const double limit = comm_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spins = 0;; spins++) {
    int pending = -1;
    for (int i = 0; i < n; i++) {
      ncclResult_t st = ncclSuccess;
      const ncclResult_t r = ncclCommGetAsyncError(comms[i], &st);
      if (r != ncclSuccess)
        st = r;
      if (st == ncclInProgress) {
        if (pending < 0)
          pending = i;
      } else if (st != ncclSuccess) {
        ::st::set_error("%s: RCCL rank %d (device %d) failed: %s", what,
                        ranks[i], devs[i], ncclGetErrorString(st));
        return -1;
      }
    }
    if (pending < 0)
      return 0;
    const double el = std::chrono::duration<double>(
                        std::chrono::steady_clock::now() - t0)
                        .count();
    if (el > limit) {
      ::st::set_error("%s: RCCL rank %d (device %d) still in progress after "
                      "%.1f s (deadline %.1f s, ST_COMM_TIMEOUT_S / "
                      "st_set_comm_timeout): a peer did not arrive; "
                      "communicator aborted",
                      what, ranks[pending], devs[pending], el, limit);
      return -1;
    }
    if (spins > 64)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    else
      std::this_thread::yield();
  }
}

// Communicator creation under the deadline.  The init runs on a helper
// thread, which also completes the non-blocking group job (its state is
// thread-local to the thread that ended the group: the helper must not exit
// before the communicators are ready), and this thread waits for it at most
// the deadline.  The helper is the communicators' ONLY owner until it
// reports done: it polls them (ncclCommGetAsyncError), stops at the first
// error, and aborts them itself on an error or when this thread gave up
// (job->cancel); this thread never aborts a communicator whose init has not
// returned (ncclCommAbort racing the init or the helper's poll was the
// use-after-free of round 4, VERDICT r04 #3 / ADVICE r04).  A missing peer
// is found before RCCL is entered (st_comm_init's rendezvous,
// st_rendezvous.hip), so past the deadline here a peer died between the
// rendezvous and the init: the helper is then left inside RCCL and the
// error says to end the process with _exit.
struct InitJob
{
  std::vector<ncclComm_t> comms; // written by RCCL in body(); read after done
  ncclResult_t r = ncclInProgress;
  int failed = -1;            // index of the communicator that reported r
  std::atomic<int> done{ 0 }; // the helper has finished (and aborted on error)
  std::atomic<int> cancel{ 0 }; // the caller gave up: abort and leave
};

int
init_with_deadline(const std::shared_ptr<InitJob>& job,
                   std::function<ncclResult_t(InitJob&)> body, const int* ranks,
                   const int* devs, const char* what)
{
  std::thread([job, body]() {
    ncclResult_t r = body(*job);
    // finish an asynchronous init here, in the thread that started it; stop
    // at the first communicator that reports an error
    while (r == ncclInProgress && !job->cancel.load(std::memory_order_acquire)) {
      bool pending = false;
      for (size_t i = 0; i < job->comms.size() && r == ncclInProgress; i++) {
        ncclComm_t c = job->comms[i];
        if (!c)
          continue;
        ncclResult_t st = ncclSuccess;
        if (ncclCommGetAsyncError(c, &st) != ncclSuccess)
          st = ncclInternalError;
        if (st == ncclInProgress)
          pending = true;
        else if (st != ncclSuccess) {
          r = st;
          job->failed = (int)i;
        }
      }
      if (r == ncclInProgress && !pending)
        r = ncclSuccess;
      if (r == ncclInProgress)
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    const bool gave_up = job->cancel.load(std::memory_order_acquire);
    if (r != ncclSuccess || gave_up) {
      for (ncclComm_t c : job->comms)
        if (c)
          (void)ncclCommAbort(c);
      if (r == ncclSuccess || r == ncclInProgress)
        r = ncclInvalidUsage; // completed or not, the caller has gone
    }
    job->r = r;
    job->done.store(1, std::memory_order_release);
  }).detach();
  const double limit = comm_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&t0]() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
      .count();
  };
  const size_t ncomm = job->comms.size();
  auto who = [&](int i) {
    if (i >= 0 || ncomm == 1)
      return "RCCL rank " + std::to_string(ranks[i < 0 ? 0 : i]) + " (device " +
             std::to_string(devs[i < 0 ? 0 : i]) + ")";
    std::string w = "RCCL ranks 0.." + std::to_string(ncomm - 1) + " (devices";
    for (size_t k = 0; k < ncomm; k++)
      w += " " + std::to_string(devs[k]);
    return w + ")";
  };
  while (!job->done.load(std::memory_order_acquire)) {
    const double el = elapsed();
    if (el > limit) {
      // hand the communicators to the helper's abort; give it a moment to
      // say whether its init has returned
      job->cancel.store(1, std::memory_order_release);
      const double t_c = elapsed();
      while (!job->done.load(std::memory_order_acquire) && elapsed() < t_c + 2.0)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      const bool stuck = !job->done.load(std::memory_order_acquire);
      // the helper may have finished with a live communicator just before
      // it could see the cancel (it read gave_up == false first): that init
      // succeeded, late, and the communicator is the caller's
      if (!stuck && job->r == ncclSuccess)
        return 0;
      ::st::set_error(
        "%s: %s still in progress after %.1f s (deadline %.1f s, "
        "ST_COMM_TIMEOUT_S / st_set_comm_timeout): a peer stopped after the "
        "rendezvous; %s",
        what, who(-1).c_str(), el, limit,
        stuck ? "the RCCL init thread has not returned and owns the "
                "communicator(s) (it aborts them if it ever returns): end the "
                "process with _exit"
              : "communicator(s) aborted by the init thread");
      return -1;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  }
  if (job->r != ncclSuccess) { // the helper has aborted the communicators
    ::st::set_error("%s: ncclCommInitRankConfig (%s) failed: %s", what,
                    who(job->failed).c_str(), ncclGetErrorString(job->r));
    return -1;
  }
  return 0;
}

// the result of a call on non-blocking communicators: ncclInProgress is
// waited for, anything else but ncclSuccess is an error
int
comm_settle(ncclResult_t r, const ncclComm_t* comms, int n, const int* ranks,
            const int* devs, const char* what)
{
  if (r == ncclSuccess)
    return 0;
  if (r != ncclInProgress) {
    ::st::set_error("%s failed: %s", what, ncclGetErrorString(r));
    return -1;
  }
  return comm_wait(comms, n, ranks, devs, what);
}

template <typename T>
ncclDataType_t
nccl_type();
template <>
ncclDataType_t
nccl_type<float>()
{
  return ncclFloat;
}
template <>
ncclDataType_t
nccl_type<double>()
{
  return ncclDouble;
}

template <typename T>
struct Shard
{
  int dev = 0;
  uint32_t row0 = 0, nrows = 0;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  T* a = nullptr;
  T* s[kDeferRoundsMax + 1] = {};   // row sums, ring slot k % nring
  T* inv[kDeferRoundsMax + 1] = {}; // 1 / s (deferred writes only)
  T* v[2] = { nullptr, nullptr };
  T* part = nullptr; // flat-round partial sums (large blocks)
  bool defer = false; // the flat round with deferred writes
  st_state* state = nullptr;
};

template <typename T>
struct Multi
{
  std::vector<Shard<T>> sh;
  std::vector<ncclComm_t> comms; // sh[p].comm, for comm_wait
  std::vector<int> ranks, devs;
  bool abort = false; // a deadline passed: abort, do not destroy
  st_state* h_state = nullptr; // pinned, 2 slots
  hipEvent_t ev[2] = { nullptr, nullptr };
  ~Multi()
  {
    // after a failed or timed-out collective, abort every communicator
    // FIRST: that stops the RCCL kernels already queued on the streams,
    // which could otherwise wait forever for a peer and hang the sync below
    if (abort)
      for (auto& d : sh)
        if (d.comm) {
          (void)ncclCommAbort(d.comm);
          d.comm = nullptr;
        }
    for (auto& d : sh) {
      (void)hipSetDevice(d.dev);
      if (d.stream)
        (void)hipStreamSynchronize(d.stream);
      if (d.comm)
        (void)ncclCommDestroy(d.comm);
      (void)hipFree(d.a);
      for (uint32_t i = 0; i <= kDeferRoundsMax; i++) {
        (void)hipFree(d.s[i]);
        (void)hipFree(d.inv[i]);
      }
      for (int i = 0; i < 2; i++)
        (void)hipFree(d.v[i]);
      (void)hipFree(d.part);
      (void)hipFree(d.state);
      if (d.stream)
        (void)hipStreamDestroy(d.stream);
    }
    if (!sh.empty())
      (void)hipSetDevice(sh[0].dev);
    for (hipEvent_t e : ev)
      if (e)
        (void)hipEventDestroy(e);
    if (h_state)
      (void)hipHostFree(h_state);
  }
};

template <typename T>
int
gather(Multi<T>& M, int which, uint32_t chunk)
{
  // P = 1 still issues the (in-place, no-op) collective, so the RCCL path
  // is exercised on a one-GPU machine too.  On the non-blocking
  // communicators the first group (connection setup) may return
  // ncclInProgress: wait for it, under the deadline, before the next launch
  // a failed enqueue still closes the group (its depth is per thread) and
  // marks the communicators for abort
  const ncclResult_t gs = ncclGroupStart();
  if (gs != ncclSuccess) {
    M.abort = true;
    ::st::set_error("st_solve_multi all-gather: ncclGroupStart failed: %s",
                    ncclGetErrorString(gs));
    return -1;
  }
  for (size_t p = 0; p < M.sh.size(); p++) {
    Shard<T>& d = M.sh[p];
    T* buf = d.s[which];
    const ncclResult_t r = ncclAllGather(buf + p * chunk, buf, chunk,
                                         nccl_type<T>(), d.comm, d.stream);
    if (r != ncclSuccess && r != ncclInProgress) {
      (void)ncclGroupEnd();
      M.abort = true;
      ::st::set_error("st_solve_multi all-gather: ncclAllGather on RCCL rank "
                      "%zu (device %d) failed: %s",
                      p, d.dev, ncclGetErrorString(r));
      return -1;
    }
  }
  if (comm_settle(ncclGroupEnd(), M.comms.data(), (int)M.comms.size(),
                  M.ranks.data(), M.devs.data(), "st_solve_multi all-gather")) {
    M.abort = true;
    return -1;
  }
  return 0;
}

template <typename T>
int64_t
solve_multi(const T* mat, uint32_t n, int ngpus, const int* devices,
            int gen_kind, uint64_t seed, T* eigen_val, T* eigen_vec,
            uint32_t* iter_cnt, const st_options* opt, st_stats* stats)
{
  ST_REQUIRE(n > 0, "dim must be > 0");
  ST_REQUIRE(ngpus >= 1, "ngpus must be >= 1");
  ST_REQUIRE(eigen_val && eigen_vec && iter_cnt, "null output pointer");
  ST_REQUIRE(gen_kind >= 0 && gen_kind <= 2, "gen_kind must be 0, 1 or 2");
  ST_REQUIRE(gen_kind != 0 || mat, "null matrix");
  int have = 0;
  ST_CHECK(hipGetDeviceCount(&have));
  const uint32_t P = (uint32_t)ngpus;
  const uint32_t chunk = (n + P - 1) / P;
  ST_REQUIRE((uint64_t)(P - 1) * chunk < n,
             "dim %u leaves a device of %u without rows", n, P);
  const double eps_d = (opt && opt->eps >= 0.0)
                         ? opt->eps
                         : (sizeof(T) == 4 ? (double)ST_EPS_F32 : ST_EPS_F64);
  const T eps = (T)eps_d;
  const uint32_t max_itr = (opt && opt->max_itr) ? opt->max_itr : ST_MAX_ITR;
  const uint32_t sem = opt ? opt->semantics : ST_SEM_SYCL;
  uint32_t batch = (opt && opt->batch) ? opt->batch : 0u;
  const bool mfree = opt && (opt->flags & ST_FLAG_MATRIX_FREE);
  const bool every = opt && (opt->flags & ST_FLAG_WRITE_EVERY_ROUND);
  ST_REQUIRE(sem <= ST_SEM_MAINPY, "unknown semantics %u", sem);
  // ring slots of the row-sum vectors: every shard gathers into the same
  // slot, so the ring is as long as the longest any shard needs
  uint32_t nring = 2;
  for (uint32_t p = 0; p < P; p++) {
    const uint32_t r0 = p * ((n + P - 1) / P), ch = (n + P - 1) / P;
    const uint32_t nr = r0 + ch <= n ? ch : n - r0;
    if (!mfree && !every && round_flat_pays(nr, n, sizeof(T)) &&
        defer_rounds(nr, n, sizeof(T)) + 1 > nring)
      nring = defer_rounds(nr, n, sizeof(T)) + 1;
  }

  Multi<T> M;
  M.sh.resize(P);
  std::vector<int> devlist(P);
  for (uint32_t p = 0; p < P; p++) {
    devlist[p] = devices ? devices[p] : (int)p;
    ST_REQUIRE(devlist[p] >= 0 && devlist[p] < have,
               "device %d out of range (%d devices)", devlist[p], have);
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t p = 0; p < P; p++) {
    Shard<T>& d = M.sh[p];
    d.dev = devlist[p];
    d.row0 = p * chunk;
    d.nrows = (d.row0 + chunk <= n) ? chunk : n - d.row0;
    ST_CHECK(hipSetDevice(d.dev));
    ST_CHECK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    ST_CHECK(hipMalloc(&d.a, sizeof(T) * (size_t)d.nrows * n));
    for (uint32_t i = 0; i < nring; i++)
      ST_CHECK(hipMalloc(&d.s[i], sizeof(T) * (size_t)P * chunk));
    for (int i = 0; i < (mfree ? 2 : 1); i++)
      ST_CHECK(hipMalloc(&d.v[i], sizeof(T) * (size_t)P * chunk));
    ST_CHECK(hipMalloc(&d.state, sizeof(st_state)));
    // the flat-form scratch: the flat rounds' and K0's (the matrix-free
    // loop's K0 too)
    if (round_flat_pays(d.nrows, n, sizeof(T)))
      ST_CHECK(hipMalloc(&d.part, sizeof(T) * round_flat_scratch(d.nrows, n)));
    d.defer = d.part != nullptr && !every && !mfree;
    if (d.defer)
      for (uint32_t i = 0; i < nring; i++)
        ST_CHECK(hipMalloc(&d.inv[i], sizeof(T) * (size_t)P * chunk));
    ST_CHECK(hipMemsetAsync(d.state, 0, sizeof(st_state), d.stream));
    if (gen_kind == 0) {
      ST_CHECK(hipMemcpyAsync(d.a, mat + (size_t)d.row0 * n,
                              sizeof(T) * (size_t)d.nrows * n,
                              hipMemcpyHostToDevice, d.stream));
    } else {
      // the generators set the error message themselves on failure
      int rc;
      if (gen_kind == 1)
        rc = sizeof(T) == 8
               ? st_generate_hilbert_f64((double*)d.a, d.nrows, n, d.row0,
                                         d.stream)
               : st_generate_hilbert_f32((float*)d.a, d.nrows, n, d.row0,
                                         d.stream);
      else
        rc = sizeof(T) == 8
               ? st_generate_random_f64((double*)d.a, d.nrows, n, d.row0,
                                        seed, d.stream)
               : st_generate_random_f32((float*)d.a, d.nrows, n, d.row0,
                                        seed, d.stream);
      if (rc != 0)
        return -1;
    }
    if (launch_fill<T>(d.v[0], n, (T)1, d.stream)) // cpp:34
      return -1;
  }
  ST_CHECK(hipSetDevice(M.sh[0].dev));
  ST_CHECK(hipHostMalloc(&M.h_state, 2 * sizeof(st_state),
                         hipHostMallocCoherent | hipHostMallocMapped));
  ST_CHECK(hipEventCreateWithFlags(&M.ev[0], hipEventDisableTiming));
  ST_CHECK(hipEventCreateWithFlags(&M.ev[1], hipEventDisableTiming));
  if (batch == 0) // as st_solve.hip: flat rounds are checked every 2 rounds
    batch = (M.sh[0].part && !mfree) ? 2u : 8u;
  {
    // ncclCommInitAll, but under the deadline: one id, a group of
    // per-device non-blocking ncclCommInitRankConfig calls on a helper
    // thread (init_with_deadline), then poll
    ncclUniqueId id;
    ST_NCCL(ncclGetUniqueId(&id));
    M.ranks.resize(P);
    for (uint32_t p = 0; p < P; p++)
      M.ranks[p] = (int)p;
    M.devs = devlist;
    auto job = std::make_shared<InitJob>();
    job->comms.assign(P, nullptr);
    const std::vector<int> devs = devlist;
    const int rc = init_with_deadline(
      job,
      [id, devs](InitJob& j) {
        ncclConfig_t cfg = comm_config();
        ncclResult_t r = ncclGroupStart();
        for (size_t p = 0; p < devs.size() && (r == ncclSuccess); p++) {
          if (hipSetDevice(devs[p]) != hipSuccess)
            r = ncclUnhandledCudaError;
          else {
            const ncclResult_t q = ncclCommInitRankConfig(
              &j.comms[p], (int)devs.size(), id, (int)p, &cfg);
            if (q != ncclSuccess && q != ncclInProgress) {
              r = q;
              j.failed = (int)p;
            }
          }
        }
        const ncclResult_t ge = ncclGroupEnd();
        return r != ncclSuccess ? r : ge;
      },
      M.ranks.data(), M.devs.data(), "st_solve_multi communicator init");
    if (rc == 0) {
      M.comms = job->comms;
      for (uint32_t p = 0; p < P; p++)
        M.sh[p].comm = M.comms[p];
    } else {
      return -1; // the helper aborted the communicators (or still owns them)
    }
  }
  for (uint32_t p = 0; p < P; p++) { // s_0 = rowsum(A_0), then gather
    Shard<T>& d = M.sh[p];
    ST_CHECK(hipSetDevice(d.dev));
    if (d.part ? launch_rowsum_flat<T>(d.a, d.s[0] + p * chunk, d.part, d.nrows, n,
                                       d.stream)
               : launch_rowsum<T>(d.a, d.s[0] + p * chunk, d.nrows, n, d.stream))
      return -1;
  }
  if (gather(M, 0, chunk))
    return -1;
  for (uint32_t p = 0; p < P; p++) { // 1 / s_0 for the deferred loop
    Shard<T>& d = M.sh[p];
    if (d.defer) {
      ST_CHECK(hipSetDevice(d.dev));
      if (launch_recip<T>(d.s[0], d.inv[0], n, d.stream))
        return -1;
    }
  }
  for (uint32_t p = 0; p < P; p++) { // the setup is not part of the loop time
    ST_CHECK(hipSetDevice(M.sh[p].dev));
    ST_CHECK(hipStreamSynchronize(M.sh[p].stream));
  }
  const double setup_ms =
    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                              t0)
      .count();

  const auto t1 = std::chrono::steady_clock::now();
  uint32_t enqueued = 0, batch_no = 0;
  bool done = false;
  while (!done && enqueued < max_itr) {
    const uint32_t b = (max_itr - enqueued) < batch ? (max_itr - enqueued) : batch;
    for (uint32_t j = 0; j < b; j++) {
      const uint32_t k = enqueued + j;
      for (uint32_t p = 0; p < P; p++) {
        Shard<T>& d = M.sh[p];
        ST_CHECK(hipSetDevice(d.dev));
        int rc;
        const uint32_t cur = k % nring, nxt = (k + 1) % nring;
        if (mfree)
          rc = launch_mfree<T>(d.a, d.s[cur], d.s[nxt] + p * chunk,
                               d.v[k & 1], d.v[(k + 1) & 1], d.nrows, n,
                               d.row0, eps, k + 1, max_itr, sem, d.state,
                               d.stream);
        else if (d.defer) {
          // stored: A_j, j = the last multiple of kDefer <= k (the block is
          // private: no flush after the loop)
          const uint32_t kDefer = defer_rounds(d.nrows, n, sizeof(T));
          const uint32_t j0 = k - k % kDefer, np = k - j0;
          const T* ps[kDeferRoundsMax];
          const T* pi[kDeferRoundsMax];
          for (uint32_t i = 0; i < np; i++) {
            ps[i] = d.s[(j0 + i) % nring];
            pi[i] = d.inv[(j0 + i) % nring];
          }
          rc = launch_round_flat_deferred<T>(
            d.a, d.s[cur], d.inv[cur], d.s[nxt] + p * chunk,
            d.inv[nxt] + d.row0, d.part, d.v[0], d.nrows, n, d.row0, eps, k,
            max_itr, sem, d.state, ps, pi, np, np + 1 == kDefer, false,
            d.stream);
        } else if (d.part) // (never matrix-free: that branch comes first)
          rc = launch_round_flat<T>(d.a, d.s[cur], d.s[nxt] + p * chunk,
                                    d.part, d.v[0], d.nrows, n, d.row0, eps, k,
                                    max_itr, sem, d.state, d.stream);
        else
          rc = launch_round<T>(d.a, d.s[cur], d.s[nxt] + p * chunk, d.v[0],
                               d.nrows, n, d.row0, eps, k, max_itr, sem,
                               d.state, d.stream);
        if (rc)
          return -1;
      }
      if (gather(M, (k + 1) % nring, chunk))
        return -1;
    }
    enqueued += b;
    const int slot = batch_no & 1;
    Shard<T>& d0 = M.sh[0];
    ST_CHECK(hipSetDevice(d0.dev));
    if (launch_state_mirror(d0.state, &M.h_state[slot], d0.stream))
      return -1;
    ST_CHECK(hipEventRecord(M.ev[slot], d0.stream));
    if (batch_no > 0) {
      ST_CHECK(hipEventSynchronize(M.ev[slot ^ 1]));
      done = M.h_state[slot ^ 1].done != 0;
    }
    batch_no++;
  }
  for (uint32_t p = 0; p < P; p++) {
    ST_CHECK(hipSetDevice(M.sh[p].dev));
    ST_CHECK(hipStreamSynchronize(M.sh[p].stream));
  }
  const double loop_ms =
    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() -
                                              t1)
      .count();
  st_state fin;
  ST_CHECK(hipSetDevice(M.sh[0].dev));
  ST_CHECK(hipMemcpy(&fin, M.sh[0].state, sizeof(st_state), hipMemcpyDeviceToHost));
  ST_REQUIRE(fin.done, "internal: loop ended without done flag");
  *eigen_val = (T)fin.lambda;
  *iter_cnt = fin.iters;
  if (mfree) {
    ST_CHECK(hipMemcpy(eigen_vec, M.sh[0].v[fin.end & 1u], sizeof(T) * (size_t)n,
                       hipMemcpyDeviceToHost));
  } else {
    for (uint32_t p = 0; p < P; p++) {
      Shard<T>& d = M.sh[p];
      ST_CHECK(hipSetDevice(d.dev));
      ST_CHECK(hipMemcpy(eigen_vec + d.row0, d.v[0] + d.row0,
                         sizeof(T) * (size_t)d.nrows, hipMemcpyDeviceToHost));
    }
  }
  if (stats) {
    std::memset(stats, 0, sizeof(*stats));
    stats->h2d_ms = setup_ms;
    stats->loop_ms = loop_ms;
    stats->rounds = fin.end;
    stats->converged = fin.stop;
  }
  return (int64_t)(setup_ms + loop_ms);
}

} // namespace

// The RCCL this library's calls bind to: ncclGetVersion and the file that
// holds the ncclAllGather the library calls (dladdr).  Inside a torch
// process that is torch's bundled librccl (loaded first, same soname), for
// a C caller the /opt/rocm one the library was linked against
// (INTEGRATION.md §5).
int
rccl_version(int* code, std::string* path)
{
  int v = 0;
  if (ncclGetVersion(&v) != ncclSuccess)
    v = 0;
  if (code)
    *code = v;
  if (path) {
    Dl_info info;
    void* fn = reinterpret_cast<void*>(&ncclAllGather);
    *path = (dladdr(fn, &info) && info.dli_fname) ? info.dli_fname : "?";
  }
  return v > 0 ? 0 : -1;
}

std::string
rccl_desc()
{
  int v = 0;
  std::string path;
  rccl_version(&v, &path);
  // NCCL_VERSION(X, Y, Z) = X*10000 + Y*100 + Z since 2.9
  return "RCCL " + std::to_string(v / 10000) + "." + std::to_string(v / 100 % 100) +
         "." + std::to_string(v % 100) + " (" + path + ")";
}

} // namespace st

// ---------------------------------------------------------------------------
// one-process-per-GPU communicator (the sharded driver's RCCL path): rank 0
// makes the 128-byte unique id, the caller broadcasts it (torch.distributed
// over TCP), every rank joins; the all-gather is then issued directly on
// the launch stream, with no cross-stream hand-off per round.  The handle
// is a CommBox: the non-blocking communicator plus the rank and device its
// deadline messages name.
// ---------------------------------------------------------------------------
namespace st {
namespace {
struct CommBox
{
  ncclComm_t c = nullptr;
  int rank = 0, dev = 0;
};

int
comm_collective(CommBox* b, ncclResult_t r, const char* what)
{
  return comm_settle(r, &b->c, 1, &b->rank, &b->dev, what);
}
} // namespace
} // namespace st

extern "C" {

int64_t
st_solve_multi_f32(const float* mat, unsigned int dim, int ngpus,
                   const int* devices, int gen_kind, uint64_t seed,
                   float* eigen_val, float* eigen_vec, unsigned int* iter_cnt,
                   const st_options* opt, st_stats* stats)
{
  st::clear_error();
  st::DeviceGuard guard;
  return st::solve_multi<float>(mat, dim, ngpus, devices, gen_kind, seed,
                                eigen_val, eigen_vec, iter_cnt, opt, stats);
}

int64_t
st_solve_multi_f64(const double* mat, unsigned int dim, int ngpus,
                   const int* devices, int gen_kind, uint64_t seed,
                   double* eigen_val, double* eigen_vec,
                   unsigned int* iter_cnt, const st_options* opt,
                   st_stats* stats)
{
  st::clear_error();
  st::DeviceGuard guard;
  return st::solve_multi<double>(mat, dim, ngpus, devices, gen_kind, seed,
                                 eigen_val, eigen_vec, iter_cnt, opt, stats);
}


double
st_set_comm_timeout(double seconds)
{
  const double old = st::comm_timeout_s();
  st::g_comm_timeout_s.store(seconds > 0.0 ? seconds : -1.0, std::memory_order_relaxed);
  return old;
}

int
st_rccl_version(int* version_code, char* path, int path_len)
{
  st::clear_error();
  std::string p;
  const int rc = st::rccl_version(version_code, &p);
  if (path && path_len > 0)
    std::snprintf(path, (size_t)path_len, "%s", p.c_str());
  if (rc)
    st::set_error("st_rccl_version: ncclGetVersion failed");
  return rc;
}

double
st_get_comm_timeout(void)
{
  return st::comm_timeout_s();
}

int
st_comm_unique_id(char* id_out /* ST_COMM_ID_BYTES */)
{
  st::clear_error();
  ST_REQUIRE(id_out, "st_comm_unique_id: null output");
  // st_rendezvous.hip; an id never joined is reaped after two deadlines
  return st::rdv_make_id(id_out, nullptr, 2.0 * st::comm_timeout_s() + 30.0);
}

int
st_comm_unique_id_addr(char* id_out, const char* addr)
{
  st::clear_error();
  ST_REQUIRE(id_out, "st_comm_unique_id_addr: null output");
  return st::rdv_make_id(id_out, addr, 2.0 * st::comm_timeout_s() + 30.0);
}

int
st_comm_id_release(const char* id)
{
  st::clear_error();
  ST_REQUIRE(id, "st_comm_id_release: null id");
  return st::rdv_release(id);
}

int
st_comm_init(void** comm, int nranks, int rank, const char* id_in, int device)
{
  st::clear_error();
  st::DeviceGuard guard;
  ST_REQUIRE(comm && id_in, "st_comm_init: null pointer");
  ST_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "st_comm_init: bad rank");
  *comm = nullptr;
  // every rank proves presence first; the host makes the RCCL id only then
  // (st_rendezvous.hip), so no rank enters RCCL while a peer is missing
  ncclUniqueId id;
  static_assert(sizeof(id.internal) == st::kRdvPayloadBytes, "RCCL id size");
  if (st::rdv_join(
        id_in, nranks, rank, device, st::comm_timeout_s(),
        [device](char* out) {
          ncclUniqueId u;
          if (hipSetDevice(device) != hipSuccess ||
              ncclGetUniqueId(&u) != ncclSuccess)
            return -1;
          std::memcpy(out, u.internal, sizeof u.internal);
          return 0;
        },
        id.internal))
    return -1;
  ST_CHECK(hipSetDevice(device));
  auto job = std::make_shared<st::InitJob>();
  job->comms.assign(1, nullptr);
  if (st::init_with_deadline(
        job,
        [id, nranks, rank, device](st::InitJob& j) {
          if (hipSetDevice(device) != hipSuccess)
            return ncclUnhandledCudaError;
          ncclConfig_t cfg = st::comm_config();
          return ncclCommInitRankConfig(&j.comms[0], nranks, id, rank, &cfg);
        },
        &rank, &device, "st_comm_init"))
    return -1;
  auto* b = new st::CommBox;
  b->c = job->comms[0];
  b->rank = rank;
  b->dev = device;
  *comm = b;
  return 0;
}

int
st_comm_destroy(void* comm)
{
  st::clear_error();
  st::DeviceGuard guard;
  if (!comm)
    return 0;
  auto* b = static_cast<st::CommBox*>(comm);
  // finalize (flushes this rank's collectives; non-blocking, so under the
  // deadline), then free; a communicator that cannot finalize is aborted
  int rc = st::comm_collective(b, ncclCommFinalize(b->c), "st_comm_destroy");
  const ncclResult_t r = rc ? ncclCommAbort(b->c) : ncclCommDestroy(b->c);
  delete b;
  if (rc)
    return -1;
  ST_NCCL(r);
  return 0;
}

int
st_comm_info(void* comm, int* nranks, int* rank, int* device)
{
  st::clear_error();
  ST_REQUIRE(comm, "st_comm_info: null communicator");
  const ncclComm_t c = static_cast<st::CommBox*>(comm)->c;
  if (nranks)
    ST_NCCL(ncclCommCount(c, nranks));
  if (rank)
    ST_NCCL(ncclCommUserRank(c, rank));
  if (device)
    ST_NCCL(ncclCommCuDevice(c, device));
  return 0;
}

int
st_allgather_f32(void* comm, const float* send, float* recv, uint64_t count,
                 void* stream)
{
  st::clear_error();
  ST_REQUIRE(comm && send && recv, "st_allgather: null pointer");
  auto* b = static_cast<st::CommBox*>(comm);
  return st::comm_collective(
    b,
    ncclAllGather(send, recv, count, ncclFloat, b->c,
                  reinterpret_cast<hipStream_t>(stream)),
    "st_allgather");
}

int
st_allgather_f64(void* comm, const double* send, double* recv, uint64_t count,
                 void* stream)
{
  st::clear_error();
  ST_REQUIRE(comm && send && recv, "st_allgather: null pointer");
  auto* b = static_cast<st::CommBox*>(comm);
  return st::comm_collective(
    b,
    ncclAllGather(send, recv, count, ncclDouble, b->c,
                  reinterpret_cast<hipStream_t>(stream)),
    "st_allgather");
}

} // extern "C"
