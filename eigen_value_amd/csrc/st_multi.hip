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

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "st_internal.h"

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
// passes (comm_wait / comm_settle).  Creation, which RCCL does not return
// from while a peer is missing, runs on a helper thread under the same
// deadline (init_with_deadline).  Past it the communicators are aborted and
// the call returns -1 with the stalled rank and device named, instead of
// hanging in ncclCommInitRank / ncclCommInitAll / the first all-gather.
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

// Communicator creation under the deadline.  RCCL 2.27's
// ncclCommInitRankConfig does not return to its caller while a peer is
// missing, non-blocking config or not, and ncclCommGetAsyncError reports
// ncclSuccess on the half-made handle meanwhile; but the handle is written
// early, and ncclCommAbort from another thread returns at once and makes
// the blocked init return an error (tools/comm_deadline_probe.cpp,
// profiles/r04_comm_deadline_probe.log).  So the init runs on a helper
// thread, which also completes the non-blocking group job (its state is
// thread-local to the thread that ended the group: the helper must not
// exit before the communicators are ready), and this thread waits for it at
// most the deadline; past it, every handle RCCL wrote is aborted and the
// helper is given a few seconds to return.  RCCL's abort does not always
// unblock it (tests/test_gpu_fullsize.py: returned at once in some runs,
// not within 10 s in another), and a process that then exits normally can
// crash in the runtimes' teardown behind the blocked thread, so the error
// says so: a job that lost a peer should end with _exit (bench.py's
// watchdog does).
struct InitJob
{
  std::vector<ncclComm_t> comms; // written by RCCL (early)
  ncclResult_t r = ncclInProgress;
  int done = 0; // __atomic
};

int
init_with_deadline(const std::shared_ptr<InitJob>& job,
                   std::function<ncclResult_t(InitJob&)> body, const int* ranks,
                   const int* devs, const char* what)
{
  std::thread([job, body]() {
    ncclResult_t r = body(*job);
    // finish an asynchronous init here, in the thread that started it
    for (bool pending = (r == ncclInProgress); pending;) {
      pending = false;
      for (ncclComm_t c : job->comms) {
        ncclResult_t st = ncclSuccess;
        if (!c)
          continue;
        if (ncclCommGetAsyncError(c, &st) != ncclSuccess)
          st = ncclInternalError;
        if (st == ncclInProgress)
          pending = true;
        else if (st != ncclSuccess && r == ncclInProgress)
          r = st;
      }
      if (pending)
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    if (r == ncclInProgress)
      r = ncclSuccess;
    job->r = r;
    __atomic_store_n(&job->done, 1, __ATOMIC_RELEASE);
  }).detach();
  const double limit = comm_timeout_s();
  const auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&t0]() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0)
      .count();
  };
  while (!__atomic_load_n(&job->done, __ATOMIC_ACQUIRE)) {
    const double el = elapsed();
    if (el > limit) {
      int aborted = 0;
      for (size_t i = 0; i < job->comms.size(); i++) {
        ncclComm_t c = __atomic_load_n(&job->comms[i], __ATOMIC_ACQUIRE);
        if (c) {
          (void)ncclCommAbort(c);
          aborted++;
        }
      }
      // the aborted init returns an error; give the helper a moment
      const double t_ab = elapsed();
      while (!__atomic_load_n(&job->done, __ATOMIC_ACQUIRE) && elapsed() < t_ab + 10.0)
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      // name the rank (or, for a single-process group, every rank and
      // device: any of them may be the one stalled)
      std::string who = "RCCL rank " + std::to_string(ranks[0]) + " (device " +
                        std::to_string(devs[0]) + ")";
      if (job->comms.size() > 1) {
        who = "RCCL ranks 0.." + std::to_string(job->comms.size() - 1) + " (devices";
        for (size_t i = 0; i < job->comms.size(); i++)
          who += " " + std::to_string(devs[i]);
        who += ")";
      }
      const bool stuck = !__atomic_load_n(&job->done, __ATOMIC_ACQUIRE);
      ::st::set_error("%s: %s still in progress after %.1f s (deadline %.1f s, "
                      "ST_COMM_TIMEOUT_S / st_set_comm_timeout): a peer did not "
                      "arrive; %d communicator(s) aborted%s",
                      what, who.c_str(), el, limit, aborted,
                      stuck ? "; the RCCL init thread did not return and is left "
                              "behind (end the process with _exit)"
                            : "");
      return -1;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(500));
  }
  if (job->r != ncclSuccess) {
    ::st::set_error("%s: ncclCommInitRankConfig (RCCL rank %d, device %d) "
                    "failed: %s",
                    what, ranks[0], devs[0], ncclGetErrorString(job->r));
    for (ncclComm_t c : job->comms)
      if (c)
        (void)ncclCommAbort(c);
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
    for (auto& d : sh) {
      (void)hipSetDevice(d.dev);
      if (d.stream)
        (void)hipStreamSynchronize(d.stream);
      if (d.comm)
        (void)(abort ? ncclCommAbort(d.comm) : ncclCommDestroy(d.comm));
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
  ST_NCCL(ncclGroupStart());
  for (size_t p = 0; p < M.sh.size(); p++) {
    Shard<T>& d = M.sh[p];
    T* buf = d.s[which];
    ST_NCCL(ncclAllGather(buf + p * chunk, buf, chunk, nccl_type<T>(), d.comm,
                          d.stream));
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
    if (!mfree && round_flat_pays(d.nrows, n, sizeof(T)))
      ST_CHECK(hipMalloc(&d.part, sizeof(T) * round_flat_scratch(d.nrows, n)));
    d.defer = d.part != nullptr && !every;
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
    batch = M.sh[0].part ? 2u : 8u;
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
            if (q != ncclSuccess && q != ncclInProgress)
              r = q;
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
      return -1; // the communicators were aborted (or are left to the helper)
    }
  }
  for (uint32_t p = 0; p < P; p++) { // s_0 = rowsum(A_0), then gather
    Shard<T>& d = M.sh[p];
    ST_CHECK(hipSetDevice(d.dev));
    if (launch_rowsum<T>(d.a, d.s[0] + p * chunk, d.nrows, n, d.stream))
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
        } else if (d.part)
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
st_comm_unique_id(char* id_out /* NCCL_UNIQUE_ID_BYTES */)
{
  st::clear_error();
  ST_REQUIRE(id_out, "st_comm_unique_id: null output");
  ncclUniqueId id;
  ST_NCCL(ncclGetUniqueId(&id));
  std::memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int
st_comm_init(void** comm, int nranks, int rank, const char* id_in, int device)
{
  st::clear_error();
  st::DeviceGuard guard;
  ST_REQUIRE(comm && id_in, "st_comm_init: null pointer");
  ST_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "st_comm_init: bad rank");
  *comm = nullptr;
  ST_CHECK(hipSetDevice(device));
  ncclUniqueId id;
  std::memcpy(id.internal, id_in, NCCL_UNIQUE_ID_BYTES);
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
