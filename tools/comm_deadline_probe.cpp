// comm_deadline_probe.cpp — where does a non-blocking RCCL init with a
// missing peer spend its time?  Rank 0 of 2 joins a fresh unique id and
// rank 1 never arrives; every step is timestamped (stderr, unbuffered):
// ncclCommInitRankConfig(blocking = 0) -> polls of ncclCommGetAsyncError
// for CDP_WAIT seconds -> ncclCommAbort (CDP_ABORT=0: skip the abort and
// leave the communicator).  Diagnoses the library's deadline path
// (st_multi.hip comm_wait) on the GPU box.
//
// Build: make -C tools comm_deadline_probe
// Run:   timeout -k 5 60 ./tools/comm_deadline_probe
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

static double
now_s()
{
  static const auto t0 = std::chrono::steady_clock::now();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

int
main()
{
  const double wait = std::getenv("CDP_WAIT") ? std::atof(std::getenv("CDP_WAIT")) : 3.0;
  const bool do_abort = !std::getenv("CDP_ABORT") || std::atoi(std::getenv("CDP_ABORT"));
  std::fprintf(stderr, "[%7.3f] hipSetDevice\n", now_s());
  if (hipSetDevice(0) != hipSuccess)
    return 2;
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  std::fprintf(stderr, "[%7.3f] ncclGetUniqueId -> %d\n", now_s(), (int)r);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.blocking = 0;
  ncclComm_t c = nullptr;
  if (std::getenv("CDP_THREAD")) {
    // the init in a helper thread; this thread waits CDP_WAIT s, then looks
    // at the handle RCCL wrote (if any), optionally aborts it, and exits
    static ncclComm_t hc = nullptr;
    static int done = 0;
    std::thread([id, cfg]() mutable {
      (void)hipSetDevice(0);
      const ncclResult_t q = ncclCommInitRankConfig(&hc, 2, id, 0, &cfg);
      std::fprintf(stderr, "[%7.3f] helper: ncclCommInitRankConfig -> %d\n", now_s(), (int)q);
      __atomic_store_n(&done, 1, __ATOMIC_RELEASE);
    }).detach();
    while (now_s() < wait + 0.3 && !__atomic_load_n(&done, __ATOMIC_ACQUIRE))
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    c = __atomic_load_n(&hc, __ATOMIC_ACQUIRE);
    std::fprintf(stderr, "[%7.3f] helper done %d, comm %p\n", now_s(),
                 __atomic_load_n(&done, __ATOMIC_ACQUIRE), (void*)c);
    if (c) {
      ncclResult_t st = ncclSuccess;
      const ncclResult_t q = ncclCommGetAsyncError(c, &st);
      std::fprintf(stderr, "[%7.3f] GetAsyncError -> %d, state %d\n", now_s(), (int)q, (int)st);
    }
    if (c && do_abort) {
      std::fprintf(stderr, "[%7.3f] ncclCommAbort ...\n", now_s());
      r = ncclCommAbort(c);
      std::fprintf(stderr, "[%7.3f] ncclCommAbort -> %d\n", now_s(), (int)r);
    }
    std::fprintf(stderr, "[%7.3f] main returns\n", now_s());
    return 0;
  }
  std::fprintf(stderr, "[%7.3f] ncclCommInitRankConfig(nranks 2, rank 0, blocking 0) ...\n",
               now_s());
  r = ncclCommInitRankConfig(&c, 2, id, 0, &cfg);
  std::fprintf(stderr, "[%7.3f] ncclCommInitRankConfig -> %d (%s), comm %p\n", now_s(), (int)r,
               ncclGetErrorString(r), (void*)c);
  if (!c)
    return 3;
  const double t_end = now_s() + wait;
  ncclResult_t st = ncclInProgress;
  int polls = 0;
  while (now_s() < t_end) {
    const ncclResult_t q = ncclCommGetAsyncError(c, &st);
    polls++;
    if (q != ncclSuccess || st != ncclInProgress) {
      std::fprintf(stderr, "[%7.3f] GetAsyncError -> %d, state %d\n", now_s(), (int)q, (int)st);
      break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  std::fprintf(stderr, "[%7.3f] %d polls, state %d (%s)\n", now_s(), polls, (int)st,
               ncclGetErrorString(st));
  if (do_abort) {
    std::fprintf(stderr, "[%7.3f] ncclCommAbort ...\n", now_s());
    r = ncclCommAbort(c);
    std::fprintf(stderr, "[%7.3f] ncclCommAbort -> %d\n", now_s(), (int)r);
  }
  std::fprintf(stderr, "[%7.3f] exit\n", now_s());
  return 0;
}
