/*
 * capi_sanitize.c — the library's host code under AddressSanitizer and
 * UndefinedBehaviorSanitizer (device code untouched: -Xarch_host only).
 * Built and run by tools/host_asan.sh on a machine without a GPU: every
 * C-ABI entry point that validates before touching the device is called
 * with good and bad arguments (the drop-in pair with a NULL queue, the
 * step kernels' argument checks, the policy query over every form and size
 * class, the tuning setters and their range checks, the communicator calls'
 * argument errors, the deadline setter, st_comm_init's pre-RCCL rendezvous
 * - a missing rank, three ranks as threads of this process, three ranks
 * beside a stray connector that never says hello and one that sends
 * garbage, a rank that hung up before the host joined, an id released
 * unjoined - and the RCCL version query), so the host-side parsing, error formatting
 * (eigen_last_error), table lookups and socket code run under the
 * sanitizers.
 * Exit 0 = clean.
 */
#include <arpa/inet.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "similarity_transform.h"
#include "st_tuning.h" /* built with -DST_TUNING_ABI=1 (tools/host_asan.sh) */

static int fails = 0;

/* three ranks of one rendezvous as threads: joined[r] = 0 (RCCL joined, a
   device) or 1 (the rendezvous passed, the RCCL id could not be made), 2 =
   anything else */
static char rdv_id[ST_COMM_ID_BYTES];
static int joined[3] = { 2, 2, 2 };

static void*
join_rank(void* arg)
{
  const int r = *(const int*)arg;
  void* c = NULL;
  if (st_comm_init(&c, 3, r, rdv_id, 0) == 0) {
    joined[r] = 0;
    st_comm_destroy(c);
  } else if (strstr(eigen_last_error(), "could not make the RCCL id") ||
             strstr(eigen_last_error(), "ncclCommInitRankConfig")) {
    joined[r] = 1;
  }
  return NULL;
}
/* a TCP connection to the id's listener (address and port at bytes 16..21
   of the id, network order), as a stray or hostile connector would make */
static int
connect_to_id(const char* idb)
{
  struct sockaddr_in sa;
  memset(&sa, 0, sizeof sa);
  sa.sin_family = AF_INET;
  memcpy(&sa.sin_addr.s_addr, idb + 16, 4);
  memcpy(&sa.sin_port, idb + 20, 2);
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd >= 0 && connect(fd, (struct sockaddr*)&sa, sizeof sa) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

static double
now_s(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      fprintf(stderr, "%s:%d: check failed: %s (%s)\n", __FILE__, __LINE__, #c,  \
              eigen_last_error());                                               \
      fails++;                                                                   \
    }                                                                            \
  } while (0)

int
main(void)
{
  setvbuf(stdout, NULL, _IONBF, 0); /* LeakSanitizer exits without a flush */
  /* the drop-in pair with a NULL queue: negative return (make_queue writes
     NULL and an error without a device; with one, the queue is released) */
  void* q = (void*)1;
  make_queue(&q);
  if (q)
    destroy_queue(q);
  else
    CHECK(strlen(eigen_last_error()) > 0);
  float m[9] = { 1, 1, 2, 2, 1, 3, 2, 3, 5 }, lam = 0, v[3];
  unsigned int it = 0;
  CHECK(max_eigen_value(NULL, m, &lam, v, 3, &it) < 0);
  CHECK(max_eigen_value_f64(NULL, NULL, NULL, NULL, 3, NULL) < 0);
  destroy_queue(NULL);

  /* the launch policy over every form, dtype and size class */
  static const unsigned int sizes[][2] = { { 1024, 1024 },  { 4096, 4096 },   { 6144, 6144 },
                                           { 8192, 8192 },  { 2880, 23040 },  { 12288, 12288 },
                                           { 32768, 32768 }, { 8192, 65536 }, { 5824, 11648 } };
  for (int d = 0; d < 2; d++)
    for (size_t i = 0; i < sizeof sizes / sizeof sizes[0]; i++)
      for (int form = 0; form <= 4; form++)
        for (unsigned int np = 0; np < 7; np++) {
          st_launch_policy p;
          memset(&p, 0xff, sizeof p);
          const int rc = st_launch_policy_query(d, sizes[i][0], sizes[i][1], form, np, &p);
          if (rc == 0)
            CHECK(p.rows >= 1 && p.rows <= 8 && p.kernel >= 0 && p.kernel <= 5);
          else
            CHECK(strlen(eigen_last_error()) > 0);
        }
  CHECK(st_launch_policy_query(1, 8192, 8192, 0, 0, NULL) < 0);
  CHECK(st_launch_policy_query(3, 8192, 8192, 0, 0, NULL) < 0);

  /* tuning setters: range checks, read-back, restore */
  CHECK(st_set_defer_caps(2, 0, 0, 4) < 0);
  const int old = st_set_defer_caps(1, 1, 6, 5);
  CHECK(old >= 0 && st_set_defer_caps(1, 1, 6, (unsigned)old) == 5);
  CHECK(st_set_every_cache(9, 0) < 0);
  CHECK(st_set_mfree_shape(9) < 0);
  {
    const int k0 = st_set_k0_reverse(1);
    CHECK(k0 >= -1 && k0 <= 1 && st_set_k0_reverse(k0) == 1);
  }
  CHECK(st_defer_ntload_class(8192, 8192, 7) < 0);
  CHECK(st_every_cache_class(8192, 8192, 1) == 1);
  CHECK(st_round_flat_pays(8192, 8192, 1) == 1 && st_defer_rounds(8192, 8192, 1) == 6);

  /* communicator calls: argument errors before any RCCL or HIP call */
  void* comm = (void*)1;
  char id[128] = { 0 };
  CHECK(st_comm_init(&comm, 2, 5, id, 0) < 0);
  CHECK(st_comm_init(NULL, 1, 0, id, 0) < 0);
  CHECK(st_comm_info(NULL, NULL, NULL, NULL) < 0);
  CHECK(st_comm_destroy(NULL) == 0);
  double buf[4];
  CHECK(st_allgather_f64(NULL, buf, buf, 1, NULL) < 0);
  const double t0 = st_set_comm_timeout(0.0);
  CHECK(st_set_comm_timeout(2.5) == t0 && st_set_comm_timeout(0.0) == 2.5);

  /* st_comm_init's rendezvous (st_rendezvous.hip): a foreign id, rank 0 of
     2 alone (missing rank named after the 1 s deadline, no RCCL state),
     three ranks as threads (the host is whichever claims the listener;
     without a device they all report the RCCL id failure) */
  memset(id, 1, sizeof id);
  CHECK(st_comm_init(&comm, 2, 0, id, 0) < 0 &&
        strstr(eigen_last_error(), "not made by st_comm_unique_id") != NULL);
  st_set_comm_timeout(1.0);
  CHECK(st_get_comm_timeout() == 1.0);
  CHECK(st_comm_unique_id(rdv_id) == 0);
  CHECK(st_comm_init(&comm, 2, 0, rdv_id, 0) < 0 &&
        strstr(eigen_last_error(), "rank 1 of 2 did not reach st_comm_init") != NULL);
  CHECK(st_comm_unique_id(rdv_id) == 0);
  pthread_t th[3];
  int ranks[3] = { 2, 0, 1 };
  for (int i = 0; i < 3; i++)
    pthread_create(&th[i], NULL, join_rank, &ranks[i]);
  for (int i = 0; i < 3; i++)
    pthread_join(th[i], NULL);
  for (int i = 0; i < 3; i++)
    CHECK(joined[i] == 0 || joined[i] == 1);
  /* a stray connector that never says hello and one that sends garbage,
     connected before the ranks: the host drops them without holding up the
     three ranks (the hellos are read from one poll set) */
  st_set_comm_timeout(20.0);
  CHECK(st_comm_unique_id(rdv_id) == 0);
  const int stray = connect_to_id(rdv_id), noisy = connect_to_id(rdv_id);
  CHECK(stray >= 0 && noisy >= 0);
  if (noisy >= 0)
    CHECK(write(noisy, "GET / HTTP/1.0\r\n\r\n", 18) == 18);
  for (int i = 0; i < 3; i++)
    joined[i] = 2;
  double t_s = now_s();
  for (int i = 0; i < 3; i++)
    pthread_create(&th[i], NULL, join_rank, &ranks[i]);
  for (int i = 0; i < 3; i++)
    pthread_join(th[i], NULL);
  for (int i = 0; i < 3; i++)
    CHECK(joined[i] == 0 || joined[i] == 1);
  CHECK(now_s() - t_s < 4.0); /* not the stray's 5 s hello window */
  if (stray >= 0)
    close(stray);
  if (noisy >= 0)
    close(noisy);
  /* the released id: its listener is closed, a peer cannot reach it */
  CHECK(st_comm_unique_id(rdv_id) == 0);
  CHECK(st_comm_id_release(rdv_id) == 0 && st_comm_id_release(rdv_id) == 1);
  CHECK(connect_to_id(rdv_id) < 0);
  st_set_comm_timeout(0.0);
  int vcode = 0;
  char vpath[512];
  CHECK(st_rccl_version(&vcode, vpath, (int)sizeof vpath) == 0 && vcode >= 22000 &&
        strstr(vpath, "librccl") != NULL);

  /* with a device: the real solve paths' host code (drop-in fp32 on a
     k_round block, fp64 on a flat block with deferred writes, the native
     multi-GPU solve at P = 1, a one-rank communicator) */
  void* wq = NULL;
  make_queue(&wq);
  if (wq) {
    static float hf[512 * 512];
    static double hd[9216];
    float vf[512];
    for (int r = 0; r < 512; r++)
      for (int c = 0; c < 512; c++)
        hf[r * 512 + c] = 1.0f / (float)(r + c + 1);
    CHECK(max_eigen_value(wq, hf, &lam, vf, 512, &it) >= 0 && it == 12);
    st_options opt = { -1.0, 0, 0, 0, 0 };
    st_stats stt;
    double ld = 0;
    CHECK(st_solve_multi_f64(NULL, 9216, 1, NULL, 2, 3, &ld, hd, &it, &opt, &stt) >= 0);
    CHECK(ld > 4000 && stt.rounds >= 1);
    char uid[128];
    void* c1 = NULL;
    int nr = 0;
    CHECK(st_comm_unique_id(uid) == 0 && st_comm_init(&c1, 1, 0, uid, 0) == 0);
    CHECK(st_comm_info(c1, &nr, NULL, NULL) == 0 && nr == 1);
    CHECK(st_comm_destroy(c1) == 0);
    destroy_queue(wq);
    printf("device paths run\n");
  }

  /* the version string and the probe switches */
  CHECK(strncmp(st_version(), "eigen_value_amd", 15) == 0);
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("host C-ABI clean under ASan/UBSan\n");
  return 0;
}
