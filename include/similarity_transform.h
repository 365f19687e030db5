/*
 * similarity_transform.h — C-ABI of libsimilarity_transform.so, the
 * MI355X (gfx950) implementation of the similarity-transform maximum
 * eigenvalue iteration.
 *
 * Plain C: pointers, sizes, no torch or HIP types in any signature
 * (streams are passed as `void*` = hipStream_t).  Citations refer to the
 * reference tree (itzmeanjan/eigen_value), path:line.
 *
 * Layers
 *   1. Drop-in exports: exactly the two symbols the reference's Python
 *      wrapper binds (wrapper/python/similarity_transform.py:33-37,63-69).
 *   2. Additions at the same level (fp64 twin, queue teardown, last error,
 *      an extended call with options and statistics).
 *   3. Device-resident solve (input already in HBM; bench and torch users).
 *   4. Step-level kernels on a caller stream: what the row-block sharded
 *      driver (eigen_value_amd/sharded.py) and the kernel unit tests call.
 *
 * Errors: nothing throws across this ABI.  Functions returning int64_t /
 * int return a negative value on error and record a message readable with
 * eigen_last_error() (thread-local).  make_queue writes NULL on failure.
 *
 * Threading: a queue (context) is used by one host thread at a time.
 */
#ifndef EIGEN_VALUE_AMD_SIMILARITY_TRANSFORM_H
#define EIGEN_VALUE_AMD_SIMILARITY_TRANSFORM_H

#include <stdint.h>

/* the library is built with -fvisibility=hidden: what this header declares
 * is its whole dynamic ABI */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

#ifdef __cplusplus
extern "C" {
#endif

/* include/similarity_transform.hpp:4-5 */
#define ST_EPS_F32 1e-3f
#define ST_EPS_F64 1e-3
#define ST_MAX_ITR 1000u

/* semantics of the round loop */
#define ST_SEM_SYCL 0u   /* similarity_transform.cpp: cyclic stop (413-417),   */
                         /* A *= (1/s_r)*s_c (324-325), count = break idx (54) */
#define ST_SEM_MAINPY 1u /* main.py: non-cyclic stop (25-27),                 */
                         /* ((1/s_r)*A)*s_c (13-16), count = itr + 1 (47)     */

/* ---------------------------------------------------------------------- */
/* 1. drop-in exports                                                      */
/* ---------------------------------------------------------------------- */

/* replaces wrapper/similarity_transform.cpp:3-12 (sycl::default_selector
 * queue).  Creates a context on the current HIP device (env
 * EIGEN_VALUE_DEVICE overrides) with its own non-blocking stream.
 * *wq = NULL on failure. */
void make_queue(void** wq);

/* replaces wrapper/similarity_transform.cpp:14-37 and, behind it,
 * similarity_transform.cpp:5-75.  fp32, reference semantics (ST_SEM_SYCL,
 * EPS = 1e-3f, MAX_ITR = 1000).  `mat` (dim x dim, row-major) is read only.
 * Writes eigen_val[0], eigen_vec[0..dim), *iter_cnt.  Returns elapsed ms
 * (steady clock, host->device copy of `mat` included, as the reference's
 * lazily-copied buffer is) or a negative value on error.  Any dim >= 1 is
 * accepted (the reference required dim % work-group-size == 0). */
int64_t max_eigen_value(void* wq, float* mat, float* eigen_val,
                        float* eigen_vec, unsigned int dim,
                        unsigned int* iter_cnt);

/* ---------------------------------------------------------------------- */
/* 2. additions                                                            */
/* ---------------------------------------------------------------------- */

/* fp64 twin of max_eigen_value (EPS = 1e-3). */
int64_t max_eigen_value_f64(void* wq, double* mat, double* eigen_val,
                            double* eigen_vec, unsigned int dim,
                            unsigned int* iter_cnt);

/* Frees a context from make_queue (the reference leaks its queue). */
void destroy_queue(void* wq);

/* Message of the last error on this thread ("" if none). */
const char* eigen_last_error(void);

typedef struct st_options
{
  double eps;         /* stop tolerance; < 0 selects the dtype default     */
  uint32_t max_itr;   /* 0 selects ST_MAX_ITR                               */
  uint32_t semantics; /* ST_SEM_SYCL or ST_SEM_MAINPY                       */
  uint32_t batch;     /* rounds enqueued per host flag check; 0 = default   */
  uint32_t flags;     /* ST_FLAG_* below                                    */
} st_options;

#define ST_FLAG_TIME_KERNELS 1u /* hipEvents around every fused launch     */
#define ST_FLAG_MATRIX_FREE 2u  /* st_mfree_round_* instead of the in-place */
                                /* transform (input never written)         */
#define ST_FLAG_WRITE_EVERY_ROUND 8u /* store the matrix every round; by    */
                                /* default the flat round (>= 144 MiB)      */
                                /* stores it every 6th round (st_defer_     */
                                /* rounds) and re-applies                   */
                                /* the pending scalings in registers:       */
                                /* identical results, fewer bytes           */
#define ST_FLAG_ROUND_LOOP 4u   /* one launch per round even where the whole */
                                /* solve fits one workgroup (n <= 128 fp64, */
                                /* 256 fp32): results are identical        */
#define ST_FLAG_TRACE_SUMS 16u  /* record every evaluated round's row sums  */
                                /* s_k (st_last_round_sums; max_itr * dim   */
                                /* elements <= 1 GiB): identical results    */

typedef struct st_stats
{
  double h2d_ms;          /* host->device copy of the input               */
  double loop_ms;         /* first kernel .. convergence observed on host */
  double d2h_ms;          /* eigenvector / eigenvalue copy back           */
  double fused_ms_total;  /* sum of fused scale+rowsum kernel times       */
  double rowsum_ms;       /* the initial row-sum pass                     */
  uint32_t fused_launches;/* fused launches timed                         */
  uint32_t rounds;        /* row-sum evaluations performed                */
  uint32_t converged;     /* 1 if the stop test passed before max_itr     */
  uint32_t reserved;
} st_stats;

/* Extended host-pointer solve.  dtype: 0 = float32, 1 = float64.
 * opt / stats may be NULL. */
int64_t max_eigen_value_ex(void* wq, int dtype, const void* mat,
                           void* eigen_val, void* eigen_vec,
                           unsigned int dim, unsigned int* iter_cnt,
                           const st_options* opt, st_stats* stats);

/* Per-round kernel times (ms) of the last solve on this queue that ran
 * with ST_FLAG_TIME_KERNELS: copies min(cap, n) values into ms and returns
 * n, the number of rounds that did work (0 if the last solve was not
 * timed), or a negative value on error. */
int st_last_round_times(void* wq, float* ms, unsigned int cap);

/* Row sums of the last solve on this queue that ran with ST_FLAG_TRACE_SUMS:
 * s_k for the evaluated rounds k = 0 .. n-1 (the vectors the stop test of
 * similarity_transform.cpp:413-421 compared), copied as min(cap_rounds, n)
 * rows of dim elements of the solve's dtype into `sums`.  Returns n (0 if the
 * last solve was not traced) or a negative value on error. */
int st_last_round_sums(void* wq, void* sums, unsigned int cap_rounds);

/* Make the context launch on a caller stream (a hipStream_t; NULL is the
 * HIP null stream, which is torch's default stream).  Returns 0 or
 * negative.  st_use_own_stream restores the context's own non-blocking
 * stream (the make_queue default). */
int st_set_stream(void* wq, void* stream);
int st_use_own_stream(void* wq);

/* ---------------------------------------------------------------------- */
/* 3. device-resident solve                                                */
/* ---------------------------------------------------------------------- */

/* d_mat: device pointer, dim x dim row-major; TRANSFORMED IN PLACE (it is
 * the private working copy the reference makes at
 * similarity_transform.cpp:14,19).  On return d_mat holds A_end, where end =
 * st_stats.rounds = the rounds evaluated: the launch that evaluates the
 * stopping round still applies its transform, so a converged solve leaves
 * one transform more than the reference's working copy, whose loop breaks
 * before compute_next_matrix (similarity_transform.cpp:45-52); an
 * exhausted solve (MAX_ITR rounds) leaves A_MAX_ITR like the reference.
 * lambda, the eigenvector and iter_cnt do not depend on it.  d_eigen_vec:
 * device pointer [dim] or
 * NULL (then eigen_vec_host must be non-NULL and receives it).
 * eigen_val / iter_cnt: host pointers.  Returns loop ms or negative. */
int64_t st_solve_device_f32(void* wq, float* d_mat, unsigned int dim,
                            float* d_eigen_vec, float* eigen_vec_host,
                            float* eigen_val, unsigned int* iter_cnt,
                            const st_options* opt, st_stats* stats);
int64_t st_solve_device_f64(void* wq, double* d_mat, unsigned int dim,
                            double* d_eigen_vec, double* eigen_vec_host,
                            double* eigen_val, unsigned int* iter_cnt,
                            const st_options* opt, st_stats* stats);

/* ---------------------------------------------------------------------- */
/* 3b. native multi-GPU solve (one process, ngpus devices, RCCL)           */
/* ---------------------------------------------------------------------- */

/* Row-block sharded solve over `ngpus` devices (`devices` = list of HIP
 * device ids, or NULL for 0..ngpus-1) with ONE ncclAllGather of the row-sum
 * vector per round.  Input: gen_kind 0 = host matrix `mat`
 * (dim x dim, row-major; each device copies its rows), 1 = Hilbert,
 * 2 = seeded random (generated on each device for its rows; `mat` unused).
 * Outputs on the host.  opt may select ST_FLAG_MATRIX_FREE.  stats->h2d_ms
 * reports the setup (allocation, input, communicator, first row sums),
 * stats->loop_ms the round loop.  Returns total ms or negative. */
int64_t st_solve_multi_f32(const float* mat, unsigned int dim, int ngpus,
                           const int* devices, int gen_kind, uint64_t seed,
                           float* eigen_val, float* eigen_vec,
                           unsigned int* iter_cnt, const st_options* opt,
                           st_stats* stats);
int64_t st_solve_multi_f64(const double* mat, unsigned int dim, int ngpus,
                           const int* devices, int gen_kind, uint64_t seed,
                           double* eigen_val, double* eigen_vec,
                           unsigned int* iter_cnt, const st_options* opt,
                           st_stats* stats);

/* One-process-per-GPU RCCL communicator for the sharded step API: one
 * process calls st_comm_unique_id (ST_COMM_ID_BYTES), the caller
 * distributes the id, every rank calls st_comm_init (nranks, its rank, its
 * HIP device); the process that made the id must join too.  st_allgather is
 * ncclAllGather on `stream` (in place when send = recv + rank*count).
 *
 * Presence before RCCL: the id is a rendezvous id, not an RCCL one - the
 * maker listens on a TCP port of the address it advertises (ST_COMM_ADDR,
 * else the first IPv4 address of NCCL_SOCKET_IFNAME's or of the first up
 * non-loopback interface, else 127.0.0.1).  st_comm_init on every rank
 * first joins it; only when all nranks are present (and still connected)
 * does the maker create the RCCL id and hand it to all, every rank
 * acknowledges it, and only on the maker's final "go" does any rank enter
 * ncclCommInitRankConfig (all ranks enter RCCL or none does).  A rank that
 * does not arrive within the deadline makes st_comm_init return -1 on every
 * present rank, eigen_last_error() naming the missing ranks, with no RCCL
 * state created (the process exits normally).  Connections that present no
 * hello within 5 s are dropped without delaying the others.
 *
 * Deadline: every communicator is non-blocking (ncclConfig_t.blocking = 0)
 * and each step that waits for peers - the rendezvous, st_comm_init's RCCL
 * init, a collective's connection setup, st_comm_destroy, and the
 * communicator setup and all-gathers of st_solve_multi_* - waits at most
 * st_set_comm_timeout() seconds (default: the environment variable
 * ST_COMM_TIMEOUT_S, else 120).  Past it the call returns -1 naming the RCCL
 * rank and HIP device still in progress; a communicator whose init has
 * returned is aborted (ncclCommAbort), one whose init has not is left to
 * the init thread, which aborts it if the init ever returns (the error then
 * says to end the process with _exit: a peer died after the rendezvous). */
#define ST_COMM_ID_BYTES 128
int st_comm_unique_id(char* id_out);
/* The same, advertising `addr` (dotted IPv4, e.g. "127.0.0.1" when every
 * rank runs on this host; NULL = the choice above). */
int st_comm_unique_id_addr(char* id_out, const char* addr);
int st_comm_init(void** comm, int nranks, int rank, const char* id_in,
                 int device);
/* Close the listener of an id this process made and will not join (e.g. its
 * maker failed before st_comm_init): 0, or 1 if there is none (already
 * joined or released, or made elsewhere).  An id never joined nor released
 * is closed by a later st_comm_unique_id once 2 x the deadline + 30 s have
 * passed. */
int st_comm_id_release(const char* id);
int st_comm_destroy(void* comm);
/* Set the RCCL deadline in seconds (<= 0: back to ST_COMM_TIMEOUT_S / 120);
 * returns the previous effective value.  Process-wide. */
double st_set_comm_timeout(double seconds);
/* The effective RCCL deadline in seconds (the setter's, ST_COMM_TIMEOUT_S or
 * 120). */
double st_get_comm_timeout(void);
/* The RCCL the library's calls are bound to: *version_code = ncclGetVersion
 * (X*10000 + Y*100 + Z) and `path` = the file holding the bound
 * ncclAllGather (dladdr); inside a torch process that is torch's bundled
 * librccl, for a C caller the /opt/rocm one the library links.  Either
 * output may be NULL.  Returns 0 or -1.  No GPU needed. */
int st_rccl_version(int* version_code, char* path, int path_len);
/* What the communicator itself reports (ncclCommCount / ncclCommUserRank /
 * ncclCommCuDevice): the ranks RCCL joined, this rank, its HIP device.
 * Any output pointer may be NULL.  Returns 0 or negative. */
int st_comm_info(void* comm, int* nranks, int* rank, int* device);
int st_allgather_f32(void* comm, const float* send, float* recv,
                     uint64_t count, void* stream);
int st_allgather_f64(void* comm, const double* send, double* recv,
                     uint64_t count, void* stream);

/* ---------------------------------------------------------------------- */
/* 4. step-level kernels (asynchronous on `stream`, a hipStream_t or NULL) */
/* ---------------------------------------------------------------------- */

/* Device state of one solve (64 bytes, zero = fresh). */
typedef struct st_state
{
  uint32_t done;   /* 1 once the stop test passed or max_itr was reached  */
  uint32_t round;  /* row-sum evaluations that did not stop               */
  uint32_t iters;  /* reference iter_count, valid once done               */
  uint32_t stop;   /* stop flag of the last evaluated round               */
  double lambda;   /* s[0] of the last evaluated round                    */
  double max;      /* max row sum of the last evaluated round             */
  uint32_t end;    /* st_round_*: 1 + the round that stopped, 0 = running */
  /* scratch of the flat round's stats launch (st_round_flat_*); zero
   * between launches, as st_state_reset leaves it */
  uint32_t arrivals; /* workgroups done                                   */
  uint64_t max_bits; /* running max (bit pattern of a value >= 0)         */
  uint32_t fail;     /* some pair |s_i - s_{i+1}| >= eps (or NaN)          */
  uint32_t pad0;
  uint64_t pad[1];
} st_state;

/* zero a state (hipMemsetAsync) */
int st_state_reset(st_state* d_state, void* stream);

/* inputs for rows [row0, row0+nrows) of an ncols-wide matrix:
 *   hilbert  A[r][c] = 1/(r+c+1) in the element type (utils.cpp:137-154)
 *   random   U(0,1] from splitmix64(seed, r*ncols+c) (replaces the
 *            non-reproducible utils.cpp:125-134)
 *   identity (utils.cpp:5-27), fill (constant value) */
int st_generate_hilbert_f32(float* d_mat, unsigned int nrows,
                            unsigned int ncols, unsigned int row0,
                            void* stream);
int st_generate_hilbert_f64(double* d_mat, unsigned int nrows,
                            unsigned int ncols, unsigned int row0,
                            void* stream);
int st_generate_random_f32(float* d_mat, unsigned int nrows,
                           unsigned int ncols, unsigned int row0,
                           uint64_t seed, void* stream);
int st_generate_random_f64(double* d_mat, unsigned int nrows,
                           unsigned int ncols, unsigned int row0,
                           uint64_t seed, void* stream);
int st_generate_identity_f32(float* d_mat, unsigned int nrows,
                             unsigned int ncols, unsigned int row0,
                             void* stream);
int st_generate_identity_f64(double* d_mat, unsigned int nrows,
                             unsigned int ncols, unsigned int row0,
                             void* stream);
int st_fill_f32(float* d_x, uint64_t count, float value, void* stream);
int st_fill_f64(double* d_x, uint64_t count, double value, void* stream);

/* s[r] = sum_c A[r][c] for the nrows local rows (similarity_transform.cpp
 * :77-152, deterministic tree order, no atomics). */
int st_rowsum_f32(const float* d_mat, float* d_s, unsigned int nrows,
                  unsigned int ncols, void* stream);
int st_rowsum_f64(const double* d_mat, double* d_s, unsigned int nrows,
                  unsigned int ncols, void* stream);
/* The same row sums in the flat form, for blocks where st_round_flat_pays
 * (what the solve loops run as their initial pass there): one short
 * workgroup per (rows, column piece) writes partial sums into d_part
 * (st_round_flat_scratch(nrows, ncols) elements), a second launch sums each
 * row's pieces in a fixed order.  Deterministic and independent of the row
 * partition among blocks of one cache class, like st_round_flat's sums. */
int st_rowsum_flat_f32(const float* d_mat, float* d_s, float* d_part,
                       unsigned int nrows, unsigned int ncols, void* stream);
int st_rowsum_flat_f64(const double* d_mat, double* d_s, double* d_part,
                       unsigned int nrows, unsigned int ncols, void* stream);

/* Fused round body: for the local rows r in [0,nrows) (global row0 + r),
 *   A[r][c] = A[r][c] * ((1/s_cur[row0+r]) * s_cur[c])     (ST_SEM_SYCL)
 *   A[r][c] = ((1/s_cur[row0+r]) * A[r][c]) * s_cur[c]     (ST_SEM_MAINPY)
 * in place (similarity_transform.cpp:286-330 / main.py:13-16), and
 * s_next[r] = sum_c of the stored A[r][c] (the next round's row sums,
 * similarity_transform.cpp:40).  s_next may be NULL (transform only).
 * d_state may be NULL; otherwise the launch is a no-op once done != 0. */
int st_scale_rowsum_f32(float* d_mat, const float* d_s_cur, float* d_s_next,
                        unsigned int nrows, unsigned int ncols,
                        unsigned int row0, unsigned int semantics,
                        const st_state* d_state, void* stream);
int st_scale_rowsum_f64(double* d_mat, const double* d_s_cur,
                        double* d_s_next, unsigned int nrows,
                        unsigned int ncols, unsigned int row0,
                        unsigned int semantics, const st_state* d_state,
                        void* stream);

/* One whole round k in ONE launch (what the solve loop runs): from the full
 * row-sum vector s_cur = s_k (length ncols), for the local rows
 * r in [0,nrows) (global row0 + r):
 *   m_k = max(0, max s_k), v[row0+r] *= s_k[row0+r]/m_k, stop_k = all
 *   |s_k[i]-s_k[i+1]| < eps (cyclic for ST_SEM_SYCL), lambda = s_k[0],
 *   A <- D_k^-1 A D_k in place and s_next[r] = row sums of the stored A.
 * d_v is the FULL eigenvector accumulator (only the local rows are
 * written).  k is the round index (0-based); d_state->end = k+1 once the
 * round stops or k+1 == max_itr, and launches for later rounds are no-ops.
 * d_state must be zeroed (st_state_reset) before round 0. */
int st_round_f32(float* d_mat, const float* d_s_cur, float* d_s_next,
                 float* d_v, unsigned int nrows, unsigned int ncols,
                 unsigned int row0, float eps, unsigned int k,
                 unsigned int max_itr, unsigned int semantics,
                 st_state* d_state, void* stream);
int st_round_f64(double* d_mat, const double* d_s_cur, double* d_s_next,
                 double* d_v, unsigned int nrows, unsigned int ncols,
                 unsigned int row0, double eps, unsigned int k,
                 unsigned int max_itr, unsigned int semantics,
                 st_state* d_state, void* stream);

/* The same round for large blocks as two launches (k_flat, k_parts in
 * st_device.h): one short workgroup per (2 rows, 256 x 16-byte column
 * piece) for the in-place transform (the HBM serves many short workgroups
 * sweeping a compact address window faster than one long stream per CU),
 * whose first row group also derives m_k / stop_k / lambda / state from the
 * full s_k; then the pieces' partial sums into s_next in a fixed order and
 * the eigenvector update.
 * Results as st_round_* except the row sums' summation order (deterministic
 * and independent of the row partition among blocks of one cache class:
 * pieces are 8 KB of a row for fp64 blocks below 2 GiB, else 4 KB).
 * d_part: scratch of
 * st_round_flat_scratch(nrows, ncols) elements.  st_round_flat_pays tells
 * whether this form is the faster one for a block (dtype 0 = f32, 1 = f64);
 * the library's own solve loops use it for such blocks. */
int st_round_flat_f32(float* d_mat, const float* d_s_cur, float* d_s_next,
                      float* d_part, float* d_v, unsigned int nrows,
                      unsigned int ncols, unsigned int row0, float eps,
                      unsigned int k, unsigned int max_itr,
                      unsigned int semantics, st_state* d_state, void* stream);
int st_round_flat_f64(double* d_mat, const double* d_s_cur, double* d_s_next,
                      double* d_part, double* d_v, unsigned int nrows,
                      unsigned int ncols, unsigned int row0, double eps,
                      unsigned int k, unsigned int max_itr,
                      unsigned int semantics, st_state* d_state, void* stream);
uint64_t st_round_flat_scratch(unsigned int nrows, unsigned int ncols);
int st_round_flat_pays(unsigned int nrows, unsigned int ncols, int dtype);
/* The launch policy, as one map: what the solve loops launch for an
 * nrows x ncols block of `dtype` (0 fp32, 1 fp64; vector path, ncols a
 * multiple of 16 / sizeof element) in `form`, with `npend` pending rounds for
 * the deferred forms - read from the same shape functions and tables the
 * launchers use (st_kernels.hip), so tests/golden/launch_policy.json pins
 * every launch shape and cache policy.  Returns 0 or negative. */
#define ST_FORM_ROUND 0       /* a round that stores A (bench step; the
                                 solve's round below 144 MiB)                 */
#define ST_FORM_DEFER_READ 1  /* deferred writes: a read-only round          */
#define ST_FORM_DEFER_STORE 2 /* deferred writes: the storing round          */
#define ST_FORM_MFREE 3       /* the matrix-free round                        */
#define ST_FORM_ROWSUM 4      /* K0, the initial row-sum pass                 */
#define ST_KERNEL_ROUND 0     /* k_round: grid-stride row groups              */
#define ST_KERNEL_FLAT 1      /* k_flat + k_parts, storing every round        */
#define ST_KERNEL_FLAT_DEFERRED 2 /* k_flat<NP> + k_parts                     */
#define ST_KERNEL_MFREE 3     /* k_mfree                                      */
#define ST_KERNEL_FUSED 4     /* k_fused: grid-stride row groups, sums only    */
#define ST_KERNEL_FLAT_SUM 5  /* k_flat_sum + k_parts                         */
typedef struct st_launch_policy
{
  int kernel;               /* ST_KERNEL_*                                    */
  int rows;                 /* rows per workgroup (flat) or per row group     */
  unsigned int tile;        /* flat: row groups per piece tile, 0 = row-major */
  unsigned int cap;         /* workgroups per CU (dynamic LDS), 0 = uncapped  */
  unsigned int grid;        /* grid-stride kernels: workgroup count cap       */
  unsigned int piece_bytes; /* flat: bytes of a row per workgroup piece       */
  int load_nt;              /* matrix loads non-temporal                      */
  int store_nt;             /* matrix stores non-temporal, -1 = no stores     */
  int alt;                  /* odd rounds walk the block in reverse           */
} st_launch_policy;
int st_launch_policy_query(int dtype, unsigned int nrows, unsigned int ncols,
                           int form, unsigned int npend, st_launch_policy* out);

/* Round k of the flat round with deferred writes (what the solve loops run
 * for blocks where st_round_flat_pays): the matrix in d_mat is the last
 * STORED one, A_j; d_pend_s / d_pend_inv list the npend = k - j pending
 * rounds' gathered row sums s_j .. s_{k-1} and their reciprocals (oldest
 * first), which are re-applied in registers before round k's own update;
 * A_{k+1} is stored when `store`.  Every value (s_{k+1}, v, the state) is
 * bit-identical to st_round_flat on a matrix stored every round.  d_inv_cur
 * = 1 / d_s_cur; d_inv_next receives 1 / s_{k+1} for the block's rows (pass
 * the rank's slot, like d_s_next).  flush = 1 (with store = 1) only stores
 * A_{k+1} - no row sums, no v update - to leave the matrix as storing every
 * round would after the last round k.  npend < m = st_defer_rounds(nrows,
 * ncols, dtype), the rounds per store, and a round with npend = m - 1 (the
 * group's last) must store: other calls return -1.  d_pend_s / d_pend_inv
 * are HOST arrays of device pointers. */
int st_round_flat_deferred_f32(float* d_mat, const float* d_s_cur,
                               const float* d_inv_cur, float* d_s_next,
                               float* d_inv_next, float* d_part, float* d_v,
                               unsigned int nrows, unsigned int ncols,
                               unsigned int row0, float eps, unsigned int k,
                               unsigned int max_itr, unsigned int semantics,
                               const float* const* d_pend_s,
                               const float* const* d_pend_inv,
                               unsigned int npend, int store, int flush,
                               st_state* d_state, void* stream);
int st_round_flat_deferred_f64(double* d_mat, const double* d_s_cur,
                               const double* d_inv_cur, double* d_s_next,
                               double* d_inv_next, double* d_part,
                               double* d_v, unsigned int nrows,
                               unsigned int ncols, unsigned int row0,
                               double eps, unsigned int k,
                               unsigned int max_itr, unsigned int semantics,
                               const double* const* d_pend_s,
                               const double* const* d_pend_inv,
                               unsigned int npend, int store, int flush,
                               st_state* d_state, void* stream);
/* d_inv[i] = 1 / d_s[i], i < n (the reciprocals of s_0) */
int st_recip_f32(const float* d_s, float* d_inv, unsigned int n, void* stream);
int st_recip_f64(const double* d_s, double* d_inv, unsigned int n,
                 void* stream);
/* rounds per store of the deferred flat round on a block (dtype 0 = f32,
 * 1 = f64): 6 on every block (the arguments are kept for future shapes) */
unsigned int st_defer_rounds(unsigned int nrows, unsigned int ncols,
                             int dtype);

/* Round k split in two launches for a sharded solve that overlaps the
 * all-gather of s_k with compute (eigen_value_amd/sharded.py, overlap).
 * [col0, col1) are the columns whose s_k values this rank computed itself
 * (normally [row0, row0 + nrows)); d_part holds nrows partial row sums.
 *   span = 1 (local; d_s_cur needs only the own slot): for those columns
 *     A[r][c] <- A[r][c] * ((1/s_k[row0+r]) * s_k[c]), d_part[r] = their
 *     sum.  No m / stop / v / state work.
 *   span = 2 (remote; d_s_cur = the full gathered s_k): exactly st_round's
 *     m_k, stop_k, v update, lambda and state, plus the other columns, and
 *     d_s_next[r] = d_part[r] + (their row sum).
 * A_{k+1}, v, m and stop are bit-identical to st_round; s_{k+1} sums the
 * two column sets separately (bit-identical to st_round when the local
 * range is all columns).  Both launches are no-ops once a previous round
 * stopped. */
int st_round_split_f32(float* d_mat, const float* d_s_cur, float* d_s_next,
                       float* d_part, float* d_v, unsigned int nrows,
                       unsigned int ncols, unsigned int row0,
                       unsigned int col0, unsigned int col1, float eps,
                       unsigned int k, unsigned int max_itr,
                       unsigned int semantics, int span, st_state* d_state,
                       void* stream);
int st_round_split_f64(double* d_mat, const double* d_s_cur,
                       double* d_s_next, double* d_part, double* d_v,
                       unsigned int nrows, unsigned int ncols,
                       unsigned int row0, unsigned int col0,
                       unsigned int col1, double eps, unsigned int k,
                       unsigned int max_itr, unsigned int semantics, int span,
                       st_state* d_state, void* stream);

/* The same two halves in the flat form (st_round_flat), for blocks where
 * st_round_flat_pays: span 1 runs k_flat over the 4 KB column pieces that
 * hold [col0, col1), span 2 over all pieces with the other columns (plus
 * the m / stop / lambda / state work of k_flat's first row group), then
 * sums remote-then-local partials into d_s_next and updates v.  d_part:
 * scratch of st_round_split_flat_scratch(nrows, ncols, col0, col1)
 * elements, shared by the two halves of a round.  A_{k+1}, v, m and stop
 * are bit-identical to st_round_flat; s_{k+1} differs from it only in the
 * summation order. */
int st_round_split_flat_f32(float* d_mat, const float* d_s_cur,
                            float* d_s_next, float* d_part, float* d_v,
                            unsigned int nrows, unsigned int ncols,
                            unsigned int row0, unsigned int col0,
                            unsigned int col1, float eps, unsigned int k,
                            unsigned int max_itr, unsigned int semantics,
                            int span, st_state* d_state, void* stream);
int st_round_split_flat_f64(double* d_mat, const double* d_s_cur,
                            double* d_s_next, double* d_part, double* d_v,
                            unsigned int nrows, unsigned int ncols,
                            unsigned int row0, unsigned int col0,
                            unsigned int col1, double eps, unsigned int k,
                            unsigned int max_itr, unsigned int semantics,
                            int span, st_state* d_state, void* stream);
uint64_t st_round_split_flat_scratch(unsigned int nrows, unsigned int ncols,
                                     unsigned int col0, unsigned int col1);

/* Matrix-free round.  The transformed matrix of
 * round k is X^-1 A_0 X with x ∝ the product of all previous row-sum
 * vectors, so its row sums are (A_0 x) ⊘ x and A_0 never has to be
 * rewritten: N^2*b bytes per round instead of 2*N^2*b.  Launch k >= 1
 * (launch 0 is st_rowsum on A_0, giving s_0; v_prev = 1 for launch 1):
 *   from the FULL s_prev = s_{k-1}: m, stop, lambda of round k-1 (recorded
 *   in d_state, end = k when round k-1 stops or k == max_itr);
 *   d_v_cur[0..ncols) = d_v_prev * (s_prev / m)   (v_{k-1}, full vector);
 *   d_s_next[r] = (Σ_c A_0[r][c] x[c]) / x[row0+r], x = v_prev ∘ s_prev,
 *   for the local rows (s_k).
 * d_mat0 is read only.  v_prev/v_cur and s_prev/s_next are ping-pong
 * buffers.  Launches after the stopping one are no-ops. */
int st_mfree_round_f32(const float* d_mat0, const float* d_s_prev,
                       float* d_s_next, const float* d_v_prev, float* d_v_cur,
                       unsigned int nrows, unsigned int ncols,
                       unsigned int row0, float eps, unsigned int k,
                       unsigned int max_itr, unsigned int semantics,
                       st_state* d_state, void* stream);
int st_mfree_round_f64(const double* d_mat0, const double* d_s_prev,
                       double* d_s_next, const double* d_v_prev,
                       double* d_v_cur, unsigned int nrows, unsigned int ncols,
                       unsigned int row0, double eps, unsigned int k,
                       unsigned int max_itr, unsigned int semantics,
                       st_state* d_state, void* stream);
/* The same matrix-free launch k in the flat form (the solve loops' choice
 * for blocks where st_round_flat_pays): one short workgroup per (rows, 4 or
 * 8 KB column piece) writes partial dot products into d_part
 * (st_round_flat_scratch(nrows, ncols) elements), a second launch sums them
 * per row and writes v_{k-1}.  Results equal st_mfree_round_* up to the
 * association of the row sums (pieces summed apart; deterministic and
 * independent of the row partition). */
int st_mfree_round_flat_f32(const float* d_mat0, const float* d_s_prev,
                            float* d_s_next, const float* d_v_prev,
                            float* d_v_cur, float* d_part, unsigned int nrows,
                            unsigned int ncols, unsigned int row0, float eps,
                            unsigned int k, unsigned int max_itr,
                            unsigned int semantics, st_state* d_state,
                            void* stream);
int st_mfree_round_flat_f64(const double* d_mat0, const double* d_s_prev,
                            double* d_s_next, const double* d_v_prev,
                            double* d_v_cur, double* d_part, unsigned int nrows,
                            unsigned int ncols, unsigned int row0, double eps,
                            unsigned int k, unsigned int max_itr,
                            unsigned int semantics, st_state* d_state,
                            void* stream);

/* Round epilogue on the full row-sum vector s[0..n): m = max(0, max s)
 * (find_max, similarity_transform.cpp:154-227), v[i] *= s[i]/m
 * (compute_eigen_vector, :229-265), stop = all |s[i]-s[i+1]| < eps over
 * the cyclic (ST_SEM_SYCL, :332-460) or open (ST_SEM_MAINPY) pairs,
 * lambda = s[0]; then done/round/iters bookkeeping against max_itr.
 * No-op once done != 0.  d_v may be NULL (no eigenvector update). */
int st_epilogue_f32(const float* d_s, float* d_v, unsigned int n, float eps,
                    unsigned int max_itr, unsigned int semantics,
                    st_state* d_state, void* stream);
int st_epilogue_f64(const double* d_s, double* d_v, unsigned int n,
                    double eps, unsigned int max_itr, unsigned int semantics,
                    st_state* d_state, void* stream);

/* Library / device facts.  st_version names the library, the target, the
 * A/B probe switches its kernels were built with ("defaults" in every
 * library build; st_probe_switches returns that part alone) and the RCCL
 * its calls are bound to (st_rccl_version). */
const char* st_version(void);
const char* st_probe_switches(void);
int st_device_count(void);

#ifdef __cplusplus
} /* extern "C" */
#endif

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
/* C++ entry mirroring include/similarity_transform.hpp:46-53
 * (int64_t similarity_transform(sycl::queue&, const float* mat, float*
 * eigen_val, float* eigen_vec, uint dim, uint wg_size, uint* iter_count)).
 * The queue becomes the opaque context; wg_size is accepted and ignored
 * (tiles are chosen by the kernels). */
inline int64_t
similarity_transform(void* q, const float* mat, float* const eigen_val,
                     float* const eigen_vec, const unsigned int dim,
                     const unsigned int /*wg_size*/,
                     unsigned int* const iter_count)
{
  return max_eigen_value_ex(q, 0, mat, eigen_val, eigen_vec, dim, iter_count,
                            nullptr, nullptr);
}
inline int64_t
similarity_transform(void* q, const double* mat, double* const eigen_val,
                     double* const eigen_vec, const unsigned int dim,
                     const unsigned int /*wg_size*/,
                     unsigned int* const iter_count)
{
  return max_eigen_value_ex(q, 1, mat, eigen_val, eigen_vec, dim, iter_count,
                            nullptr, nullptr);
}
#endif

#endif /* EIGEN_VALUE_AMD_SIMILARITY_TRANSFORM_H */
