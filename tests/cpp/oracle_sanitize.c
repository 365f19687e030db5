/*
 * oracle_sanitize.c — the CPU oracle (oracle/st_oracle.c) under
 * AddressSanitizer + UndefinedBehaviorSanitizer (a CPU
 * sanitizer run of the checker).  Test infrastructure: built and run by
 * tests/test_oracle.py::test_oracle_under_sanitizers with
 *   gcc -fsanitize=address,undefined -fno-sanitize-recover=all -fopenmp
 *       tests/cpp/oracle_sanitize.c oracle/st_oracle.c
 * It exercises every entry point the tests use, at sizes that cross the
 * oracle's internal boundaries (the 128-element pairwise leaves, the
 * 8192-element numpy buffer, ragged rows, one-element and 3x3 inputs, the
 * streaming solve's row chunks), and checks the 3x3 known answer of the
 * reference's tests/test.cpp:99-102 and the README.md:70 round count.
 * Exit 0 = clean; any sanitizer report aborts with a non-zero status.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void orc_hilbert_f64(double*, uint32_t, uint32_t, uint32_t);
void orc_hilbert_f32(float*, uint32_t, uint32_t, uint32_t);
void orc_random_f64(double*, uint32_t, uint32_t, uint32_t, uint64_t);
void orc_random_f32(float*, uint32_t, uint32_t, uint32_t, uint64_t);
void orc_rowsum_f64(const double*, double*, uint32_t, uint32_t);
double orc_find_max_f64(const double*, uint32_t);
int orc_stop_f64(const double*, uint32_t, double, int);
void orc_compute_next_f64(double*, const double*, uint32_t, uint32_t, uint32_t, int);
int orc_similarity_transform_f64(const double*, uint32_t, double, uint32_t, int, int,
                                 double*, double*, uint32_t*, double*, double*, uint32_t*);
int orc_similarity_transform_f32(const float*, uint32_t, float, uint32_t, int, int,
                                 float*, float*, uint32_t*, double*, double*, uint32_t*);
int orc_similarity_transform_gen_f64(int, uint64_t, uint32_t, double, uint32_t, int, int,
                                     uint32_t, double*, double*, uint32_t*, double*,
                                     uint32_t*);

static int fails = 0;
#define CHECK(c)                                                                 \
  do {                                                                           \
    if (!(c)) {                                                                  \
      fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #c);     \
      fails++;                                                                   \
    }                                                                            \
  } while (0)

static void
solve_sizes(void)
{
  /* pairwise leaf (128), numpy buffer (8192) and ragged boundaries */
  static const uint32_t ns[] = { 1, 2, 3, 127, 128, 129, 257, 1000 };
  for (size_t i = 0; i < sizeof ns / sizeof ns[0]; i++) {
    const uint32_t n = ns[i];
    double* a = malloc(sizeof(double) * n * n);
    float* af = malloc(sizeof(float) * n * n);
    double* v = malloc(sizeof(double) * n);
    float* vf = malloc(sizeof(float) * n);
    double dsum[1000];
    double lam = 0, ms = 0;
    float lamf = 0;
    uint32_t it = 0, rounds = 0;
    orc_random_f64(a, n, n, 0, 7);
    orc_random_f32(af, n, n, 0, 7);
    for (int sem = 0; sem < 2; sem++) {
      CHECK(orc_similarity_transform_f64(a, n, 1e-3, 1000, sem, 2, &lam, v, &it, dsum, &ms,
                                         &rounds) == 0);
      CHECK(lam > 0 && rounds >= 1 && (it >= 1 || (n == 1 && sem == 0)));
      CHECK(orc_similarity_transform_f32(af, n, 1e-3f, 30, sem, 2, &lamf, vf, &it, NULL,
                                         NULL, NULL) == 0);
    }
    orc_hilbert_f64(a, n, n, 0);
    CHECK(orc_similarity_transform_f64(a, n, 1e-3, 1000, 0, 1, &lam, v, &it, NULL, NULL,
                                       NULL) == 0);
    free(a);
    free(af);
    free(v);
    free(vf);
  }
}

static void
long_rows(void)
{
  /* row sums across the 8192-element buffer boundary, ragged tails */
  const uint32_t nr = 3, nc = 8192 * 2 + 77;
  double* m = malloc(sizeof(double) * nr * nc);
  double s[3], full[8192 * 2 + 77];
  orc_random_f64(m, nr, nc, 5, 11);
  orc_rowsum_f64(m, s, nr, nc);
  for (uint32_t c = 0; c < nc; c++)
    full[c] = 1.0 + (double)c / nc;
  orc_compute_next_f64(m, full, nr, nc, 0, 0);
  orc_compute_next_f64(m, full, nr, nc, 0, 1);
  CHECK(orc_find_max_f64(s, 3) > 0);
  CHECK(orc_stop_f64(s, 3, 1e300, 1) == 1);
  free(m);
}

static void
known_answers(void)
{
  /* tests/test.cpp:84-102 of the reference: the 3x3 matrix
     {1,1,2; 2,1,3; 2,3,5} gives 7.53114 and v = (0.394074, 0.578844,
     0.997451) within EPS = 1e-3 (fp32, SYCL semantics) */
  float b[9] = { 1, 1, 2, 2, 1, 3, 2, 3, 5 }, vb[3], lamb = 0;
  uint32_t it = 0;
  CHECK(orc_similarity_transform_f32(b, 3, 1e-3f, 1000, 0, 1, &lamb, vb, &it, NULL, NULL,
                                     NULL) == 0);
  CHECK(fabsf(lamb - 7.53114f) < 1e-3f);
  CHECK(fabsf(vb[0] - 0.394074f) < 1e-3f && fabsf(vb[1] - 0.578844f) < 1e-3f &&
        fabsf(vb[2] - 0.997451f) < 1e-3f);
  /* README.md:70: Hilbert 128 fp32 stops after 9 rounds */
  float* h = malloc(sizeof(float) * 128 * 128);
  float* vf = malloc(sizeof(float) * 128);
  float lamf = 0;
  orc_hilbert_f32(h, 128, 128, 0);
  CHECK(orc_similarity_transform_f32(h, 128, 1e-3f, 1000, 0, 1, &lamf, vf, &it, NULL, NULL,
                                     NULL) == 0);
  CHECK(it == 9);
  free(h);
  free(vf);
}

static void
streaming(void)
{
  /* the generated (streaming) solve in chunks that do not divide n, against
     the plain loop on the same matrix: bit-identical */
  const uint32_t n = 301;
  double* a = malloc(sizeof(double) * n * n);
  double *v1 = malloc(sizeof(double) * n), *v2 = malloc(sizeof(double) * n);
  double l1 = 0, l2 = 0;
  uint32_t i1 = 0, i2 = 0;
  orc_random_f64(a, n, n, 0, 3);
  CHECK(orc_similarity_transform_f64(a, n, 1e-3, 1000, 0, 2, &l1, v1, &i1, NULL, NULL,
                                     NULL) == 0);
  CHECK(orc_similarity_transform_gen_f64(2, 3, n, 1e-3, 1000, 0, 2, 37, &l2, v2, &i2, NULL,
                                         NULL) == 0);
  CHECK(l1 == l2 && i1 == i2);
  for (uint32_t r = 0; r < n; r++)
    CHECK(v1[r] == v2[r]);
  /* argument errors are refused, not read past */
  CHECK(orc_similarity_transform_gen_f64(3, 0, n, 1e-3, 10, 0, 1, 0, &l2, v2, &i2, NULL,
                                         NULL) == -1);
  CHECK(orc_similarity_transform_f64(NULL, n, 1e-3, 10, 0, 1, &l2, v2, &i2, NULL, NULL,
                                     NULL) == -1);
  free(a);
  free(v1);
  free(v2);
}

int
main(void)
{
  solve_sizes();
  long_rows();
  known_answers();
  streaming();
  if (fails) {
    fprintf(stderr, "%d checks failed\n", fails);
    return 1;
  }
  printf("oracle clean under ASan/UBSan\n");
  return 0;
}
