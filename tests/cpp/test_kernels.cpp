// test_kernels.cpp — C++ counterpart of the reference's tests/test.cpp
// (itzmeanjan/eigen_value tests/test.cpp:10-111): every kernel on synthetic
// buffers, then the 3x3 known answer through the C++ entry point.  Calls
// only the C-ABI of libsimilarity_transform.so (include/similarity_transform.h).
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "similarity_transform.h"

#define CHECK(x)                                                               \
  do {                                                                         \
    if (!(x)) {                                                                \
      std::fprintf(stderr, "FAILED %s:%d: %s (%s)\n", __FILE__, __LINE__, #x,  \
                   eigen_last_error());                                        \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

static const unsigned N = 1u << 10; // tests/test.cpp:7

int
main()
{
  CHECK(st_device_count() > 0);
  float *d_mat, *d_vec, *d_v;
  st_state* d_state;
  CHECK(hipMalloc(&d_mat, sizeof(float) * N * N) == hipSuccess);
  CHECK(hipMalloc(&d_vec, sizeof(float) * N) == hipSuccess);
  CHECK(hipMalloc(&d_v, sizeof(float) * N) == hipSuccess);
  CHECK(hipMalloc(&d_state, sizeof(st_state)) == hipSuccess);
  std::vector<float> vec(N), v(N);

  // sum across rows of the identity == 1 (test.cpp:22-30)
  CHECK(st_generate_identity_f32(d_mat, N, N, 0, nullptr) == 0);
  CHECK(st_rowsum_f32(d_mat, d_vec, N, N, nullptr) == 0);
  CHECK(hipMemcpy(vec.data(), d_vec, sizeof(float) * N, hipMemcpyDeviceToHost) == hipSuccess);
  for (unsigned i = 0; i < N; i++)
    CHECK(vec[i] == 1.f);
  std::printf("sum across row works !\n");

  // max of r+1 == N (test.cpp:32-41), eigenvector update (test.cpp:43-54)
  for (unsigned i = 0; i < N; i++)
    vec[i] = (float)(i + 1);
  CHECK(hipMemcpy(d_vec, vec.data(), sizeof(float) * N, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(st_fill_f32(d_v, N, 1.f, nullptr) == 0);
  CHECK(st_state_reset(d_state, nullptr) == 0);
  CHECK(st_epilogue_f32(d_vec, d_v, N, ST_EPS_F32, ST_MAX_ITR, ST_SEM_SYCL, d_state, nullptr) == 0);
  st_state h;
  CHECK(hipMemcpy(&h, d_state, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess);
  CHECK(h.max == (double)N);
  std::printf("max from vector works !\n");
  CHECK(hipMemcpy(v.data(), d_v, sizeof(float) * N, hipMemcpyDeviceToHost) == hipSuccess);
  float max_dev = 0.f;
  for (unsigned i = 0; i < N; i++)
    max_dev = std::fmax(max_dev, std::fabs(vec[i] / (float)N - v[i]));
  std::printf("maximum deviation in computing eigen vector %g\n", max_dev);
  CHECK(max_dev == 0.f);

  // stop criteria: success data 1 + 1e-4, fail data (r+1)*1e-4 (test.cpp:56-73)
  for (unsigned i = 0; i < N; i++)
    vec[i] = 1.f + 1e-4f;
  CHECK(hipMemcpy(d_vec, vec.data(), sizeof(float) * N, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(st_state_reset(d_state, nullptr) == 0);
  CHECK(st_epilogue_f32(d_vec, nullptr, N, ST_EPS_F32, ST_MAX_ITR, ST_SEM_SYCL, d_state, nullptr) == 0);
  CHECK(hipMemcpy(&h, d_state, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess);
  std::printf("stopping criteria test result [success]: %u\n", h.stop);
  CHECK(h.stop == 1);
  for (unsigned i = 0; i < N; i++)
    vec[i] = (float)(i + 1) * 1e-4f;
  CHECK(hipMemcpy(d_vec, vec.data(), sizeof(float) * N, hipMemcpyHostToDevice) == hipSuccess);
  CHECK(st_state_reset(d_state, nullptr) == 0);
  CHECK(st_epilogue_f32(d_vec, nullptr, N, ST_EPS_F32, ST_MAX_ITR, ST_SEM_SYCL, d_state, nullptr) == 0);
  CHECK(hipMemcpy(&h, d_state, sizeof(h), hipMemcpyDeviceToHost) == hipSuccess);
  std::printf("stopping criteria test result [fail]: %u\n", h.stop);
  CHECK(h.stop == 0);

  // 3x3 known answer through the C++ entry point (test.cpp:79-104)
  void* q = nullptr;
  make_queue(&q);
  CHECK(q != nullptr);
  const float mat[9] = { 1, 1, 2, 2, 1, 3, 2, 3, 5 };
  float eigen_val = 0.f, eigen_vec[3];
  unsigned iter_count = 0;
  int64_t ts = similarity_transform(q, mat, &eigen_val, eigen_vec, 3, 3, &iter_count);
  CHECK(ts >= 0);
  CHECK(std::fabs(eigen_val - 7.53114f) < ST_EPS_F32);
  CHECK(std::fabs(eigen_vec[0] - 0.394074f) < ST_EPS_F32);
  CHECK(std::fabs(eigen_vec[1] - 0.578844f) < ST_EPS_F32);
  CHECK(std::fabs(eigen_vec[2] - 0.997451f) < ST_EPS_F32);
  std::printf("similarity transform worked !\t\t[ %u iterations ]\t\t%lld ms\n",
              iter_count, (long long)ts);
  destroy_queue(q);
  (void)hipFree(d_mat);
  (void)hipFree(d_vec);
  (void)hipFree(d_v);
  (void)hipFree(d_state);
  return 0;
}
