// h2d_probe.cpp — the input path of the drop-in call:
// how fast can a caller's PAGEABLE host matrix reach HBM, and does pinning
// or chunking pay for a single call?
//   pageable   one hipMemcpyAsync from the caller's buffer (what
//              max_eigen_value does)
//   chunked    the same in 16 / 64 MiB pieces (lets a K0 row-sum pass run on
//              landed rows while later rows are still being staged)
//   register   hipHostRegister the caller's buffer, copy, unregister
//              (pinning cost included: a one-shot call pays it)
//   pinned     copy from an already pinned buffer (the PCIe ceiling)
//
// Build: make -C tools h2d_probe    Run: ./tools/h2d_probe [MiB...]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIPCHECK(x)                                                            \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,           \
                   hipGetErrorString(e));                                      \
      std::exit(2);                                                            \
    }                                                                          \
  } while (0)

template <typename F>
static double
best_ms(F f, int reps = 5)
{
  double best = 1e30;
  for (int r = 0; r < reps; r++) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    const double ms = std::chrono::duration<double, std::milli>(
                        std::chrono::steady_clock::now() - t0)
                        .count();
    best = ms < best ? ms : best;
  }
  return best;
}

int
main(int argc, char** argv)
{
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; i++)
    sizes.push_back((size_t)std::atoll(argv[i]));
  if (sizes.empty())
    sizes = { 64, 256, 512, 2048 };
  hipStream_t s;
  HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (size_t mib : sizes) {
    const size_t bytes = mib << 20;
    char* host = (char*)std::malloc(bytes);
    std::memset(host, 1, bytes); // touch every page
    char* pinned = nullptr;
    HIPCHECK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
    std::memset(pinned, 1, bytes);
    void* dev = nullptr;
    HIPCHECK(hipMalloc(&dev, bytes));
    auto rate = [&](double ms) { return bytes / (ms * 1e-3) / 1e9; };

    const double pageable = best_ms([&] {
      HIPCHECK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
      HIPCHECK(hipStreamSynchronize(s));
    });
    double chunked[2];
    const size_t pieces[2] = { (size_t)16 << 20, (size_t)64 << 20 };
    for (int c = 0; c < 2; c++)
      chunked[c] = best_ms([&] {
        for (size_t off = 0; off < bytes; off += pieces[c]) {
          const size_t len = bytes - off < pieces[c] ? bytes - off : pieces[c];
          HIPCHECK(hipMemcpyAsync((char*)dev + off, host + off, len,
                                  hipMemcpyHostToDevice, s));
        }
        HIPCHECK(hipStreamSynchronize(s));
      });
    const double reg = best_ms([&] {
      HIPCHECK(hipHostRegister(host, bytes, hipHostRegisterDefault));
      HIPCHECK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
      HIPCHECK(hipStreamSynchronize(s));
      HIPCHECK(hipHostUnregister(host));
    });
    const double pin = best_ms([&] {
      HIPCHECK(hipMemcpyAsync(dev, pinned, bytes, hipMemcpyHostToDevice, s));
      HIPCHECK(hipStreamSynchronize(s));
    });
    std::printf("%6zu MiB  pageable %8.3f ms %6.1f GB/s | chunked16 %8.3f ms "
                "%6.1f | chunked64 %8.3f ms %6.1f | register+copy %8.3f ms "
                "%6.1f | pinned %8.3f ms %6.1f GB/s\n",
                mib, pageable, rate(pageable), chunked[0], rate(chunked[0]),
                chunked[1], rate(chunked[1]), reg, rate(reg), pin, rate(pin));
    HIPCHECK(hipFree(dev));
    HIPCHECK(hipHostFree(pinned));
    std::free(host);
  }
  HIPCHECK(hipStreamDestroy(s));
  return 0;
}
