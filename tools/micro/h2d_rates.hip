// Host -> device upload rates for an 80 MB count matrix (config 3), GPU box:
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/h2d_rates tools/micro/h2d_rates.hip -lpthread
//   ./tools/micro/h2d_rates [MB]
// 1. pageable hipMemcpyAsync (what the host-count entries do): host-blocking time, completion
// 2. pinned staging: one-thread memcpy into a pinned buffer, then the DMA
// 3. pinned staging with T threads copying in parallel
// 4. pipelined: K pieces, T threads copy piece j while piece j-1's DMA runs
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

static void par_copy(char* dst, const char* src, size_t n, int T) {
  std::vector<std::thread> th;
  const size_t chunk = (n + T - 1) / T;
  for (int t = 0; t < T; ++t) {
    const size_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) th.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::atoi(argv[1]) : 80;
  const size_t n = mb << 20;
  char* src = static_cast<char*>(std::malloc(n));
  for (size_t i = 0; i < n; ++i) src[i] = (char)(i * 7);
  void* dev = nullptr;
  CK(hipMalloc(&dev, n));
  char* pin = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pin), n, hipHostMallocDefault));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  for (int rep = 0; rep < 3; ++rep) {
    // 1. pageable
    auto t0 = clk::now();
    CK(hipMemcpyAsync(dev, src, n, hipMemcpyHostToDevice, st));
    auto t1 = clk::now();
    CK(hipStreamSynchronize(st));
    auto t2 = clk::now();
    std::printf("rep %d pageable: call returns %.3f ms, done %.3f ms (%.1f GB/s)\n", rep, ms(t0, t1), ms(t0, t2),
                n / ms(t0, t2) / 1e6);
    // 2. pinned DMA alone
    t0 = clk::now();
    CK(hipMemcpyAsync(dev, pin, n, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    t1 = clk::now();
    std::printf("rep %d pinned DMA: %.3f ms (%.1f GB/s)\n", rep, ms(t0, t1), n / ms(t0, t1) / 1e6);
    // 3. host copies into pinned
    for (int T : {1, 4, 8, 16}) {
      t0 = clk::now();
      par_copy(pin, src, n, T);
      t1 = clk::now();
      std::printf("rep %d memcpy to pinned, %2d threads: %.3f ms (%.1f GB/s)\n", rep, T, ms(t0, t1),
                  n / ms(t0, t1) / 1e6);
    }
    // 4. pipelined pieces
    for (int K : {4, 8, 16}) {
      for (int T : {4, 8}) {
        t0 = clk::now();
        const size_t piece = (n + K - 1) / K;
        for (int j = 0; j < K; ++j) {
          const size_t lo = j * piece, len = std::min(n, lo + piece) - lo;
          par_copy(pin + lo, src + lo, len, T);
          CK(hipMemcpyAsync(static_cast<char*>(dev) + lo, pin + lo, len, hipMemcpyHostToDevice, st));
        }
        t1 = clk::now();
        CK(hipStreamSynchronize(st));
        t2 = clk::now();
        std::printf("rep %d pipelined K=%2d T=%d: host %.3f ms, done %.3f ms (%.1f GB/s)\n", rep, K, T, ms(t0, t1),
                    ms(t0, t2), n / ms(t0, t2) / 1e6);
      }
    }
  }
  return 0;
}
