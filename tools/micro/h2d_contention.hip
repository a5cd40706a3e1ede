// Does a pageable host -> device copy issued from one thread stall while another thread of the
// same process launches small kernels and waits for them (the host-count entry: the upload
// thread's pieces against the caller's unique-set builds and their host syncs)?  GPU box:
//   hipcc --offload-arch=gfx950 -O2 -o tools/micro/h2d_contention tools/micro/h2d_contention.hip -lpthread
//   ./tools/micro/h2d_contention
// The uploader copies 8 x 10 MB pageable pieces back to back on its own stream; meanwhile the
// main thread runs one of: nothing; kernel + small D2H + hipStreamSynchronize loops; the same
// with hipEventSynchronize; with a hipEventQuery spin; kernel launches only.  Reported: the
// uploader's wall time for the 80 MB and its slowest piece.
#include <hip/hip_runtime.h>

#include <atomic>
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

__global__ void tiny(int* p, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 3 + 1;
}

static void par_copy(char* dst, const char* src, size_t n, int T) {
  std::vector<std::thread> th;
  const size_t chunk = (n + T - 1) / T;
  for (int t = 0; t < T; ++t) {
    const size_t lo = t * chunk, hi = std::min(n, lo + chunk);
    if (lo < hi) th.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
  }
  for (auto& x : th) x.join();
}

int main() {
  const int K = 8;
  const size_t piece = size_t(10) << 20, n = K * piece;
  char* src = static_cast<char*>(std::malloc(n));
  for (size_t i = 0; i < n; ++i) src[i] = (char)(i * 7);
  void* dev = nullptr;
  CK(hipMalloc(&dev, n));
  int* work = nullptr;
  CK(hipMalloc(&work, sizeof(int) * 65536));
  int* land = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&land), 4096, hipHostMallocDefault));
  char* pin = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pin), n, hipHostMallocDefault));
  hipStream_t su, sm;
  CK(hipStreamCreateWithFlags(&su, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sm, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const char* names[] = {"idle", "kernel+d2h+streamsync", "kernel+d2h+eventsync", "kernel+d2h+eventquery spin",
                         "kernel launches only"};
  for (int rep = 0; rep < 2; ++rep)
    for (int mode = 0; mode < 5; ++mode)
      for (int up = 0; up < 2; ++up) {  // 0: pageable pieces, 1: 8-thread copy into pinned + DMA per piece
        CK(hipDeviceSynchronize());
        std::atomic<bool> done{false};
        double worst = 0, total = 0;
        std::thread uth([&] {
          auto t0 = clk::now();
          for (int j = 0; j < K; ++j) {
            auto a = clk::now();
            if (up == 0) {
              CK(hipMemcpyAsync((char*)dev + j * piece, src + j * piece, piece, hipMemcpyHostToDevice, su));
            } else {
              par_copy(pin + j * piece, src + j * piece, piece, 8);
              CK(hipMemcpyAsync((char*)dev + j * piece, pin + j * piece, piece, hipMemcpyHostToDevice, su));
            }
            auto b = clk::now();
            worst = std::max(worst, ms(a, b));
          }
          CK(hipStreamSynchronize(su));
          total = ms(t0, clk::now());
          done = true;
        });
        int loops = 0;
        while (!done) {
          if (mode == 0) {
            std::this_thread::sleep_for(std::chrono::microseconds(20));
            continue;
          }
          hipLaunchKernelGGL(tiny, dim3(256), dim3(256), 0, sm, work, 65536);
          if (mode == 4) {
            if (++loops % 64 == 0) CK(hipStreamSynchronize(sm));
            continue;
          }
          CK(hipMemcpyAsync(land, work, 256, hipMemcpyDeviceToHost, sm));
          if (mode == 1) CK(hipStreamSynchronize(sm));
          if (mode == 2) {
            CK(hipEventRecord(ev, sm));
            CK(hipEventSynchronize(ev));
          }
          if (mode == 3) {
            CK(hipEventRecord(ev, sm));
            while (hipEventQuery(ev) == hipErrorNotReady) {
            }
          }
          ++loops;
        }
        uth.join();
        CK(hipStreamSynchronize(sm));
        std::printf("rep %d main=%-28s upload=%s: 80 MB in %.3f ms (%.1f GB/s), slowest piece call %.3f ms, main loops %d\n",
                    rep, names[mode], up ? "pinned8" : "pageable", total, n / total / 1e6, worst, loops);
      }
  return 0;
}
