// Host -> device upload of an int32 count matrix as 16-bit counts (GPU box):
//   hipcc --offload-arch=gfx950 -O3 -o tools/micro/h2d_u16 tools/micro/h2d_u16.hip -lpthread
//   ./tools/micro/h2d_u16 [MB of int32 counts, default 240 = config 4]
// 1. pageable hipMemcpyAsync of the int32 matrix (what the host-count entries do)
// 2. a persistent pool of T threads narrows each slot's int32 counts to uint16 into a pinned
//    ring slot (range-checked), the slot's DMA goes up, a widening kernel writes the int32
//    counts on the device behind it; slots of S MB of int32 source, 4 slots in the ring
// The end-to-end time is from the first narrowing to the last widening kernel's completion.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
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

__global__ void k_widen(const uint16_t* __restrict__ in, int* __restrict__ out, size_t n) {
  const size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const ushort4 v = *reinterpret_cast<const ushort4*>(in + i);
    *reinterpret_cast<int4*>(out + i) = make_int4(v.x, v.y, v.z, v.w);
  } else {
    for (size_t j = i; j < n; ++j) out[j] = in[j];
  }
}

// persistent narrowing pool: job = (src, dst, n); thread t takes share t of T
struct Pool {
  int T;
  std::vector<std::thread> th;
  std::atomic<long long> gen{0};
  std::atomic<int> done{0};
  std::atomic<bool> stop{false};
  const int* src = nullptr;
  uint16_t* dst = nullptr;
  size_t n = 0;
  std::atomic<unsigned> bad{0};
  static unsigned narrow(const int* s, uint16_t* d, size_t n) {
    unsigned b = 0;
    for (size_t i = 0; i < n; ++i) {
      const unsigned v = (unsigned)s[i];
      b |= v >> 16;
      d[i] = (uint16_t)v;
    }
    return b;
  }
  void share(int t) {
    const size_t a = (n * t / T) & ~size_t(15), e = (t + 1 == T) ? n : ((n * (t + 1) / T) & ~size_t(15));
    if (e > a) bad.fetch_or(narrow(src + a, dst + a, e - a));
  }
  explicit Pool(int T_) : T(T_) {
    for (int t = 1; t < T; ++t)
      th.emplace_back([this, t] {
        long long seen = 0;
        for (;;) {
          long long g;
          while ((g = gen.load(std::memory_order_acquire)) == seen && !stop.load()) {
          }
          if (stop.load()) return;
          seen = g;
          share(t);
          done.fetch_add(1, std::memory_order_acq_rel);
        }
      });
  }
  unsigned run(const int* s, uint16_t* d, size_t nn) {
    src = s;
    dst = d;
    n = nn;
    bad = 0;
    done = 0;
    gen.fetch_add(1, std::memory_order_acq_rel);
    share(0);
    while (done.load(std::memory_order_acquire) != T - 1) {
    }
    return bad.load();
  }
  ~Pool() {
    stop = true;
    for (auto& x : th) x.join();
  }
};

int main(int argc, char** argv) {
  const size_t mb = argc > 1 ? std::atoi(argv[1]) : 240;
  const size_t n = (mb << 20) / 4;  // counts
  std::vector<int> src(n);
  for (size_t i = 0; i < n; ++i) src[i] = (int)((i * 2654435761u) >> 27) % 9 == 0 ? (int)(i % 300) : 0;
  int* dev = nullptr;
  uint16_t* dev16 = nullptr;
  CK(hipMalloc(&dev, n * 4));
  CK(hipMalloc(&dev16, n * 2));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  constexpr int kSlots = 4;
  const size_t kMaxSlot = size_t(16) << 20;  // bytes of uint16 per slot at most
  uint16_t* pin = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pin), kSlots * kMaxSlot, hipHostMallocDefault));
  hipEvent_t ev[kSlots];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  std::vector<int> back(n);
  for (int rep = 0; rep < 3; ++rep) {
    auto t0 = clk::now();
    CK(hipMemcpyAsync(dev, src.data(), n * 4, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    auto t1 = clk::now();
    std::printf("rep %d pageable int32: %.3f ms (%.1f GB/s of int32)\n", rep, ms(t0, t1), n * 4 / ms(t0, t1) / 1e6);
    for (int T : {4, 8, 12, 16}) {
      Pool pool(T);
      for (size_t slot_mb : {2, 4, 8, 16}) {
        const size_t per = std::min(kMaxSlot / 2, (slot_mb << 20) / 4);  // counts per slot
        bool used[kSlots] = {};
        CK(hipMemsetAsync(dev, 0, n * 4, st));
        CK(hipStreamSynchronize(st));
        t0 = clk::now();
        unsigned bad = 0;
        int k = 0;
        for (size_t off = 0; off < n; off += per, k = (k + 1) % kSlots) {
          const size_t m = std::min(per, n - off);
          if (used[k]) CK(hipEventSynchronize(ev[k]));
          uint16_t* slot = pin + (size_t)k * (kMaxSlot / 2);
          bad |= pool.run(src.data() + off, slot, m);
          CK(hipMemcpyAsync(dev16 + off, slot, m * 2, hipMemcpyHostToDevice, st));
          CK(hipEventRecord(ev[k], st));
          used[k] = true;
          hipLaunchKernelGGL(k_widen, dim3((unsigned)((m / 4 + 255) / 256 + 1)), dim3(256), 0, st, dev16 + off,
                             dev + off, m);
        }
        t1 = clk::now();
        CK(hipStreamSynchronize(st));
        auto t2 = clk::now();
        std::printf("rep %d u16 T=%2d slot %2zu MB: host %.3f ms, done %.3f ms (%.1f GB/s of int32)%s\n", rep, T,
                    slot_mb, ms(t0, t1), ms(t0, t2), n * 4 / ms(t0, t2) / 1e6, bad ? " [out of range]" : "");
        if (rep == 0 && T == 8 && slot_mb == 4) {
          CK(hipMemcpy(back.data(), dev, n * 4, hipMemcpyDeviceToHost));
          std::printf("  round trip %s\n", std::memcmp(back.data(), src.data(), n * 4) ? "MISMATCH" : "ok");
        }
      }
    }
  }
  return 0;
}
