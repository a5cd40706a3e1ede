// Microbenchmark: can FP64 MFMA (v_mfma_f64_16x16x4_f64) and FP64 VALU FMA run
// concurrently on one SIMD?  Each wave issues 4 independent MFMA chains and NV
// independent VALU FMA chains per iteration; the combined FP64 rate against the two
// pure rates tells whether a bootstrap kernel could split boots between the units.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NM, int NV>
__global__ __launch_bounds__(256) void k_mix(double* out, int iters, double a0, double b0) {
  d4 c[NM > 0 ? NM : 1];
  for (int j = 0; j < (NM > 0 ? NM : 1); ++j) c[j] = d4{0, 0, 0, 0};
  double v[NV > 0 ? NV : 1];
  for (int j = 0; j < (NV > 0 ? NV : 1); ++j) v[j] = j;
  double a = a0 + threadIdx.x, b = b0 - threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NM; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = fma(a, b, v[j]);
  }
  double s = 0;
  for (int j = 0; j < NM; ++j) s += c[j][0] + c[j][3];
  for (int j = 0; j < NV; ++j) s += v[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NM, int NV>
void run(double* out) {
  const int blocks = 256 * 8, iters = 2000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_mix<NM, NV>), dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  const double waves = (double)blocks * 4;
  const double fm = waves * iters * NM * 1024.0, fv = waves * 64.0 * iters * NV;
  printf("NM=%d NV=%2d: %.3f ms  mfma %.1f + valu %.1f = %.1f TFLOP/s\n", NM, NV, ms, 2 * fm / ms / 1e9,
         2 * fv / ms / 1e9, 2 * (fm + fv) / ms / 1e9);
}

int main() {
  double* out;
  hipMalloc(&out, sizeof(double) * 256 * 4096);
  run<4, 0>(out);
  run<8, 0>(out);
  run<0, 16>(out);
  run<4, 4>(out);
  run<4, 8>(out);
  run<4, 16>(out);
  run<4, 32>(out);
  run<2, 16>(out);
  return 0;
}
