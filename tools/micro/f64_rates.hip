// Microbenchmark: FP64 MFMA (v_mfma_f64_16x16x4_f64) vs FP64 VALU FMA throughput on one
// MI355X, all CUs busy.  Informs the bootstrap kernel's design.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_mfma(double* out, int iters, double a0, double b0) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = a0 + threadIdx.x, b = b0 - threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}

__global__ __launch_bounds__(256) void k_valu(double* out, int iters, double a0, double b0) {
  double c[8];
  for (int j = 0; j < 8; ++j) c[j] = j;
  double a = a0 + threadIdx.x, b = b0 - threadIdx.x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(a, b, c[j]);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  hipMalloc(&out, sizeof(double) * 256 * 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double fma_mfma = (double)blocks * 4 /*waves*/ * iters * 4 * 1024;
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0, 2.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms2;
    hipEventElapsedTime(&ms2, e0, e1);
    const double fma_valu = (double)blocks * 256 * iters * 8;
    printf("mfma f64: %.3f ms  %.1f TFLOP/s   valu f64 fma: %.3f ms  %.1f TFLOP/s\n", ms,
           2 * fma_mfma / ms / 1e9, ms2, 2 * fma_valu / ms2 / 1e9);
  }
  return 0;
}
