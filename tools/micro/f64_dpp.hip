// Microbenchmark: FP64 FMA issue rates for the bootstrap's multiplicity operand, all CUs busy.
//   valu : v_fmac_f64, every operand a VGPR (the ceiling)
//   sgpr : the multiplicity as an SGPR operand (k_boot2 / k_boot_tiles today)
//   dpp  : the multiplicity broadcast from a VGPR lane of each 16-lane row (row_newbcast:j,
//          DPP64, gfx90a+), i.e. the operand comes from a vector load instead of s_load
// Each wave runs 16 independent accumulator chains (one per broadcast lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"

template <int J>
__device__ __forceinline__ double bcast(double w) {
  return __builtin_amdgcn_update_dpp(0.0, w, 0x150 + J, 0xf, 0xf, false);
}

template <int J>
__device__ __forceinline__ void fmac_bcast(double& acc, double w, double x) {
  // acc += (lane J of w's 16-lane row) * x; DPP64 reads src0 from the row's lane J
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(w), "v"(x), "n"(J));
}

__global__ __launch_bounds__(256) void k_dppasm(double* out, int iters, double a0) {
  double c[16];
  for (int j = 0; j < 16; ++j) c[j] = j;
  const double x = a0 + threadIdx.x;
  double w = a0 * (threadIdx.x & 15);
  asm volatile("s_nop 4" : "+v"(w));  // w's VALU write clears the DPP read hazard
#define STEPA(J) fmac_bcast<J>(c[J], w, x);
  for (int i = 0; i < iters; ++i) {
    STEPA(0) STEPA(1) STEPA(2) STEPA(3) STEPA(4) STEPA(5) STEPA(6) STEPA(7)
    STEPA(8) STEPA(9) STEPA(10) STEPA(11) STEPA(12) STEPA(13) STEPA(14) STEPA(15)
  }
  double s = 0;
  for (int j = 0; j < 16; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_valu(double* out, int iters, double a0) {
  double c[16];
  for (int j = 0; j < 16; ++j) c[j] = j;
  const double x = a0 + threadIdx.x;
  double w[16];
  for (int j = 0; j < 16; ++j) w[j] = a0 * j;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < 16; ++j) c[j] = fma(w[j], x, c[j]);
  }
  double s = 0;
  for (int j = 0; j < 16; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_sgpr(double* out, const double* __restrict__ W, int iters, double a0) {
  double c[16];
  for (int j = 0; j < 16; ++j) c[j] = j;
  const double x = a0 + threadIdx.x;
  for (int i = 0; i < iters; ++i) {
    const double* __restrict__ wp = W + (i & 63) * 16;
#pragma unroll
    for (int j = 0; j < 16; ++j) c[j] = fma(wp[j], x, c[j]);
  }
  double s = 0;
  for (int j = 0; j < 16; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_dpp(double* out, int iters, double a0) {
  double c[16];
  for (int j = 0; j < 16; ++j) c[j] = j;
  const double x = a0 + threadIdx.x;
  const double w = a0 * (threadIdx.x & 15);
#define STEP(J) c[J] = fma(bcast<J>(w), x, c[J]);
  for (int i = 0; i < iters; ++i) {
    STEP(0) STEP(1) STEP(2) STEP(3) STEP(4) STEP(5) STEP(6) STEP(7)
    STEP(8) STEP(9) STEP(10) STEP(11) STEP(12) STEP(13) STEP(14) STEP(15)
  }
  double s = 0;
  for (int j = 0; j < 16; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double *out, *W;
  hipMalloc(&out, sizeof(double) * 256 * 4096);
  hipMalloc(&W, sizeof(double) * 64 * 16);
  hipMemset(W, 0, sizeof(double) * 64 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * 8, iters = 2000;
  const double fmas = (double)blocks * 256 * iters * 16;
  for (int rep = 0; rep < 2; ++rep) {
    float ms[4];
    for (int k = 0; k < 4; ++k) {
      hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0);
      if (k == 1) hipLaunchKernelGGL(k_sgpr, dim3(blocks), dim3(256), 0, 0, out, W, iters, 1.0);
      if (k == 2) hipLaunchKernelGGL(k_dpp, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0);
      if (k == 3) hipLaunchKernelGGL(k_dppasm, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[k], e0, e1);
    }
    printf("f64 fma TFLOP/s: valu %.1f  sgpr-operand %.1f  mov_dpp+fma %.1f  fmac_dpp %.1f\n",
           2 * fmas / ms[0] / 1e9, 2 * fmas / ms[1] / 1e9, 2 * fmas / ms[2] / 1e9, 2 * fmas / ms[3] / 1e9);
  }
  return 0;
}
