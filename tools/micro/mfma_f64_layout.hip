// Checks the lane maps of v_mfma_f64_16x16x4_f64 with exact integer data (asymmetric B):
// A[i][k] = i + 100 k, B[k][j] = 7 j + 1000 k; lane l passes A[l&15][l>>4], B[l>>4][l&15]
// and reports where each C element lands, against C[i][j] = sum_k A[i][k] B[k][j].
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ void k(double* out) {
  const int l = threadIdx.x, r = l & 15, q = l >> 4;
  const double a = r + 100.0 * q, b = 7.0 * r + 1000.0 * q;
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int j = 0; j < 4; ++j) out[l * 4 + j] = c[j];
}
int main() {
  double* d;
  (void)hipMalloc(&d, 256 * sizeof(double));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[256];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int ok_a = 0, ok_b = 0;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 4; ++j) {
      // hypothesis A: col = l & 15, row = (l >> 4) + 4 j; hypothesis B: row = l & 15, col = ...
      auto C = [](int i, int jj) { double s = 0; for (int kk = 0; kk < 4; ++kk) s += (i + 100.0 * kk) * (7.0 * jj + 1000.0 * kk); return s; };
      if (h[l * 4 + j] == C((l >> 4) + 4 * j, l & 15)) ok_a++;
      if (h[l * 4 + j] == C(l & 15, (l >> 4) + 4 * j)) ok_b++;
    }
  printf("col=lane&15,row=(lane>>4)+4j: %d/256   row=lane&15,col=(lane>>4)+4j: %d/256\n", ok_a, ok_b);
  printf("lane 0: %g %g %g %g  lane 17: %g %g %g %g\n", h[0], h[1], h[2], h[3], h[68], h[69], h[70], h[71]);
  return 0;
}
