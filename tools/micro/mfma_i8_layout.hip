// Layout check for the int8 MFMAs the bootstrap uses (gfx950):
//   v_mfma_i32_32x32x32_i8 and v_mfma_i32_16x16x64_i8.
// Lane l holds 16 int8 of A (row l & 31 | l & 15) and 16 of B (column l & 31 | l & 15); the
// slot (lane group h = l >> 5 | l >> 4, byte j) carries the same k for both, so any
// consistent k assignment gives the product.  C/D: the standard f32 maps (32x32: col = l & 31,
// row = (r & 3) + 8 (r >> 2) + 4 (l >> 5); 16x16: col = l & 15, row = 4 (l >> 4) + r).
// Exact integer data, asymmetric B; prints PASS/FAIL per shape.
// build: hipcc -O2 --offload-arch=gfx950 mfma_i8_layout.hip -o mfma_i8_layout
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

__global__ void k32(const signed char* A, const signed char* B, int* C) {  // A 32x32 (row-major), B 32x32 (k-major)
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  i32x4v a, b;
  signed char* pa = reinterpret_cast<signed char*>(&a);
  signed char* pb = reinterpret_cast<signed char*>(&b);
  for (int j = 0; j < 16; ++j) {
    const int k = 16 * h + j;
    pa[j] = A[r * 32 + k];
    pb[j] = B[k * 32 + r];
  }
  i32x16 c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * h, col = r;
    C[row * 32 + col] = c[q];
  }
}

__global__ void k16(const signed char* A, const signed char* B, int* C) {  // A 16x64, B 64x16
  const int l = threadIdx.x, r = l & 15, h = l >> 4;
  i32x4v a, b;
  signed char* pa = reinterpret_cast<signed char*>(&a);
  signed char* pb = reinterpret_cast<signed char*>(&b);
  for (int j = 0; j < 16; ++j) {
    const int k = 16 * h + j;
    pa[j] = A[r * 64 + k];
    pb[j] = B[k * 16 + r];
  }
  i32x4 c = {};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int q = 0; q < 4; ++q) C[(4 * h + q) * 16 + r] = c[q];
}

static bool run(int M, int N, int K, bool big) {
  std::vector<signed char> A(M * K), B(K * N);
  srand(7 + M);
  for (auto& x : A) x = (signed char)(rand() % 255 - 127);
  for (int k = 0; k < K; ++k)
    for (int n = 0; n < N; ++n) B[k * N + n] = (signed char)((k * 7 + n * 3 + (k * n) % 11) % 255 - 127);
  std::vector<int> want(M * N, 0), got(M * N, -1);
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n)
      for (int k = 0; k < K; ++k) want[m * N + n] += (int)A[m * K + k] * (int)B[k * N + n];
  signed char *dA, *dB;
  int* dC;
  (void)hipMalloc(&dA, A.size());
  (void)hipMalloc(&dB, B.size());
  (void)hipMalloc(&dC, sizeof(int) * M * N);
  (void)hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice);
  if (big)
    hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  else
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(got.data(), dC, sizeof(int) * M * N, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < M * N; ++i) bad += got[i] != want[i];
  printf("%dx%dx%d i8: %s (%d of %d wrong)\n", M, N, K, bad ? "FAIL" : "PASS", bad, M * N);
  (void)hipFree(dA);
  (void)hipFree(dB);
  (void)hipFree(dC);
  return bad == 0;
}

int main() {
  const bool a = run(32, 32, 32, true);
  const bool b = run(16, 16, 64, false);
  return (a && b) ? 0 : 1;
}
