// Probe: v_mfma_i32_16x16x64_i8 operand / result lane layout (A 16x64, B stored [16 cols][64 k]).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(const int8_t* A, const int8_t* B, int* D, float* Df) {
  const int l = threadIdx.x;
  i32x4 a = *reinterpret_cast<const i32x4*>(A + (l & 15) * 64 + 16 * (l >> 4));
  i32x4 b = *reinterpret_cast<const i32x4*>(B + (l & 15) * 64 + 16 * (l >> 4));
  i32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
  // the same through the f32x4 carrier used by the GEMM
  f32x4 cf = {0.f, 0.f, 0.f, 0.f};
  cf = __builtin_bit_cast(f32x4, __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, __builtin_bit_cast(i32x4, cf), 0, 0, 0));
  for (int r = 0; r < 4; ++r) Df[(4 * (l >> 4) + r) * 16 + (l & 15)] = (float)__builtin_bit_cast(int, cf[r]);
}
int main() {
  int8_t hA[16 * 64], hB[16 * 64];
  for (int i = 0; i < 16 * 64; ++i) { hA[i] = (int8_t)((i * 7) % 11 - 5); hB[i] = (int8_t)((i * 5) % 13 - 6); }
  int8_t *dA, *dB; int* dD; float* dF;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 1024); hipMalloc(&dF, 1024);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dA, dB, dD, dF);
  int hD[256]; float hF[256];
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost); hipMemcpy(hF, dF, 1024, hipMemcpyDeviceToHost);
  int bad = 0, badf = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int kk = 0; kk < 64; ++kk) s += hA[i * 64 + kk] * hB[j * 64 + kk];
      if (s != hD[i * 16 + j]) { if (bad < 5) printf("D[%d][%d] = %d want %d\n", i, j, hD[i * 16 + j], s); ++bad; }
      if ((float)s != hF[i * 16 + j]) { if (badf < 5) printf("F[%d][%d] = %f want %d\n", i, j, hF[i * 16 + j], s); ++badf; }
    }
  printf("int mismatches %d, f32-carrier mismatches %d\n", bad, badf);
  return 0;
}
