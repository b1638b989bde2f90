// Probe: operand lane map of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3, unit scales) and
// v_mfma_f32_16x16x32_fp8_fp8 on gfx950, with exact small-integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
typedef int intx8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ unsigned char f2e4(float f) {
  return (unsigned char)(__builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false) & 0xff);
}

// hypothesis H: lane l holds k = kmap(l, j) for j in [0,32)
__device__ int kmap(int h, int l, int j) {
  int g = l >> 4;
  if (h == 0) return 32 * g + j;                       // contiguous 32
  if (h == 1) return 8 * g + 32 * (j >> 3) + (j & 7);  // 8-element chunks interleaved over groups
  return 16 * g + 64 * (j >> 4) + (j & 15);            // 16-element chunks
}

__global__ void k128(const float* A, const float* B, float* D, int h) {
  int l = threadIdx.x;
  unsigned char a[32], b[32];
  for (int j = 0; j < 32; ++j) {
    int k = kmap(h, l, j);
    a[j] = f2e4(A[(l & 15) * 128 + k]);   // A[m][k]
    b[j] = f2e4(B[k * 16 + (l & 15)]);    // B[k][n]
  }
  intx8 av, bv;
  memcpy(&av, a, 32);
  memcpy(&bv, b, 32);
  floatx4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
  for (int v = 0; v < 4; ++v) D[(4 * (l >> 4) + v) * 16 + (l & 15)] = c[v];  // D[row][col]
}

__global__ void k32(const float* A, const float* B, float* D) {
  int l = threadIdx.x;
  unsigned char a[8], b[8];
  for (int j = 0; j < 8; ++j) {
    int k = 8 * (l >> 4) + j;
    a[j] = f2e4(A[(l & 15) * 128 + k]);
    b[j] = f2e4(B[k * 16 + (l & 15)]);
  }
  long av, bv;
  memcpy(&av, a, 8);
  memcpy(&bv, b, 8);
  floatx4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(av, bv, c, 0, 0, 0);
  for (int v = 0; v < 4; ++v) D[(4 * (l >> 4) + v) * 16 + (l & 15)] = c[v];
}

int main() {
  float hA[16 * 128], hB[128 * 16], ref[256], ref32[256], hD[256];
  srand(1);
  for (int i = 0; i < 16 * 128; ++i) hA[i] = (float)((rand() % 7) - 3);
  for (int i = 0; i < 128 * 16; ++i) hB[i] = (float)((rand() % 5) - 2);
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      float s = 0, s32 = 0;
      for (int k = 0; k < 128; ++k) s += hA[m * 128 + k] * hB[k * 16 + n];
      for (int k = 0; k < 32; ++k) s32 += hA[m * 128 + k] * hB[k * 16 + n];
      ref[m * 16 + n] = s;
      ref32[m * 16 + n] = s32;
    }
  float *dA, *dB, *dD;
  hipMalloc(&dA, sizeof(hA)); hipMalloc(&dB, sizeof(hB)); hipMalloc(&dD, sizeof(hD));
  hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
  for (int h = 0; h < 3; ++h) {
    hipLaunchKernelGGL(k128, dim3(1), dim3(64), 0, 0, dA, dB, dD, h);
    hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
    double err = 0;
    for (int i = 0; i < 256; ++i) err = fmax(err, fabs(hD[i] - ref[i]));
    printf("16x16x128 f8f6f4 hypothesis %d: max err %g %s\n", h, err, err == 0 ? "MATCH" : "");
  }
  hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < 256; ++i) err = fmax(err, fabs(hD[i] - ref32[i]));
  printf("16x16x32 fp8_fp8 (k = 8*(l>>4)+j): max err %g %s\n", err, err == 0 ? "MATCH" : "");
  return 0;
}
