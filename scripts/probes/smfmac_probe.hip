// Hardware probe of v_smfmac_f32_16x16x64_f16 operand / index semantics (one wave).
// Hypothesis: lane l (row/col l&15, k-slice g=l>>4) holds B[k=16g+i][n] (i<16) and 8 compressed
// A values; value v belongs to the group of 4 k = 16g + 4(v>>1) + pos, pos = idx bits [2v+1:2v].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k(float* out, const _Float16* Ac, const int* idx, const _Float16* B, int mode) {
  int l = threadIdx.x, g = l >> 4, r = l & 15;
  h8 a; h16 b;
  for (int v = 0; v < 8; ++v) a[v] = Ac[r * 32 + 8 * g + v];   // compressed row: 32 values per 64 k
  for (int i = 0; i < 16; ++i) b[i] = B[(16 * g + i) * 16 + r];
  int id = idx[r * 4 + g];
  if (mode == 1) id = id | (id << 16);
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b, acc, id, 0, 0);
  for (int v = 0; v < 4; ++v) out[(4 * g + v) * 16 + r] = acc[v];
}

int main() {
  const int M = 16, N = 16, K = 64;
  float A[M][K] = {}, Bf[K][N];
  _Float16 Ac[M * 32], Bh[K * N];
  int idx[M * 4];
  srand(1);
  for (int m = 0; m < M; ++m)
    for (int q = 0; q < K / 4; ++q) {
      int p0 = rand() % 4, p1 = rand() % 4;
      while (p1 == p0) p1 = rand() % 4;
      if (p1 < p0) { int t = p0; p0 = p1; p1 = t; }
      float x0 = (rand() % 17 - 8) / 4.0f, x1 = (rand() % 17 - 8) / 4.0f;
      A[m][4 * q + p0] = x0; A[m][4 * q + p1] = x1;
      Ac[m * 32 + 2 * q] = (_Float16)x0; Ac[m * 32 + 2 * q + 1] = (_Float16)x1;
      int gi = q / 4, w = q % 4;  // lane group gi holds groups 4gi..4gi+3
      if (w == 0) idx[m * 4 + gi] = 0;
      idx[m * 4 + gi] |= (p0 | (p1 << 2)) << (4 * w);
    }
  for (int kk = 0; kk < K; ++kk)
    for (int n = 0; n < N; ++n) { Bf[kk][n] = (rand() % 9 - 4) / 2.0f; Bh[kk * N + n] = (_Float16)Bf[kk][n]; }
  float* dO; _Float16 *dA, *dB; int* dI;
  hipMalloc(&dO, M * N * 4); hipMalloc(&dA, sizeof(Ac)); hipMalloc(&dB, sizeof(Bh)); hipMalloc(&dI, sizeof(idx));
  hipMemcpy(dA, Ac, sizeof(Ac), hipMemcpyHostToDevice);
  hipMemcpy(dB, Bh, sizeof(Bh), hipMemcpyHostToDevice);
  hipMemcpy(dI, idx, sizeof(idx), hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    float O[M * N];
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dO, dA, dI, dB, mode);
    hipMemcpy(O, dO, sizeof(O), hipMemcpyDeviceToHost);
    double err = 0;
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        float ref = 0;
        for (int kk = 0; kk < K; ++kk) ref += A[m][kk] * Bf[kk][n];
        err = fmax(err, fabs(ref - O[m * N + n]));
      }
    printf("mode %d max_err %g  (O[0]=%g)\n", mode, err, O[0]);
  }
  return 0;
}
