// fp6 operand layout probe, part 2: full 16x16 outputs for selected A patterns (B = 1.0 everywhere,
// unit scales).  Pattern p: 0 = every field of every lane; 1 = every field of lanes 16-31 only;
// 2 = field 0 of lane 16 only; 3 = every field of lane 0 only; 4 = A = 1.0 in dword d only (all lanes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef int intx8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ void put6(unsigned char* p, int f, unsigned v) {
  const int bit = 6 * f;
  unsigned w = p[bit / 8] | (p[bit / 8 + 1] << 8);
  w |= (v & 63u) << (bit % 8);
  p[bit / 8] = w & 255;
  p[bit / 8 + 1] = (w >> 8) & 255;
}

__global__ void probe(int pat, int arg, float* D) {
  const int l = threadIdx.x, g = l >> 4;
  const unsigned one = 8u;  // e2m3 1.0
  unsigned char a[33], b[33];
  for (int j = 0; j < 33; ++j) { a[j] = 0; b[j] = 0; }
  for (int f = 0; f < 32; ++f) put6(b, f, one);
  for (int f = 0; f < 32; ++f) {
    bool on = (pat == 0) || (pat == 1 && g == 1) || (pat == 2 && l == 16 && f == 0) || (pat == 3 && l == 0) ||
              (pat == 4 && (6 * f) / 32 == arg);
    if (on) put6(a, f, one);
  }
  intx8 av = {0, 0, 0, 0, 0, 0, 0, 0}, bv = {0, 0, 0, 0, 0, 0, 0, 0};
  memcpy(&av, a, 24);
  memcpy(&bv, b, 24);
  floatx4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 2, 2, 0, 127, 0, 127);
  for (int v = 0; v < 4; ++v) D[(4 * g + v) * 16 + (l & 15)] = c[v];
}

int main() {
  float* dD;
  float h[256];
  (void)hipMalloc(&dD, sizeof(h));
  for (int pat = 0; pat < 5; ++pat) {
    for (int arg = 0; arg < (pat == 4 ? 6 : 1); ++arg) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, pat, arg, dD);
      (void)hipMemcpy(h, dD, sizeof(h), hipMemcpyDeviceToHost);
      printf("pattern %d arg %d:\n", pat, arg);
      for (int m = 0; m < 16; ++m) {
        printf("  ");
        for (int n = 0; n < 16; ++n) printf("%4g", h[m * 16 + n]);
        printf("\n");
      }
    }
  }
  (void)hipFree(dD);
  return 0;
}
