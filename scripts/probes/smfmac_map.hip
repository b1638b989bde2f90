// Discovery probe: which B register element does compressed A value v (lane group g) with index
// field p multiply?  B element i of lane l holds code 100*(l>>4) + i (+1000 for lane&15 != 0).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k(float* out, int g0, int v0, int p, int abid_mode) {
  int l = threadIdx.x, g = l >> 4, r = l & 15;
  h8 a; h16 b;
  for (int v = 0; v < 8; ++v) a[v] = (_Float16)((r == 0 && g == g0 && v == v0) ? 1.f : 0.f);
  for (int i = 0; i < 16; ++i) b[i] = (_Float16)(float)(100 * g + i + (r ? 1000 : 0));
  int id = 0;
  for (int f = 0; f < 16; ++f) id |= p << (2 * f);
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b, acc, id, 0, 0);
  for (int v = 0; v < 4; ++v) out[(4 * g + v) * 16 + r] = acc[v];
}

int main() {
  float* dO; hipMalloc(&dO, 256 * 4);
  float O[256];
  for (int g0 = 0; g0 < 4; ++g0)
    for (int v0 = 0; v0 < 8; ++v0) {
      printf("g=%d v=%d:", g0, v0);
      for (int p = 0; p < 4; ++p) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dO, g0, v0, p, 0);
        hipMemcpy(O, dO, sizeof(O), hipMemcpyDeviceToHost);
        // find nonzero outputs in column 0
        printf("  p%d->", p);
        for (int m = 0; m < 16; ++m) if (O[m * 16] != 0.f) printf("[m%d]%g ", m, O[m * 16]);
      }
      printf("\n");
    }
  return 0;
}
