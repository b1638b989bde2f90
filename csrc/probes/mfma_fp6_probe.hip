// Probe: fp6 operands of v_mfma_scale_f32_16x16x128_f8f6f4 (e2m3 = format 2, e3m2 = format 3).
// Which 32-K scale block does 6-bit field f (bits 6f..6f+5 of the 192-bit lane operand) of a lane
// in group g = lane>>4 belong to?  A = 1.0 in field f of every lane of group g only, B = 1.0 in
// every field; then lane group s's A scale is doubled: the output doubles iff the element's K
// block is s.  Prints, for every (g, f), the block s (and the value, which checks the encoding).
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/fp6probe mfma_fp6_probe.hip
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

template <int FMT>
__global__ void probe(int g_data, int f_data, int s_grp, float* D) {
  const int l = threadIdx.x, g = l >> 4;
  const unsigned one = FMT == 2 ? 8u : 12u;  // e2m3 1.0 = 0 01 000, e3m2 1.0 = 0 011 00
  unsigned char a[33], b[33];
  for (int j = 0; j < 33; ++j) { a[j] = 0; b[j] = 0; }
  for (int f = 0; f < 32; ++f) put6(b, f, one);
  if (g == g_data) put6(a, f_data, one);
  intx8 av = {0, 0, 0, 0, 0, 0, 0, 0}, bv = {0, 0, 0, 0, 0, 0, 0, 0};
  memcpy(&av, a, 24);
  memcpy(&bv, b, 24);
  const int sa = (s_grp >= 0 && g == s_grp) ? 128 : 127;
  floatx4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, FMT, FMT, 0, sa, 0, 127);
  if (l == 0) D[0] = c[0];  // row 0, col 0 (lane 0 holds D[0..3][0])
}

template <int FMT>
void run(const char* name) {
  float* dD;
  float h;
  hipMalloc(&dD, 4);
  int contiguous = 0, halves = 0;
  for (int g = 0; g < 4; ++g) {
    printf("%s g%d:", name, g);
    for (int f = 0; f < 32; ++f) {
      hipLaunchKernelGGL(probe<FMT>, dim3(1), dim3(64), 0, 0, g, f, -1, dD);
      hipMemcpy(&h, dD, 4, hipMemcpyDeviceToHost);
      const float base = h;
      int blk = -1;
      for (int s = 0; s < 4; ++s) {
        hipLaunchKernelGGL(probe<FMT>, dim3(1), dim3(64), 0, 0, g, f, s, dD);
        hipMemcpy(&h, dD, 4, hipMemcpyDeviceToHost);
        if (h != base) blk = s;
      }
      printf(" %d", blk);
      if (f == 0) printf("(v=%g)", base);
      if (blk == g) ++contiguous;
      if (blk == 2 * (f >= 16) + (g >> 1)) ++halves;
    }
    printf("\n");
  }
  printf("%s: %d/128 fields match 'group g = K block g' (fp4-like), %d/128 match the fp8-like two halves\n", name,
         contiguous, halves);
  hipFree(dD);
}

int main() {
  run<2>("e2m3");
  run<3>("e3m2");
  return 0;
}
