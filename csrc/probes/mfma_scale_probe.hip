// Probe: which (row, 32-K block) does the e8m0 scale supplied by lane L of
// v_mfma_scale_f32_16x16x128_f8f6f4 apply to, for fp8 (e4m3) and fp4 (e2m1) operands?
// Operand data as in tl/gemm.h: lane l holds row l&15 and the 32 consecutive K starting at
// 32*(l>>4) (fp8: 32 bytes, fp4: 16 bytes, low nibble = even k).  A is non-zero in ONE K block b
// at a time; lane L's A-scale is doubled; every output row that changes is recorded.
// Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/probe mfma_scale_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
typedef int intx8 __attribute__((ext_vector_type(8)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <int FMT>
__global__ void probe(int blk, int lane_sel, int which, float* D) {
  const int l = threadIdx.x, g = l >> 4;
  unsigned char a[32], b[32];
  for (int j = 0; j < 32; ++j) { a[j] = 0; b[j] = 0; }
  if (FMT == 0) {  // e4m3 1.0 = 0x38
    for (int j = 0; j < 32; ++j) { a[j] = (g == blk) ? 0x38 : 0; b[j] = 0x38; }
  } else {         // e2m1 1.0 = 0x2, two per byte
    for (int j = 0; j < 16; ++j) { a[j] = (g == blk) ? 0x22 : 0; b[j] = 0x22; }
  }
  intx8 av, bv;
  memcpy(&av, a, 32);
  memcpy(&bv, b, 32);
  int sa = 127, sb = 127;
  if (which == 0 && l == lane_sel) sa = 128;
  if (which == 1 && l == lane_sel) sb = 128;
  floatx4 c = {0, 0, 0, 0};
  // plain operand order: instruction A = our A (rows m), instruction B = our B (cols n)
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, FMT, FMT, 0, sa, 0, sb);
  for (int v = 0; v < 4; ++v) D[(4 * g + v) * 16 + (l & 15)] = c[v];  // D[m][n]
}

template <int FMT>
void run(const char* name) {
  float* dD;
  float hD[256];
  hipMalloc(&dD, sizeof(hD));
  for (int which = 0; which < 2; ++which) {
    int bad = 0;
    for (int L = 0; L < 64; ++L) {
      printf("%s %s-scale lane %2d ->", name, which ? "B" : "A", L);
      for (int blk = 0; blk < 4; ++blk) {
        hipLaunchKernelGGL(probe<FMT>, dim3(1), dim3(64), 0, 0, blk, L, which, dD);
        hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
        // baseline: 32 per (row, col) for the one non-zero block; collect changed rows / cols
        unsigned rows = 0, cols = 0;
        float val = 0;
        for (int m = 0; m < 16; ++m)
          for (int n = 0; n < 16; ++n)
            if (hD[m * 16 + n] != 32.0f) { rows |= 1u << m; cols |= 1u << n; val = hD[m * 16 + n]; }
        if (rows) printf(" blk%d:rows=%04x cols=%04x v=%g", blk, rows, cols, val);
        const unsigned want = 1u << (L & 15);
        const bool hit = rows != 0;
        const bool expect = blk == (L >> 4);
        if (hit != expect || (hit && (which == 0 ? rows != want || cols != 0xffff : cols != want || rows != 0xffff)))
          ++bad;
      }
      printf("\n");
    }
    printf("%s %s-scale: %d entries differ from lane->(row l&15, block l>>4)\n", name, which ? "B" : "A", bad);
  }
  hipFree(dD);
}

int main() {
  run<0>("fp8");
  run<4>("fp4");
  return 0;
}
