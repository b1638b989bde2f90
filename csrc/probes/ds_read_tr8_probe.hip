// Probe of ds_read_b64_tr_b8 (gfx950): LDS holds a 64 x 16 byte tile with byte(r, c) = r * 16 + c
// (row-major, 16 bytes per row); every lane (g = lane >> 4, i = lane & 15) supplies the address of
// row 8 * g + (i >> 1), columns 8 * (i & 1) .. +7 (the hypothesis: a 16-lane group transposes an
// 8-row x 16-column byte block, lane i receiving column i of the 8 rows).  Prints what each lane
// receives, byte by byte, and whether it equals rows 8g .. 8g + 7 of column i.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int v2i __attribute__((ext_vector_type(2)));

__global__ void probe(unsigned char* out) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[64 * 16];
  const int lane = threadIdx.x;
  for (int e = lane; e < 64 * 16; e += 64) lds[e] = (unsigned char)e;
  __syncthreads();
  const int g = lane >> 4, i = lane & 15;
  const int row = 8 * g + (i >> 1), col = 8 * (i & 1);
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (__attribute__((address_space(3))) v2i*)((__attribute__((address_space(3))) unsigned char*)lds + row * 16 + col));
  unsigned char* o = out + lane * 8;
  for (int b = 0; b < 4; ++b) {
    o[b] = (unsigned char)(v.x >> (8 * b));
    o[4 + b] = (unsigned char)(v.y >> (8 * b));
  }
}

int main() {
  unsigned char* d;
  unsigned char h[64 * 8];
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  int ok = 1;
  for (int lane = 0; lane < 64; ++lane) {
    const int g = lane >> 4, i = lane & 15;
    printf("lane %2d:", lane);
    for (int b = 0; b < 8; ++b) {
      printf(" %3d", h[lane * 8 + b]);
      if (h[lane * 8 + b] != (unsigned char)((8 * g + b) * 16 + i)) ok = 0;
    }
    printf("\n");
  }
  printf("hypothesis (lane i of group g gets rows 8g..8g+7 of column i): %s\n", ok ? "CONFIRMED" : "REJECTED");
  hipFree(d);
  return 0;
}
