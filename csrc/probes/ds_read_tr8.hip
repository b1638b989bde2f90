// Probe: which LDS bytes does ds_read_b64_tr_b8 return to each lane when lane l supplies byte
// address 8*l?  Output: src[l][b] = LDS byte index delivered in byte b of lane l.
// Build + run: hipcc --offload-arch=gfx950 -O2 -o /tmp/tr8 csrc/probes/ds_read_tr8.hip && /tmp/tr8
#include <hip/hip_runtime.h>
#include <cstdio>

typedef int int2v __attribute__((ext_vector_type(2)));

__global__ void probe(unsigned char* out, int pass) {
  __shared__ unsigned char lds[1024];
  for (int j = threadIdx.x; j < 1024; j += 64)
    lds[j] = pass == 0 ? (unsigned char)(j & 255) : (unsigned char)(j >> 8);
  __syncthreads();
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  typedef __attribute__((address_space(3))) int2v lds_i2;
  int2v r = __builtin_amdgcn_ds_read_tr8_b64_v2i32((lds_i2*)((lds_u8*)lds + threadIdx.x * 8));
  unsigned char* p = reinterpret_cast<unsigned char*>(&r);
  for (int b = 0; b < 8; ++b) out[threadIdx.x * 8 + b] = p[b];
}

int main() {
  unsigned char *d, h0[512], h1[512];
  hipMalloc(&d, 512);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 0);
  hipMemcpy(h0, d, 512, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 1);
  hipMemcpy(h1, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int b = 0; b < 8; ++b) printf(" %4d", h0[l * 8 + b] + 256 * h1[l * 8 + b]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
