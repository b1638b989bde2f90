// Probe: which weight element the fp4 GEMV pairs with x[k] -- y = w[k0] for a one-hot x at k0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "tl/tl.h"
typedef __bf16 b2 __attribute__((ext_vector_type(2)));

__global__ void one(const bfloat16_t* X, const uint8_t* Bq, float* Y) {
  const tl::intx4 w = reinterpret_cast<const tl::intx4*>(Bq)[0];
  float acc = 0.f;
  for (int q = 0; q < 4; ++q) {
    const tl::intx4 xv = reinterpret_cast<const tl::intx4*>(X)[q];
    const uint32_t u = (uint32_t)w[q];
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 0),
                                          __builtin_bit_cast(b2, xv[0]), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 1),
                                          __builtin_bit_cast(b2, xv[1]), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 2),
                                          __builtin_bit_cast(b2, xv[2]), acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, 1.0f, 3),
                                          __builtin_bit_cast(b2, xv[3]), acc, false);
  }
  if (threadIdx.x == 0) Y[0] = acc;
}

int main() {
  const float e2m1[16] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -0.f, -0.5f, -1, -1.5f, -2, -3, -4, -6};
  uint8_t wq[16];
  for (int i = 0; i < 16; ++i) wq[i] = (uint8_t)((i * 7 + 3) & 0x77) | (uint8_t)((i & 1) << 3);
  bfloat16_t* dx;
  uint8_t* dw;
  float* dy;
  (void)hipMalloc(&dx, 64);
  (void)hipMalloc(&dw, 16);
  (void)hipMalloc(&dy, 4);
  (void)hipMemcpy(dw, wq, 16, hipMemcpyHostToDevice);
  for (int k0 = 0; k0 < 32; ++k0) {
    uint16_t xb[32] = {0};
    xb[k0] = 0x3f80;  // 1.0
    (void)hipMemcpy(dx, xb, 64, hipMemcpyHostToDevice);
    one<<<1, 64>>>(dx, dw, dy);
    float y;
    (void)hipMemcpy(&y, dy, 4, hipMemcpyDeviceToHost);
    const uint8_t byte = wq[k0 / 2];
    printf("k0 %2d: got %5g  expect w[k0] %5g   (byte %02x)\n", k0, y, e2m1[(k0 & 1) ? byte >> 4 : byte & 15], byte);
  }
  return 0;
}
