// Probe: what v_cvt_scalef32_pk_bf16_fp4 (__builtin_amdgcn_cvt_scalef32_pk_bf16_fp4) returns for a
// known word, each byte selector and two scales; the host prints it next to the OCP e2m1 table.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__global__ void probe(const uint32_t* words, float* out) {
  const int i = threadIdx.x;
  if (i >= 4) return;
  const uint32_t u = words[i];
  const float s1 = 1.0f, s8 = 8.0f;
  bf16x2 r[8];
  r[0] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s1, 0);
  r[1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s1, 1);
  r[2] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s1, 2);
  r[3] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s1, 3);
  r[4] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s8, 0);
  r[5] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s8, 1);
  r[6] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s8, 2);
  r[7] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, s8, 3);
  for (int j = 0; j < 8; ++j) {
    out[i * 16 + 2 * j] = (float)r[j][0];
    out[i * 16 + 2 * j + 1] = (float)r[j][1];
  }
}

int main() {
  const float e2m1[16] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -0.f, -0.5f, -1, -1.5f, -2, -3, -4, -6};
  uint32_t h[4] = {0x76543210u, 0xFEDCBA98u, 0x1F2E3D4Cu, 0x00000071u};
  uint32_t* dw;
  float* dout;
  hipMalloc(&dw, sizeof(h));
  hipMalloc(&dout, 64 * sizeof(float));
  hipMemcpy(dw, h, sizeof(h), hipMemcpyHostToDevice);
  probe<<<1, 64>>>(dw, dout);
  float o[64];
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 4; ++i) {
    printf("word %08x\n", h[i]);
    for (int j = 0; j < 8; ++j) {
      const int sel = j & 3;
      const float sc = j < 4 ? 1.f : 8.f;
      const uint32_t byte = (h[i] >> (8 * sel)) & 0xff;
      const float lo = e2m1[byte & 15] * sc, hi = e2m1[byte >> 4] * sc;
      const bool ok = o[i * 16 + 2 * j] == lo && o[i * 16 + 2 * j + 1] == hi;
      bad += !ok;
      printf("  scale %g sel %d: got (%g, %g) expect lo-nibble-first (%g, %g) %s\n", sc, sel, o[i * 16 + 2 * j],
             o[i * 16 + 2 * j + 1], lo, hi, ok ? "ok" : "MISMATCH");
    }
  }
  printf("%d mismatches\n", bad);
  return 0;
}
