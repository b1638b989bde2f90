// Probe: v_dot2_f32_bf16 on known pairs, and tl::mxfp4_gemv (tl/gemv.h) on a small random
// problem against a host fp32 reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include "tl/tl.h"
#include "tl/gemv.h"

__global__ void dot_probe(float* out) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  b2 a = {(__bf16)1.5f, (__bf16)-2.0f};
  b2 b = {(__bf16)4.0f, (__bf16)0.25f};
  out[0] = __builtin_amdgcn_fdot2_f32_bf16(a, b, 10.0f, false);  // 6 - 0.5 + 10 = 15.5
}

template <int M, int BN, int TH>
__global__ void __launch_bounds__(TH) gemv(const bfloat16_t* X, const uint8_t* Bq, const uint8_t* S, bfloat16_t* Y,
                                           int N, int K) {
  __shared__ float red[(TH / 64) * BN * M];
  tl::mxfp4_gemv<M, BN, TH>(X, Bq, S, Y, N, K, blockIdx.x * BN, red);
}

__constant__ float kE2M1[16] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -0.f, -0.5f, -1, -1.5f, -2, -3, -4, -6};

// one thread per (m, n): the inner loop of mxfp4_gemv with one of its two halves replaced
template <int MODE>
__global__ void gemv_var(const bfloat16_t* X, const uint8_t* Bq, const uint8_t* S, float* Y, int M, int N, int K) {
  typedef __bf16 b2 __attribute__((ext_vector_type(2)));
  const int m = threadIdx.x / N, n = threadIdx.x % N;
  if (m >= M) return;
  float acc = 0.f;
  for (int c = 0; c < K / 32; ++c) {
    const tl::intx4 w = reinterpret_cast<const tl::intx4*>(Bq + n * (K / 2))[c];
    const float sc = __builtin_bit_cast(float, (uint32_t)S[n * (K / 32) + c] << 23);
    for (int q = 0; q < 4; ++q) {
      typedef __bf16 b8 __attribute__((ext_vector_type(8)));
      const b8 xv = reinterpret_cast<const b8*>(X + m * K + c * 32)[q];
      const uint32_t u = (uint32_t)w[q];
      for (int b = 0; b < 4; ++b) {
        b2 wp;
        if (MODE == 2) {
          const uint32_t byte = (u >> (8 * b)) & 0xff;
          wp[0] = (__bf16)(kE2M1[byte & 15] * sc);
          wp[1] = (__bf16)(kE2M1[byte >> 4] * sc);
        } else {
          wp = b == 0 ? __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc, 0)
             : b == 1 ? __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc, 1)
             : b == 2 ? __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc, 2)
                      : __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc, 3);
        }
        const b2 xp = b == 0 ? __builtin_shufflevector(xv, xv, 0, 1) : b == 1 ? __builtin_shufflevector(xv, xv, 2, 3)
                    : b == 2 ? __builtin_shufflevector(xv, xv, 4, 5) : __builtin_shufflevector(xv, xv, 6, 7);
        if (MODE == 1) acc += (float)wp[0] * (float)xp[0] + (float)wp[1] * (float)xp[1];
        else acc = __builtin_amdgcn_fdot2_f32_bf16(wp, xp, acc, false);
      }
    }
  }
  Y[m * N + n] = acc;
}

static float bf(float x) {  // round to bf16
  uint32_t u;
  std::memcpy(&u, &x, 4);
  u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
  std::memcpy(&x, &u, 4);
  return x;
}

int main() {
  float* d;
  (void)hipMalloc(&d, 4);
  dot_probe<<<1, 64>>>(d);
  float h;
  (void)hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
  printf("fdot2 bf16: got %g expect 15.5 %s\n", h, h == 15.5f ? "ok" : "MISMATCH");
  const float e2m1[16] = {0, 0.5f, 1, 1.5f, 2, 3, 4, 6, -0.f, -0.5f, -1, -1.5f, -2, -3, -4, -6};
  constexpr int M = 2, N = 64, K = 256, BN = 8, TH = 256;
  static uint16_t xb[M * K];
  static float xf[M * K];
  static uint8_t wq[N * K / 2], sc[N * K / 32];
  srand(1);
  for (int i = 0; i < M * K; ++i) {
    float v = bf((rand() % 2001 - 1000) / 500.0f);
    xf[i] = v;
    uint32_t u;
    std::memcpy(&u, &v, 4);
    xb[i] = u >> 16;
  }
  for (int i = 0; i < N * K / 2; ++i) wq[i] = rand() & 0xff;
  for (int i = 0; i < N * K / 32; ++i) sc[i] = 124 + rand() % 6;
  bfloat16_t *dx, *dy;
  uint8_t *dw, *ds;
  (void)hipMalloc(&dx, sizeof(xb));
  (void)hipMalloc(&dw, sizeof(wq));
  (void)hipMalloc(&ds, sizeof(sc));
  (void)hipMalloc(&dy, M * N * 2);
  (void)hipMemcpy(dx, xb, sizeof(xb), hipMemcpyHostToDevice);
  (void)hipMemcpy(dw, wq, sizeof(wq), hipMemcpyHostToDevice);
  (void)hipMemcpy(ds, sc, sizeof(sc), hipMemcpyHostToDevice);
  gemv<M, BN, TH><<<N / BN, TH>>>(dx, dw, ds, dy, N, K);
  static uint16_t yb[M * N];
  (void)hipMemcpy(yb, dy, sizeof(yb), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      double ref = 0;
      for (int k = 0; k < K; ++k) {
        const uint8_t byte = wq[n * K / 2 + k / 2];
        const float w = e2m1[(k & 1) ? byte >> 4 : byte & 15] * ldexpf(1.f, sc[n * K / 32 + k / 32] - 127);
        ref += (double)w * xf[m * K + k];
      }
      uint32_t u = (uint32_t)yb[m * N + n] << 16;
      float got;
      std::memcpy(&got, &u, 4);
      if (fabs(got - ref) > 0.02 * fabs(ref) + 0.05) {
        if (bad < 8) printf("  y[%d][%d] got %g ref %g\n", m, n, got, ref);
        ++bad;
      }
    }
  printf("mxfp4_gemv: %d / %d mismatches\n", bad, M * N);
  float* dyf;
  (void)hipMalloc(&dyf, M * N * 4);
  static float yf[M * N];
  for (int mode = 0; mode < 3; ++mode) {
    if (mode == 0) gemv_var<0><<<1, M * N>>>(dx, dw, ds, dyf, M, N, K);
    if (mode == 1) gemv_var<1><<<1, M * N>>>(dx, dw, ds, dyf, M, N, K);
    if (mode == 2) gemv_var<2><<<1, M * N>>>(dx, dw, ds, dyf, M, N, K);
    (void)hipMemcpy(yf, dyf, sizeof(yf), hipMemcpyDeviceToHost);
    int bad2 = 0;
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        double ref = 0;
        for (int k = 0; k < K; ++k) {
          const uint8_t byte = wq[n * K / 2 + k / 2];
          const float w = e2m1[(k & 1) ? byte >> 4 : byte & 15] * ldexpf(1.f, sc[n * K / 32 + k / 32] - 127);
          ref += (double)w * xf[m * K + k];
        }
        if (fabs(yf[m * N + n] - ref) > 1e-3 * fabs(ref) + 1e-3) {
          if (bad2 < 3) printf("  mode %d y[%d][%d] got %g ref %g\n", mode, m, n, yf[m * N + n], ref);
          ++bad2;
        }
      }
    printf("variant mode %d (0 cvt+dot2, 1 cvt+fma, 2 lut+dot2): %d / %d mismatches\n", mode, bad2, M * N);
  }
  return 0;
}
