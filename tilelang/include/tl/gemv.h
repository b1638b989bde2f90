// tl/gemv.h — decode-sized (M <= 8) GEMV over OCP MXFP4 weights on gfx950.
//
// y[m][n] = sum_k x[m][k] * w[n][k], x bf16 [M][K], w = Bq [N][K/2] (two e2m1 codes per byte, low
// nibble = even k) with S [N][K/32] e8m0 block scales.  Weight bytes are the whole cost (4.25
// bits per element), so the kernel is a single HBM stream:
//   * a thread owns 32-wide K chunks (16 weight bytes + 1 scale byte): one 16-byte non-temporal
//     load per (row, chunk), BLOCK_N rows in flight per thread;
//   * v_cvt_scalef32_pk_bf16_fp4 expands two codes per instruction with the e8m0 scale folded in
//     (no LUT, no exponent arithmetic; fp4 x 2^e is exact in bf16) and v_dot2_f32_bf16 multiplies
//     the pair against the thread's packed bf16 x chunk, held in registers: two instructions per
//     two weights, fp32 accumulation;
//   * wave shuffles + one LDS exchange per block reduce the BLOCK_N x M partial sums.
#pragma once

namespace tl {

typedef __bf16 tl_bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 tl_bf16x8 __attribute__((ext_vector_type(8)));

template <int M, int BLOCK_N, int THREADS, int RG = BLOCK_N>
TL_DEVICE void mxfp4_gemv(const bfloat16_t* __restrict__ X, const uint8_t* __restrict__ Bq,
                          const uint8_t* __restrict__ S, bfloat16_t* __restrict__ Y, int N, int K, int n0,
                          float* __restrict__ red) {
  // BLOCK_N rows per block in groups of RG (RG x M accumulators per thread): a block reads x once
  // per group from L1/L2, so x traffic per weight byte is 4M / BLOCK_N (was 4M / RG with one group:
  // 16x the weight bytes at M = 8) while the register footprint stays RG x M
  static_assert(THREADS % 64 == 0 && RG * M <= THREADS && BLOCK_N % RG == 0, "mxfp4_gemv: block shape");
  constexpr int NW = THREADS / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunks = K >> 5;
  for (int g0 = 0; g0 < BLOCK_N; g0 += RG) {
    float acc[RG][M];
#pragma unroll
    for (int n = 0; n < RG; ++n)
#pragma unroll
      for (int m = 0; m < M; ++m) acc[n][m] = 0.f;
    for (int c = tid; c < chunks; c += THREADS) {
      // the thread's x chunk stays packed: 16 bf16 pairs per row
      tl_bf16x8 x[M][4];
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int q = 0; q < 4; ++q) x[m][q] = reinterpret_cast<const tl_bf16x8*>(X + (long long)m * K + c * 32)[q];
      intx4 w[RG];
      float sc[RG];
#pragma unroll
      for (int n = 0; n < RG; ++n) {
        const int row = min(n0 + g0 + n, N - 1);
        w[n] = __builtin_nontemporal_load(reinterpret_cast<const intx4*>(Bq + (long long)row * (K >> 1)) + c);
        sc[n] = __builtin_bit_cast(float, (uint32_t)S[(long long)row * chunks + c] << 23);
      }
#pragma unroll
      for (int n = 0; n < RG; ++n) {
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          // dword d of the weights = k in [8d, 8d + 8): byte b -> bf16 pair k = 8d + 2b, +1
          const uint32_t u = (uint32_t)w[n][d];
          const tl_bf16x2 w0 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc[n], 0);
          const tl_bf16x2 w1 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc[n], 1);
          const tl_bf16x2 w2 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc[n], 2);
          const tl_bf16x2 w3 = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp4(u, sc[n], 3);
#pragma unroll
          for (int m = 0; m < M; ++m) {
            // x pairs for k = 8d .. 8d + 7 are elements 2b, 2b + 1 of x[m][d].  Pairs are taken with
            // shufflevector: bit-casting the dwords of an int vector to bf16x2 miscompiles on ROCm
            // 7.2 (every pair became dword 0 -- csrc/probes/fp4_perm_probe.hip)
            const tl_bf16x8 xv = x[m][d];
            float a = acc[n][m];
            a = __builtin_amdgcn_fdot2_f32_bf16(w0, __builtin_shufflevector(xv, xv, 0, 1), a, false);
            a = __builtin_amdgcn_fdot2_f32_bf16(w1, __builtin_shufflevector(xv, xv, 2, 3), a, false);
            a = __builtin_amdgcn_fdot2_f32_bf16(w2, __builtin_shufflevector(xv, xv, 4, 5), a, false);
            a = __builtin_amdgcn_fdot2_f32_bf16(w3, __builtin_shufflevector(xv, xv, 6, 7), a, false);
            acc[n][m] = a;
          }
        }
      }
    }
    // wave reduction, then one LDS exchange across the block's waves
#pragma unroll
    for (int n = 0; n < RG; ++n)
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float v = acc[n][m];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if (lane == 0) red[wave * (RG * M) + n * M + m] = v;
      }
    __syncthreads();
    if (tid < RG * M) {
      float v = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < NW; ++w2) v += red[w2 * (RG * M) + tid];
      const int n = g0 + tid / M, m = tid % M;
      if (n0 + n < N) Y[(long long)m * N + n0 + n] = (bfloat16_t)v;
    }
    __syncthreads();  // red is reused by the next group
  }
}

}  // namespace tl
