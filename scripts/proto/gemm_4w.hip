// Prototype: 256x256x64 fp16 NT GEMM (A [M][K], B [N][K], C [M][N] fp16) with FOUR waves (one
// per SIMD, a 128x128 piece each, accumulators in the accumulator file) and a register-pipelined
// 4-phase schedule; A/B'd through scripts/proto/gemm_8ph_ab.py (--src gemm_4w.hip).
//
//   * LDS: as gemm_8ph.hip -- 2 buffers x 4 half-tile slots [128 rows][64 k] fp16 (A0 A1 B0 B1),
//     chunks XOR-swizzled by (row >> 1) & 7 on the LDS-DMA source address.
//   * phase p of tile t: the MFMAs of one 64x64 quadrant piece x K=64 (32 per wave) run on
//     fragments read in phase p-1, while the fragments of phase p+1 are read (orders at PHASE);
//     the loop body is two tiles, so every slot and register piece is static.
//   * every phase ends with lgkmcnt(0) + s_barrier (its reads retired), so a slot read in phase q
//     is restaged from phase q+1; P1 waits vmcnt(12): tile t+1 landed, 3 half-tiles (12 DMAs)
//     left in flight.  DMA through buffer resources: one per-lane offset, the rest in SGPRs.
#include "tl/tl.h"

#ifndef GM
#define GM 4096
#endif
#ifndef GN
#define GN 4096
#endif
#ifndef GK
#define GK 4096
#endif
#ifndef PRIO
#define PRIO 0
#endif
#ifndef ASM_MFMA
#define ASM_MFMA 1  // accumulators pinned in the accumulator file ("+a"): the compiler's own MFMA
                    // scheduling renames D != C and spills at 256 accumulators + fragments
#endif

namespace p4 {
using namespace tl;
typedef mfma_traits<half_t> MT;
typedef MT::frag F;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HALF = 128 * BK;
constexpr int NT = GK / BK;
static_assert(NT % 2 == 0 && NT >= 4, "K tiles: even, >= 4");

TL_DEVICE void bar_lgkm() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int SLOT_OFF>
TL_DEVICE void read_piece(const half_t* smem, F (&p)[4][2], int r0, int lrow, const int (&cx)[2]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      p[i][kk] = *reinterpret_cast<const F*>(smem + SLOT_OFF + (r0 + i * 16) * BK + lrow + cx[kk]);
}

template <int QA, int QB>
TL_DEVICE void mma(const F (&a)[4][2], const F (&b)[4][2], floatx4 (&acc)[2][2][4][4]) {
#if PRIO
  __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
#if ASM_MFMA
        asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc[QA][QB][mi][ni]) : "v"(b[ni][kk]), "v"(a[mi][kk]));
#else
        acc[QA][QB][mi][ni] = MT::mma16(b[ni][kk], a[mi][kk], acc[QA][QB][mi][ni]);
#endif
      }
#if PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}
}  // namespace p4

extern "C" __global__ void __launch_bounds__(256) gemm_kernel(half_t* __restrict__ A, half_t* __restrict__ B,
                                                              half_t* __restrict__ C) {
  using namespace p4;
  __shared__ __attribute__((aligned(1024))) char tl_smem[135168];
  half_t* smem = reinterpret_cast<half_t*>(tl_smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int bid = blockIdx.x + blockIdx.y * gridDim.x;
  bid = tl::xcd_remap(bid, gridDim.x * gridDim.y);
  int bx, by;
  tl::rasterize_row<8>(bid, gridDim.x, gridDim.y, bx, by);

  // LDS-DMA: chunks q = j*256 + tid (j = 0..3): LDS row q >> 3, position q & 7 holding global
  // chunk (q & 7) ^ ((row >> 1) & 7)
  const int dc = (tid & 7) ^ ((tid >> 4) & 7);
  // buffer-resource DMA: one per-lane 32-bit offset, the slot / piece / tile part in SGPRs
  const uint32_t voff = (uint32_t)(((tid >> 3) * GK + dc * 8) * 2);
  const __amdgpu_buffer_rsrc_t ra_ = tl::make_rsrc(A + (long)by * BM * GK, (uint32_t)(BM * GK * 2));
  const __amdgpu_buffer_rsrc_t rb_ = tl::make_rsrc(B + (long)bx * BN * GK, (uint32_t)(BN * GK * 2));
  half_t* dwave = smem + wave * 512;
  auto stage = [&](int buf, int slot, int tile) {
    half_t* l = dwave + (buf * 4 + slot) * HALF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int soff = (((slot & 1) * 128 + j * 32) * GK + tile * BK) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(slot < 2 ? ra_ : rb_, (tl::lds_void_t*)(l + j * 2048), 16, voff, soff, 0, 0);
    }
  };
  const int lrow = (lane & 15) * BK;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {((lane >> 4) ^ sw) * 8, ((4 + (lane >> 4)) ^ sw) * 8};
  const int ra = wm * 64, rb = wn * 64;  // piece row offsets inside an A / B slot

  floatx4 acc[2][2][4][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[i][j][m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  F a0[4][2], a1[4][2], b0[4][2], b1[4][2];
  // prologue: tiles 0 and 1 staged (per-tile order A0 B0 B1 A1), tile 0 landed; A0 / B0 of tile
  // 0 read; then A0 of tile 2 (what P3 of tile -1 stages)
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  stage(1, 0, 1);
  stage(1, 2, 1);
  stage(1, 3, 1);
  stage(1, 1, 1);
  tl::wait_vmcnt<16>();
  bar_lgkm();
  read_piece<0 * HALF>(smem, a0, ra, lrow, cx);
  read_piece<2 * HALF>(smem, b0, rb, lrow, cx);
  bar_lgkm();
  stage(0, 0, 2);

// even tile (buffer 0): Q00 Q01 Q11 Q10, reads B1 / A1 / A0' / B1' (next tile), stages
//   B0(t+2) B1(t+2) A1(t+2) A0(t+3)
// odd tile (buffer 1): Q01 Q00 Q10 Q11, reads B0 / A1 / A0'' / B0'' (next tile), stages
//   B1(t+2) B0(t+2) A1(t+2) A0(t+3)
// so four fragment pieces (A0 A1 B0 B1) suffice: every read goes to a piece the current and the
// next quadrant do not use
#define PHASE(BUF, P, T)                                                                          \
  {                                                                                               \
    constexpr int SB = (BUF) * 4 * HALF, SN = ((BUF) ^ 1) * 4 * HALF;                             \
    constexpr bool EV = (BUF) == 0;                                                               \
    if constexpr (P == 0) {                                                                       \
      if (EV) read_piece<SB + 3 * HALF>(smem, b1, rb, lrow, cx);                                  \
      else read_piece<SB + 2 * HALF>(smem, b0, rb, lrow, cx);                                     \
      if ((T) + 2 < NT) stage(BUF, EV ? 2 : 3, (T) + 2);                                          \
      if (EV) mma<0, 0>(a0, b0, acc); else mma<0, 1>(a0, b1, acc);                                \
    } else if constexpr (P == 1) {                                                                \
      read_piece<SB + 1 * HALF>(smem, a1, ra, lrow, cx);                                          \
      if ((T) + 2 < NT) stage(BUF, EV ? 3 : 2, (T) + 2);                                          \
      if (EV) mma<0, 1>(a0, b1, acc); else mma<0, 0>(a0, b0, acc);                                \
      if ((T) + 2 < NT) tl::wait_vmcnt<12>();                                                     \
      else tl::wait_vmcnt<0>();                                                                   \
    } else if constexpr (P == 2) {                                                                \
      read_piece<SN + 0 * HALF>(smem, a0, ra, lrow, cx); /* unconditional: no phi, no copy */    \
      if ((T) + 2 < NT) stage(BUF, 1, (T) + 2);                                                   \
      if (EV) mma<1, 1>(a1, b1, acc); else mma<1, 0>(a1, b0, acc);                                \
    } else {                                                                                      \
      if (EV) read_piece<SN + 3 * HALF>(smem, b1, rb, lrow, cx);                                  \
      else read_piece<SN + 2 * HALF>(smem, b0, rb, lrow, cx);                                     \
      if ((T) + 3 < NT) stage((BUF) ^ 1, 0, (T) + 3);                                             \
      if (EV) mma<1, 0>(a1, b0, acc); else mma<1, 1>(a1, b1, acc);                                \
    }                                                                                             \
    bar_lgkm();                                                                                   \
  }

  for (int t = 0; t < NT; t += 2) {
    PHASE(0, 0, t)
    PHASE(0, 1, t)
    PHASE(0, 2, t)
    PHASE(0, 3, t)
    PHASE(1, 0, t + 1)
    PHASE(1, 1, t + 1)
    PHASE(1, 2, t + 1)
    PHASE(1, 3, t + 1)
  }
#undef PHASE

#if ASM_MFMA
  // the compiler does not know the asm wrote the accumulators with an MFMA: cover the XDL
  // write -> v_accvgpr_read hazard of the last MFMAs before the epilogue reads them
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
#endif
  half_t* Cs = smem;
  constexpr int LDC = BN + 8;
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const floatx4 v = acc[qa][qb][mi][ni];
          half_t o[4] = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
          const int r = qa * 128 + wm * 64 + mi * 16 + (lane & 15);
          const int c = qb * 128 + wn * 64 + ni * 16 + 4 * (lane >> 4);
          tl::store_vec<half_t, 4>(&Cs[r * LDC + c], o);
        }
  tl::sync_threads();
#pragma unroll
  for (int i = 0; i < (BM * BN) / (256 * 8); ++i) {
    const int e = (i * 256 + tid) * 8, r = e / BN, c = e % BN;
    tl::copy_bytes<16>(&C[(long)(by * BM + r) * GN + bx * BN + c], &Cs[r * LDC + c]);
  }
}
