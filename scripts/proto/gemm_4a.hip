// Prototype: 256x256x64 NT GEMM (A [M][K], B [N][K], C [M][N] fp16) on FOUR waves (one per
// SIMD) in the DSL's 2x2 wave layout -- wave (wm, wn) owns the contiguous 128x128 piece, whose 256
// fp32 accumulators live in the accumulator file at LITERAL registers (scripts/proto/agpr_mfma.h:
// asm MFMAs clobbering their own a[R:R+3], so hipcc neither renames nor spills them; the
// measured hipBLASLt NT kernel is this shape: 4 waves, MFMA busy 0.85 of CU busy vs 0.67 for the
// 8-wave quad loop, profiles/r5/pmc_quad/).  A/B'd through scripts/proto/gemm_8ph_ab.py.
//
//   * LDS: 2 buffers x 4 interleaved half-tile slots [128][64] (A half qa = block rows
//     {wm*128 + qa*64 + r}, B half qb = block cols {wn*128 + qb*64 + c}), chunks XOR-swizzled by
//     (row >> 1) & 7 on the LDS-DMA source; buffer-resource DMA, 4 per thread per half-tile.
//   * phase = one 64x64 quadrant of the wave's piece x K=64 (32 MFMAs), on fragments read in the
//     phase before, while the next phase's fragments are read (orders at PHASE, alternating by
//     tile parity so four register pieces A0 A1 B0 B1 suffice); every phase closes with
//     lgkmcnt(0) + s_barrier; P1 waits vmcnt(12): the next tile landed, 3 half-tiles in flight.
#include "tl/tl.h"
#include "agpr_mfma.h"

#ifndef GM
#define GM 4096
#endif
#ifndef GN
#define GN 4096
#endif
#ifndef GK
#define GK 4096
#endif

namespace p4a {
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

// quadrant (QA, QB): accumulator tile (QA*4 + mi, QB*4 + ni) of the wave's 8x8 -> a[(mi_g*8 + ni_g)*4]
template <int QA, int QB, int KK, int MI, int NI>
TL_DEVICE void mma1(const F (&a)[4][2], const F (&b)[4][2]) {
  agpr::acc<((QA * 4 + MI) * 8 + QB * 4 + NI) * 4>::mma(b[NI][KK], a[MI][KK]);
}
template <int QA, int QB, int KK, int MI>
TL_DEVICE void mma_row(const F (&a)[4][2], const F (&b)[4][2]) {
  mma1<QA, QB, KK, MI, 0>(a, b);
  mma1<QA, QB, KK, MI, 1>(a, b);
  mma1<QA, QB, KK, MI, 2>(a, b);
  mma1<QA, QB, KK, MI, 3>(a, b);
}
template <int QA, int QB>
TL_DEVICE void mma(const F (&a)[4][2], const F (&b)[4][2]) {
  mma_row<QA, QB, 0, 0>(a, b);
  mma_row<QA, QB, 0, 1>(a, b);
  mma_row<QA, QB, 0, 2>(a, b);
  mma_row<QA, QB, 0, 3>(a, b);
  mma_row<QA, QB, 1, 0>(a, b);
  mma_row<QA, QB, 1, 1>(a, b);
  mma_row<QA, QB, 1, 2>(a, b);
  mma_row<QA, QB, 1, 3>(a, b);
}

template <int I> TL_DEVICE void zero_all() {
  if constexpr (I < 256) {
    agpr::acc<I>::zero();
    zero_all<I + 4>();
  }
}
template <int I> TL_DEVICE void read_all(floatx4* out) {
  if constexpr (I < 256) {
    out[I / 4] = agpr::acc<I>::read();
    read_all<I + 4>(out);
  }
}
}  // namespace p4a

extern "C" __global__ void __launch_bounds__(256) gemm_kernel(half_t* __restrict__ A, half_t* __restrict__ B,
                                                              half_t* __restrict__ C) {
  using namespace p4a;
  __shared__ __attribute__((aligned(1024))) char tl_smem[135168];
  half_t* smem = reinterpret_cast<half_t*>(tl_smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int bid = blockIdx.x + blockIdx.y * gridDim.x;
  bid = tl::xcd_remap(bid, gridDim.x * gridDim.y);
  int bx, by;
  tl::rasterize_row<8>(bid, gridDim.x, gridDim.y, bx, by);

  // DMA: chunk q = j*256 + tid (j = 0..3) -> LDS row j*32 + rr, position tid & 7 holding global
  // chunk (tid & 7) ^ ((tid >> 4) & 7); half q' row j*32 + rr = block row/col
  // (j >> 1) * 128 + q' * 64 + (j & 1) * 32 + rr
  const int rr = tid >> 3;
  const int dc = (tid & 7) ^ ((tid >> 4) & 7);
  const uint32_t voffa = (uint32_t)((rr * GK + dc * 8) * 2);
  const __amdgpu_buffer_rsrc_t ra = tl::make_rsrc(A + (long)by * BM * GK, (uint32_t)(BM * GK * 2));
  const __amdgpu_buffer_rsrc_t rb = tl::make_rsrc(B + (long)bx * BN * GK, (uint32_t)(BN * GK * 2));
  half_t* dwave = smem + wave * 512;
  auto stage = [&](int buf, int slot, int tile) {
    half_t* l = dwave + (buf * 4 + slot) * HALF;
    const int q = slot & 1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int soff = (((j >> 1) * 128 + q * 64 + (j & 1) * 32) * GK + tile * BK) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(slot < 2 ? ra : rb, (tl::lds_void_t*)(l + j * 2048), 16, voffa, soff,
                                                0, 0);
    }
  };
  const int lrow = (lane & 15) * BK;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {((lane >> 4) ^ sw) * 8, ((4 + (lane >> 4)) ^ sw) * 8};
  const int ra0 = wm * 64, rb0 = wn * 64;  // piece row offsets inside an A / B slot

  zero_all<0>();
  asm volatile("s_nop 2" ::: "memory");

  F a0[4][2], a1[4][2], b0[4][2], b1[4][2];
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
  read_piece<0 * HALF>(smem, a0, ra0, lrow, cx);
  read_piece<2 * HALF>(smem, b0, rb0, lrow, cx);
  bar_lgkm();
  stage(0, 0, 2);

// even tile (buffer 0): Q00 Q01 Q11 Q10 reading B1 / A1 / A0' / B1' ; odd: Q01 Q00 Q10 Q11 reading
// B0 / A1 / A0'' / B0''; staging B0|B1 (t+2), B1|B0 (t+2), A1 (t+2), A0 (t+3)
#define PHASE(BUF, P, T)                                                                          \
  {                                                                                               \
    constexpr int SB = (BUF) * 4 * HALF, SN = ((BUF) ^ 1) * 4 * HALF;                             \
    constexpr bool EV = (BUF) == 0;                                                               \
    if constexpr (P == 0) {                                                                       \
      if (EV) read_piece<SB + 3 * HALF>(smem, b1, rb0, lrow, cx);                                 \
      else read_piece<SB + 2 * HALF>(smem, b0, rb0, lrow, cx);                                    \
      if ((T) + 2 < NT) stage(BUF, EV ? 2 : 3, (T) + 2);                                          \
      if (EV) mma<0, 0>(a0, b0); else mma<0, 1>(a0, b1);                                          \
    } else if constexpr (P == 1) {                                                                \
      read_piece<SB + 1 * HALF>(smem, a1, ra0, lrow, cx);                                         \
      if ((T) + 2 < NT) stage(BUF, EV ? 3 : 2, (T) + 2);                                          \
      if (EV) mma<0, 1>(a0, b1); else mma<0, 0>(a0, b0);                                          \
      if ((T) + 2 < NT) tl::wait_vmcnt<12>();                                                     \
      else tl::wait_vmcnt<0>();                                                                   \
    } else if constexpr (P == 2) {                                                                \
      read_piece<SN + 0 * HALF>(smem, a0, ra0, lrow, cx);                                         \
      if ((T) + 2 < NT) stage(BUF, 1, (T) + 2);                                                   \
      if (EV) mma<1, 1>(a1, b1); else mma<1, 0>(a1, b0);                                          \
    } else {                                                                                      \
      if (EV) read_piece<SN + 3 * HALF>(smem, b1, rb0, lrow, cx);                                 \
      else read_piece<SN + 2 * HALF>(smem, b0, rb0, lrow, cx);                                    \
      if ((T) + 3 < NT) stage((BUF) ^ 1, 0, (T) + 3);                                             \
      if (EV) mma<1, 0>(a1, b0); else mma<1, 1>(a1, b1);                                          \
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

  // XDL write -> v_accvgpr_read: the last MFMAs' results settle before the epilogue reads them
  asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");
  floatx4 acc[64];
  read_all<0>(acc);
  half_t* Cs = smem;
  constexpr int LDC = BN + 8;
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const floatx4 v = acc[mi * 8 + ni];
      half_t o[4] = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
      const int r = wm * 128 + mi * 16 + (lane & 15);
      const int c = wn * 128 + ni * 16 + 4 * (lane >> 4);
      tl::store_vec<half_t, 4>(&Cs[r * LDC + c], o);
    }
  tl::sync_threads();
#pragma unroll
  for (int i = 0; i < (BM * BN) / (256 * 8); ++i) {
    const int e = (i * 256 + tid) * 8, r = e / BN, c = e % BN;
    tl::copy_bytes<16>(&C[(long)(by * BM + r) * GN + bx * BN + c], &Cs[r * LDC + c]);
  }
}
