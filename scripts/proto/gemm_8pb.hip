// Prototype: the 8-phase quadrant GEMM (gemm_8ph.hip) on the DSL's standard 4x2 wave layout
// (each wave a contiguous 64x128 piece of the 256x256 tile, accumulator index mi*8 + ni as
// tl::gemm_ss), so it can replace the K loop of a DSL kernel without changing the C fragment.
//
//   * a phase computes quadrant (qa, qb) of EVERY wave's piece: rows wm*64 + qa*32 + [0, 32),
//     cols wn*128 + qb*64 + [0, 64) -- 2 x 4 MFMA tiles x K=64 = 16 MFMAs per wave.
//   * so a phase reads one A half-tile qa = the block rows {wm*64 + qa*32 + r} (four 32-row
//     groups) and one B half-tile qb = the block cols {wn*128 + qb*64 + c} (two 64-col groups):
//     "interleaved" half-tiles, gathered by the per-lane LDS-DMA source address.
//   * staging, waits and barriers as gemm_8ph.hip (slots A0 A1 B0 B1, one half-tile per phase,
//     vmcnt(6) once per K tile); DMA through buffer resources (32-bit per-lane offsets).
//   NN=1: B is [K][N] (N-contiguous): a B slot is [64 k][128 n] read with ds_read_b64_tr_b16,
//   16-byte chunks XOR-swizzled by 2*((k & 3) | ((k >> 3 & 1) << 2)) (the 8 rows one 32-lane
//   group reads land in 8 distinct 32-byte bank windows).
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
#ifndef NN
#define NN 0
#endif
#ifndef B1
#define B1 0
#endif
#ifndef YPRIO
#define YPRIO 0  // 1: waves 4-7 at issue priority 1 for the whole kernel (guide T5 static form)
#endif
#ifndef SINGLE
#define SINGLE 0  // 1: one barrier per K tile, the whole next tile staged in phase 0 (classic 2-stage)
#endif
#ifndef PREB1
#define PREB1 0  // 1 (with MERGE): B1 read in phase 1 into a second B register set, so the MFMAs after
                 // the mid-tile barrier start on resident operands
#endif
#ifndef MERGE
#define MERGE 0  // 1: two barriers per K tile (phases paired), A0/B0 restaged after the pair
#endif
#ifndef RPIPE
#define RPIPE 0  // 1: fragments read one phase ahead (quadrant order alternating by tile parity)
#endif

namespace pb {
using namespace tl;
typedef mfma_traits<half_t> MT;
typedef MT::frag F;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HALF = 128 * BK;  // halfs per half-tile slot (16 KiB)
constexpr int NT = GK / BK;
static_assert(NT % 2 == 0 && NT >= 4, "K tiles: even, >= 4");

TL_DEVICE void bar() { asm volatile("s_barrier" ::: "memory"); }

TL_DEVICE int nn_h(int k) { return (k & 3) | (((k >> 3) & 1) << 2); }

// A piece of quadrant row qa: 2 m-tiles x 2 k-steps, LDS rows wm*32 + mi*16 + (lane & 15)
template <int SLOT_OFF>
TL_DEVICE void read_a(const half_t* smem, F (&a)[2][2], int wm, int lrow, const int (&cx)[2]) {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      a[mi][kk] = *reinterpret_cast<const F*>(smem + SLOT_OFF + (wm * 32 + mi * 16) * BK + lrow + cx[kk]);
}

// B piece of quadrant column qb: 4 n-tiles x 2 k-steps
template <int SLOT_OFF>
TL_DEVICE void read_b(const half_t* smem, F (&b)[4][2], int wn, int lane, int lrow, const int (&cx)[2]) {
#if NN
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int col = wn * 64 + ni * 16 + 4 * p;
      const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
      const half_t* p0 = smem + SLOT_OFF + r0 * 128 + (((col >> 3) ^ (2 * nn_h(r0))) << 3) + (col & 7);
      const half_t* p1 = smem + SLOT_OFF + r1 * 128 + (((col >> 3) ^ (2 * nn_h(r1))) << 3) + (col & 7);
      shortx4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) shortx4*)(
          (__attribute__((address_space(3))) char*)(p0)));
      shortx4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) shortx4*)(
          (__attribute__((address_space(3))) char*)(p1)));
      b[ni][kk] = __builtin_bit_cast(F, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
#else
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      b[ni][kk] = *reinterpret_cast<const F*>(smem + SLOT_OFF + (wn * 64 + ni * 16) * BK + lrow + cx[kk]);
#endif
}

template <int QA, int QB>
TL_DEVICE void mma(const F (&a)[2][2], const F (&b)[4][2], floatx4 (&acc)[4][8]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[QA * 2 + mi][QB * 4 + ni] = MT::mma16(b[ni][kk], a[mi][kk], acc[QA * 2 + mi][QB * 4 + ni]);
}
}  // namespace pb

extern "C" __global__ void __launch_bounds__(512) gemm_kernel(half_t* __restrict__ A, half_t* __restrict__ B,
                                                              half_t* __restrict__ C) {
  using namespace pb;
  __shared__ __attribute__((aligned(1024))) char tl_smem[135168];
  half_t* smem = reinterpret_cast<half_t*>(tl_smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int bid = blockIdx.x + blockIdx.y * gridDim.x;
  bid = tl::xcd_remap(bid, gridDim.x * gridDim.y);
  int bx, by;
  tl::rasterize_row<8>(bid, gridDim.x, gridDim.y, bx, by);

  // A half-tile qa (and NT B half-tile qb): chunk q = j*512 + tid -> LDS row r = j*64 + (tid >> 3),
  // position tid & 7 holding global chunk (tid & 7) ^ ((tid >> 4) & 7);
  // A row of LDS row r: (r >> 5) * 64 + qa * 32 + (r & 31);  NT B row: (r >> 6) * 128 + qb * 64 + (r & 63)
  const int dc = (tid & 7) ^ ((tid >> 4) & 7);
  const int rr = tid >> 3;
  // buffer-resource DMA: ONE per-lane 32-bit byte offset per operand; the slot / piece / K-tile
  // parts are constants or SGPRs (A: LDS row j*64 + rr of half qa is block row
  // (2j + (rr >> 5)) * 64 + qa * 32 + (rr & 31) = row(j=0, qa=0) + 128 j + 32 qa)
  const uint32_t voffa = (uint32_t)((((rr >> 5) * 64 + (rr & 31)) * GK + dc * 8) * 2);
  auto soffa = [](int qa, int j) { return (j * 128 + qa * 32) * GK * 2; };
#if NN
  // B slot [64 k][128 n]: chunk q = j*512 + tid -> k row j*32 + (tid >> 4), position tid & 15
  // holding n-chunk c = (tid & 15) ^ 2 h(k); n of chunk c: (c >> 3) * 128 + qb * 64 + (c & 7) * 8
  // (h(k) is the same for j = 0, 1: k differs by 32)
  const int kb = tid >> 4;
  const int cb = (tid & 15) ^ (2 * nn_h(kb));
  const uint32_t voffb = (uint32_t)((kb * GN + (cb >> 3) * 128 + (cb & 7) * 8) * 2);
  auto soffb = [](int qb, int j) { return (j * 32 * GN + qb * 64) * 2; };
  const __amdgpu_buffer_rsrc_t rb_ = tl::make_rsrc(B + (long)bx * BN, (uint32_t)(((long)(GK - 1) * GN + BN) * 2));
  constexpr int BSTEP = BK * GN * 2;  // bytes of one K tile of B
#else
  // NT B: LDS row j*64 + rr of half qb is block col j*128 + qb*64 + rr
  const uint32_t voffb = (uint32_t)((rr * GK + dc * 8) * 2);
  auto soffb = [](int qb, int j) { return (j * 128 + qb * 64) * GK * 2; };
  const __amdgpu_buffer_rsrc_t rb_ = tl::make_rsrc(B + (long)bx * BN * GK, (uint32_t)(BN * GK * 2));
  constexpr int BSTEP = BK * 2;
#endif
  const __amdgpu_buffer_rsrc_t ra_ = tl::make_rsrc(A + (long)by * BM * GK, (uint32_t)(BM * GK * 2));
  half_t* dwave = smem + wave * 512;
  auto stage = [&](int buf, int slot, int tile) {
    tl::lds_void_t* l = (tl::lds_void_t*)(dwave + (buf * 4 + slot) * HALF);
    tl::lds_void_t* l1 = (tl::lds_void_t*)(dwave + (buf * 4 + slot) * HALF + 4096);
    if (slot < 2) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, l, 16, voffa, tile * BK * 2 + soffa(slot, 0), 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_, l1, 16, voffa, tile * BK * 2 + soffa(slot, 1), 0, 0);
    } else {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb_, l, 16, voffb, tile * BSTEP + soffb(slot - 2, 0), 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb_, l1, 16, voffb, tile * BSTEP + soffb(slot - 2, 1), 0, 0);
    }
  };
  const int lrow = (lane & 15) * BK;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {((lane >> 4) ^ sw) * 8, ((4 + (lane >> 4)) ^ sw) * 8};

  floatx4 acc[4][8];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

#if RPIPE
  // tiles 0 and 1 staged, tile 0 landed, A0 / B0 of tile 0 read, then B0 of tile 2 (what P3 of
  // tile -1 stages)
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  stage(0, 3, 0);
  stage(1, 0, 1);
  stage(1, 2, 1);
  stage(1, 1, 1);
  stage(1, 3, 1);
  tl::wait_vmcnt<8>();
  bar();
#elif SINGLE
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  stage(0, 3, 0);
  tl::wait_vmcnt<0>();
  bar();
#else
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  stage(0, 3, 0);
  stage(1, 0, 1);  // what P1-P3 of tile -1 stage
  stage(1, 2, 1);
  stage(1, 1, 1);
  tl::wait_vmcnt<6>();
  bar();
#endif

  // quadrant order (0,0) (1,0) (1,1) (0,1): reads A0+B0 / A1 / B1 / none -- both A pieces and
  // ONE B piece in registers; slots are restaged after their last read: P0 B1 of tile t+1,
  // P1 A0, P2 B0, P3 A1 of tile t+2
  F fa0[2][2], fa1[2][2], fb[4][2];
#if YPRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#if RPIPE
  F fb1[4][2];
#endif
#if PREB1
  F fbb[4][2];
#endif
#if PREB1
#define FBB fbb
#else
#define FBB fb
#endif
#if !RPIPE
#define PHASE(BUF, P, T)                                                                          \
  {                                                                                               \
    constexpr int SB = (BUF) * 4 * HALF;                                                          \
    if constexpr (P == 0) {                                                                       \
      read_a<SB + 0 * HALF>(smem, fa0, wm, lrow, cx);                                             \
      read_b<SB + 2 * HALF>(smem, fb, wn, lane, lrow, cx);                                        \
      if (SINGLE) {                                                                               \
        if ((T) + 1 < NT) {                                                                       \
          stage((BUF) ^ 1, 0, (T) + 1); stage((BUF) ^ 1, 2, (T) + 1);                             \
          stage((BUF) ^ 1, 1, (T) + 1); stage((BUF) ^ 1, 3, (T) + 1);                             \
        }                                                                                         \
      } else if ((T) + 1 < NT) stage((BUF) ^ 1, 3, (T) + 1);                                      \
    } else if constexpr (P == 1) {                                                                \
      read_a<SB + 1 * HALF>(smem, fa1, wm, lrow, cx);                                             \
      if (PREB1) read_b<SB + 3 * HALF>(smem, FBB, wn, lane, lrow, cx);                            \
      if (!SINGLE && !MERGE && (T) + 2 < NT) stage(BUF, 0, (T) + 2);                              \
    } else if constexpr (P == 2) {                                                                \
      if (!PREB1) read_b<SB + 3 * HALF>(smem, fb, wn, lane, lrow, cx);                            \
      if (!SINGLE && MERGE && (T) + 2 < NT) stage(BUF, 0, (T) + 2);                               \
      if (!SINGLE && (T) + 2 < NT) stage(BUF, 2, (T) + 2);                                        \
    } else {                                                                                      \
      if (!SINGLE && (T) + 2 < NT) stage(BUF, 1, (T) + 2);                                        \
    }                                                                                             \
    if (B1) bar();                                                                                \
    if constexpr (P == 0) mma<0, 0>(fa0, fb, acc);                                                \
    else if constexpr (P == 1) mma<1, 0>(fa1, fb, acc);                                           \
    else if constexpr (P == 2) mma<1, 1>(fa1, FBB, acc);                                          \
    else mma<0, 1>(fa0, FBB, acc);                                                                \
    if constexpr (P == 3) {                                                                       \
      if (SINGLE) tl::wait_vmcnt<0>();                                                            \
      else if ((T) + 2 < NT) tl::wait_vmcnt<6>();                                                 \
      else if ((T) + 1 < NT) tl::wait_vmcnt<0>();                                                 \
    }                                                                                             \
    if (SINGLE ? P == 3 : (!MERGE || P == 1 || P == 3)) bar();                                    \
  }

#else
  // RPIPE: the operands of phase p+1 are read during phase p (every phase closes with
  // lgkmcnt(0) + s_barrier, so a slot read in phase q is restaged from q+1):
  //   even tile: Q00 (A0,B0) read A1 | Q10 (A1,B0) read B1 | Q11 (A1,B1) read B0' | Q01 (A0,B1) read A1'
  //   odd tile:  Q10 (A1,B0) read A0 | Q00 (A0,B0) read B1 | Q01 (A0,B1) read B0' | Q11 (A1,B1) read A0'
  //   staging:   even P0 A0(t+2) P1 A1(t+2) P2 B1(t+2) P3 B0(t+3);  odd P0 A1(t+2) P1 A0(t+2)
  //              P2 B1(t+2) P3 B0(t+3);  P1 waits vmcnt(6) (tile t+1 landed)
#define PHASE(BUF, P, T)                                                                          \
  {                                                                                               \
    constexpr int SB = (BUF) * 4 * HALF, SN = ((BUF) ^ 1) * 4 * HALF;                             \
    constexpr bool EV = (BUF) == 0;                                                               \
    if constexpr (P == 0) {                                                                       \
      if (EV) read_a<SB + 1 * HALF>(smem, fa1, wm, lrow, cx);                                     \
      else read_a<SB + 0 * HALF>(smem, fa0, wm, lrow, cx);                                        \
      if ((T) + 2 < NT) stage(BUF, EV ? 0 : 1, (T) + 2);                                          \
      if (EV) mma<0, 0>(fa0, fb, acc); else mma<1, 0>(fa1, fb, acc);                              \
    } else if constexpr (P == 1) {                                                                \
      read_b<SB + 3 * HALF>(smem, fb1, wn, lane, lrow, cx);                                       \
      if ((T) + 2 < NT) stage(BUF, EV ? 1 : 0, (T) + 2);                                          \
      if (EV) mma<1, 0>(fa1, fb, acc); else mma<0, 0>(fa0, fb, acc);                              \
      if ((T) + 2 < NT) tl::wait_vmcnt<6>();                                                      \
      else tl::wait_vmcnt<0>();                                                                   \
    } else if constexpr (P == 2) {                                                                \
      read_b<SN + 2 * HALF>(smem, fb, wn, lane, lrow, cx);                                        \
      if ((T) + 2 < NT) stage(BUF, 3, (T) + 2);                                                   \
      if (EV) mma<1, 1>(fa1, fb1, acc); else mma<0, 1>(fa0, fb1, acc);                            \
    } else {                                                                                      \
      if (EV) read_a<SN + 1 * HALF>(smem, fa1, wm, lrow, cx);                                     \
      else read_a<SN + 0 * HALF>(smem, fa0, wm, lrow, cx);                                        \
      if ((T) + 3 < NT) stage((BUF) ^ 1, 2, (T) + 3);                                             \
      if (EV) mma<0, 1>(fa0, fb1, acc); else mma<1, 1>(fa1, fb1, acc);                            \
    }                                                                                             \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");                              \
  }
#endif

#if RPIPE
  read_a<0 * HALF>(smem, fa0, wm, lrow, cx);
  read_b<2 * HALF>(smem, fb, wn, lane, lrow, cx);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  stage(0, 2, 2);
#endif
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

  half_t* Cs = smem;
  constexpr int LDC = BN + 8;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      const floatx4 v = acc[mi][ni];
      half_t o[4] = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
      const int r = wm * 64 + mi * 16 + (lane & 15);
      const int c = wn * 128 + ni * 16 + 4 * (lane >> 4);
      tl::store_vec<half_t, 4>(&Cs[r * LDC + c], o);
    }
  tl::sync_threads();
#pragma unroll
  for (int i = 0; i < (BM * BN) / (512 * 8); ++i) {
    const int e = (i * 512 + tid) * 8, r = e / BN, c = e % BN;
    tl::copy_bytes<16>(&C[(long)(by * BM + r) * GN + bx * BN + c], &Cs[r * LDC + c]);
  }
}
