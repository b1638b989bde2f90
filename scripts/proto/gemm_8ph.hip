// Prototype: 256x256x64 fp16 NT GEMM (A [M][K], B [N][K], C [M][N] fp16) with the 8-phase
// quadrant schedule of the MI355X guide (cdna_hip_programming.md "The 256^2 8-phase template",
// T2-T5), compiled through tilelang's postproc hook (scripts/proto/gemm_8ph_ab.py) in place of
// the DSL kernel so it is A/B'd in one process against the DSL schedule and hipBLASLt.
//
// Schedule (one K tile = 4 phases, the loop body = 2 K tiles so every LDS slot address is a
// compile-time constant):
//   * LDS: 2 buffers x 4 half-tile slots of [128 rows][64 k] fp16 (A rows 0-127 / 128-255,
//     B rows 0-127 / 128-255), 16-byte chunks XOR-swizzled by (row >> 1) & 7 on the SOURCE
//     address of the lane-linear LDS-DMA (conflict-free ds_read_b128 for the MFMA pattern).
//   * every phase: all 8 waves compute one 128x128 quadrant of the block tile x K=64 (16 MFMAs
//     per wave, a 64x32 piece); quadrant order (0,0) (0,1) (1,1) (1,0), so the phases read
//     A0+B0 / B1 / A1 / nothing (B0 kept in registers).
//   * each phase stages ONE half-tile (2 global_load_lds per thread) into a slot whose last
//     read was in an earlier phase (retired by that phase's lgkmcnt before its closing barrier):
//     P0: A1 of tile t+1, P1-P3: A0 / B0 / B1 of tile t+2.  Counted vmcnt(6) once per K tile
//     (in P3) leaves the 3 half-tiles of tile t+2 in flight across the barrier.
//   * PRIO: s_setprio(1) around the MFMA cluster (T5); B1: a barrier between the reads + DMA
//     issue and the MFMAs (the guide's two-barrier phase).
//   * STAGGER (needs B1): waves 4-7 run one barrier behind waves 0-3 (the guide template's
//     `if (wr == 1) s_barrier`), so in every barrier interval one half of the workgroup issues its
//     reads + DMAs while the other half runs its MFMA cluster.  A DMA is then visible to the other
//     half one barrier later, so the counted wait moves into every phase: vmcnt(8) (the four newest
//     half-tiles in flight) retires each half-tile two phases before its first read.
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
#define PRIO 1
#endif
#ifndef B1
#define B1 1
#endif
#ifndef ASM_DMA
#define ASM_DMA 0
#endif
#ifndef PRE_B1
#define PRE_B1 0  // 1: P0 also reads B1 (P1 and P3 are then pure-MFMA phases)
#endif
#ifndef YPRIO
#define YPRIO 0  // 1: waves 4-7 run at priority 1 for the whole kernel (guide T5 static form)
#endif
#ifndef STAGGER
#define STAGGER 0
#endif
#ifndef RO
#define RO 0  // 1: pin kk-major read order so the first MFMAs wait for half the reads only
#endif

namespace p8 {
using namespace tl;
typedef mfma_traits<half_t> MT;
typedef MT::frag F;
constexpr int BM = 256, BN = 256, BK = 64;
constexpr int HALF = 128 * BK;  // halfs per half-tile slot (16 KiB)
constexpr int NT = GK / BK;
static_assert(NT % 2 == 0 && NT >= 4, "K tiles: even, >= 4");
static_assert(!STAGGER || B1, "the stagger needs the two-barrier phase");

TL_DEVICE void bar() { asm volatile("s_barrier" ::: "memory"); }

TL_DEVICE void dma16(const half_t* g, half_t* l) {
#if ASM_DMA
  // hidden from the compiler's waitcnt bookkeeping (it would otherwise wait for the DMA before
  // any LDS read it cannot prove disjoint); counted by the explicit vmcnt below
  unsigned keep;
  const unsigned dst = (unsigned)(uintptr_t)(lds_void_t*)l;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
#else
  glds16(g, l);
#endif
}

struct Frags {
  F a[4][2];   // A piece of the current quadrant row: mi x kk
  F b0[2][2];  // B piece, quadrant column 0: ni x kk
  F b1[2][2];  // B piece, quadrant column 1
};

template <int SLOT_OFF>
TL_DEVICE void read_a(const half_t* smem, F (&a)[4][2], int wm, int lrow, const int (&cx)[2]) {
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      a[mi][kk] = *reinterpret_cast<const F*>(smem + SLOT_OFF + (wm * 64 + mi * 16) * BK + lrow + cx[kk]);
}

template <int SLOT_OFF>
TL_DEVICE void read_b(const half_t* smem, F (&b)[2][2], int wn, int lrow, const int (&cx)[2]) {
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      b[ni][kk] = *reinterpret_cast<const F*>(smem + SLOT_OFF + (wn * 32 + ni * 16) * BK + lrow + cx[kk]);
}

// kk-major reads of an A piece and a B piece (RO=1): all kk=0 operands first
template <int A_OFF, int B_OFF>
TL_DEVICE void read_ab_kk(const half_t* smem, F (&a)[4][2], F (&b)[2][2], int wm, int wn, int lrow, const int (&cx)[2]) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
      a[mi][kk] = *reinterpret_cast<const F*>(smem + A_OFF + (wm * 64 + mi * 16) * BK + lrow + cx[kk]);
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
      b[ni][kk] = *reinterpret_cast<const F*>(smem + B_OFF + (wn * 32 + ni * 16) * BK + lrow + cx[kk]);
  }
}

template <int QA, int QB>
TL_DEVICE void mma(const F (&a)[4][2], const F (&b)[2][2], floatx4 (&acc)[2][2][4][2]) {
#if PRIO
  __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) acc[QA][QB][mi][ni] = MT::mma16(b[ni][kk], a[mi][kk], acc[QA][QB][mi][ni]);
#if PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}
}  // namespace p8

extern "C" __global__ void __launch_bounds__(512) gemm_kernel(half_t* __restrict__ A, half_t* __restrict__ B,
                                                              half_t* __restrict__ C) {
  using namespace p8;
  __shared__ __attribute__((aligned(1024))) char tl_smem[135168];
  half_t* smem = reinterpret_cast<half_t*>(tl_smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  int bid = blockIdx.x + blockIdx.y * gridDim.x;
  bid = tl::xcd_remap(bid, gridDim.x * gridDim.y);
  int bx, by;
  tl::rasterize_row<8>(bid, gridDim.x, gridDim.y, bx, by);

  // LDS-DMA: thread tid fills chunks q = j*512 + tid (j = 0, 1) of a half-tile: LDS row q >> 3,
  // position q & 7, holding global chunk (q & 7) ^ ((row >> 1) & 7)
  const int dc = (tid & 7) ^ ((tid >> 4) & 7);
  const long doff0 = (long)(tid >> 3) * GK + dc * 8, doff1 = doff0 + 64L * GK;
  const half_t* Ab = A + (long)by * BM * GK;
  const half_t* Bb = B + (long)bx * BN * GK;
  half_t* dwave = smem + wave * 512;
  auto stage = [&](int buf, int slot, int tile) {
    const half_t* g = (slot < 2 ? Ab + (long)slot * 128 * GK : Bb + (long)(slot - 2) * 128 * GK) + tile * BK;
    half_t* l = dwave + (buf * 4 + slot) * HALF;
    dma16(g + doff0, l);
    dma16(g + doff1, l + 4096);
  };
  // fragment reads: row r0 + (lane & 15), chunk kk*4 + (lane >> 4), swizzled by (lane >> 1) & 7
  const int lrow = (lane & 15) * BK;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {(((lane >> 4)) ^ sw) * 8, ((4 + (lane >> 4)) ^ sw) * 8};

  floatx4 acc[2][2][4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[i][j][m][n] = floatx4{0.f, 0.f, 0.f, 0.f};

  // prologue: tile 0 (all four slots of buffer 0) + tile 1's A0 / B0 / B1 (what P1-P3 of tile -1
  // would have staged); tile 0 landed, 3 half-tiles in flight
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 3, 0);
  stage(0, 1, 0);
  stage(1, 0, 1);
  stage(1, 2, 1);
  stage(1, 3, 1);
  tl::wait_vmcnt<6>();
  bar();

  Frags f;
  if (STAGGER && wave >= 4) bar();
#if YPRIO
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
#endif
#define PHASE(BUF, P, T)                                                                          \
  {                                                                                               \
    constexpr int SB = (BUF) * 4 * HALF;                                                          \
    if constexpr (P == 0) {                                                                       \
      if (RO) {                                                                                   \
        read_ab_kk<SB + 0 * HALF, SB + 2 * HALF>(smem, f.a, f.b0, wm, wn, lrow, cx);              \
      } else {                                                                                    \
        read_a<SB + 0 * HALF>(smem, f.a, wm, lrow, cx);                                           \
        read_b<SB + 2 * HALF>(smem, f.b0, wn, lrow, cx);                                          \
      }                                                                                           \
      if (PRE_B1) read_b<SB + 3 * HALF>(smem, f.b1, wn, lrow, cx);                                \
      if ((T) + 1 < NT) stage((BUF) ^ 1, 1, (T) + 1);                                             \
    } else if constexpr (P == 1) {                                                                \
      if (!PRE_B1) read_b<SB + 3 * HALF>(smem, f.b1, wn, lrow, cx);                               \
      if ((T) + 2 < NT) stage(BUF, 0, (T) + 2);                                                   \
    } else if constexpr (P == 2) {                                                                \
      read_a<SB + 1 * HALF>(smem, f.a, wm, lrow, cx);                                             \
      if ((T) + 2 < NT) stage(BUF, 2, (T) + 2);                                                   \
    } else {                                                                                      \
      if ((T) + 2 < NT) stage(BUF, 3, (T) + 2);                                                   \
    }                                                                                             \
    if (STAGGER) tl::wait_lgkmcnt<0>(); /* WAR: the other half restages a slot read here */     \
    if (B1) bar();                                                                                \
    if constexpr (P == 0) mma<0, 0>(f.a, f.b0, acc);                                              \
    else if constexpr (P == 1) mma<0, 1>(f.a, f.b1, acc);                                         \
    else if constexpr (P == 2) mma<1, 1>(f.a, f.b1, acc);                                         \
    else mma<1, 0>(f.a, f.b0, acc);                                                               \
    if (STAGGER) {                                                                                \
      if ((T) + 2 < NT) tl::wait_vmcnt<8>();                                                      \
      else tl::wait_vmcnt<0>();                                                                   \
    } else if constexpr (P == 3) {                                                                \
      if ((T) + 2 < NT) tl::wait_vmcnt<6>();                                                      \
      else if ((T) + 1 < NT) tl::wait_vmcnt<0>();                                                 \
    }                                                                                             \
    bar();                                                                                        \
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
  if (STAGGER && wave < 4) bar();

  // epilogue: fragments -> row-padded LDS tile -> 16-byte row stores
  half_t* Cs = smem;
  constexpr int LDC = BN + 8;
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const floatx4 v = acc[qa][qb][mi][ni];
          half_t o[4] = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
          const int r = qa * 128 + wm * 64 + mi * 16 + (lane & 15);
          const int c = qb * 128 + wn * 32 + ni * 16 + 4 * (lane >> 4);
          tl::store_vec<half_t, 4>(&Cs[r * LDC + c], o);
        }
  tl::sync_threads();
#pragma unroll
  for (int i = 0; i < (BM * BN) / (512 * 8); ++i) {
    const int e = (i * 512 + tid) * 8, r = e / BN, c = e % BN;
    tl::copy_bytes<16>(&C[(long)(by * BM + r) * GN + bx * BN + c], &Cs[r * LDC + c]);
  }
}
