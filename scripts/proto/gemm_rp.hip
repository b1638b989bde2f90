// Prototype: 256x256x64 fp16 GEMM main-loop variants (A [M][K], B [K][N], C [M][N] fp16).
// Compiled through tilelang's postproc hook (scripts/proto/gemm_rp_ab.py) in place of the
// DSL-generated kernel so the variants are A/B'd in one process against hipBLASLt.
//   WAVES_M   4 -> 4x2 waves (64x128 per wave), 2 -> 2x4 waves (128x64 per wave)
//   PREFETCH 0 -> read the half-tile's fragments after its barrier (current DSL schedule)
//            1 -> fragments of half-tile h+1 are read while half-tile h's MFMAs run
//   ILV      sched_group_barrier interleave of ds_read / MFMA (PREFETCH=1 only)
//   PRIO     s_setprio(1) around the MFMA cluster
#include "tl/tl.h"

#ifndef WAVES_M
#define WAVES_M 4
#endif
#ifndef PREFETCH
#define PREFETCH 1
#endif
#ifndef ILV
#define ILV 1
#endif
#ifndef PRIO
#define PRIO 0
#endif
#ifndef YOUNG_PRIO
#define YOUNG_PRIO 0
#endif
#ifndef GM
#define GM 4096
#endif
#ifndef GN
#define GN 4096
#endif
#ifndef GK
#define GK 4096
#endif

namespace proto {
using namespace tl;
typedef mfma_traits<half_t> MT;
typedef MT::frag F;
constexpr int BM = 256, BN = 256, KH = 32;
constexpr int WARPS_M = WAVES_M, WARPS_N = 8 / WAVES_M;
constexpr int WM = BM / WARPS_M, WN = BN / WARPS_N, M_REP = WM / 16, N_REP = WN / 16;
constexpr uint32_t SWZ_A = 48u, SWZ_B = 16912u;  // the DSL's conflict-free swizzles
constexpr int SLOT = (BM * KH + KH * BN);        // halfs per half-tile slot (A then B)
constexpr int NLOAD = M_REP + 2 * N_REP;         // ds_read instructions per half-tile

struct Frags {
  F a[M_REP];
  F b[N_REP];
};

TL_DEVICE void load_frags(const half_t* __restrict__ As, const half_t* __restrict__ Bs, Frags& __restrict__ f, int wm, int wn, int lane) {
#pragma unroll
  for (int mi = 0; mi < M_REP; ++mi) f.a[mi] = ld_operand<half_t, BM, KH, SWZ_A, false, 0>(As, wm * WM + mi * 16, 0, lane);
#pragma unroll
  for (int ni = 0; ni < N_REP; ++ni) f.b[ni] = ld_operand<half_t, KH, BN, SWZ_B, true, 0>(Bs, wn * WN + ni * 16, 0, lane);
}

TL_DEVICE void mma(const Frags& f, floatx4* acc) {
#pragma unroll
  for (int ni = 0; ni < N_REP; ++ni)
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi) acc[mi * N_REP + ni] = MT::mma16(f.b[ni], f.a[mi], acc[mi * N_REP + ni]);
}

TL_DEVICE void interleave() {
#if ILV
  __builtin_amdgcn_sched_group_barrier(0x020, 4, 0);  // the half-tile's LDS-DMA issues first
#pragma unroll
  for (int i = 0; i < NLOAD; ++i) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 ds_read
  }
  __builtin_amdgcn_sched_group_barrier(0x008, M_REP * N_REP - NLOAD, 0);
#endif
}

// per-thread DMA source offsets (elements) of the two 16-byte pieces of an A / B half-tile
struct Dma {
  long a[2], b[2];
  TL_DEVICE Dma(int by, int bx, int tid) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int c = r * 512 + tid;
      const int ra = c >> 2, ca = (c & 3) ^ (((ra >> 2) & 1) << 1);
      a[r] = (long)(by * BM + ra) * GK + ca * 8;
      const int rb = c >> 5;
      const int sw = ((rb & 1) << 1) ^ (((rb >> 1) & 1) << 2) ^ (((rb >> 3) & 1) << 3);
      const int cb = (c & 31) ^ sw;
      b[r] = (long)rb * GN + bx * BN + cb * 8;
    }
  }
};

TL_DEVICE void issue(const half_t* A, const half_t* B, const Dma& d, int h, half_t* slot, int wave, int lane) {
  const long ka = (long)h * KH, kb = (long)h * KH * GN;
#pragma unroll
  for (int r = 0; r < 2; ++r) glds16(A + d.a[r] + ka, slot + ((r * 8 + wave) * 64) * 8);
#pragma unroll
  for (int r = 0; r < 2; ++r) glds16(B + d.b[r] + kb, slot + BM * KH + ((r * 8 + wave) * 64) * 8);
}

TL_DEVICE void prio_on() {
#if PRIO
  __builtin_amdgcn_s_setprio(1);
#endif
}
TL_DEVICE void prio_off() {
#if PRIO
  __builtin_amdgcn_s_setprio(0);
#endif
}
}  // namespace proto

extern "C" __global__ void __launch_bounds__(512) gemm_kernel(half_t* __restrict__ A, half_t* __restrict__ B,
                                                              half_t* __restrict__ C) {
  using namespace proto;
  __shared__ __attribute__((aligned(1024))) char tl_smem[135168];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WARPS_N, wn = wave % WARPS_N;
  int bid = blockIdx.x + blockIdx.y * gridDim.x;
  bid = tl::xcd_remap(bid, gridDim.x * gridDim.y);
  int bx, by;
  tl::rasterize_row<8>(bid, gridDim.x, gridDim.y, bx, by);
  half_t* smem = reinterpret_cast<half_t*>(tl_smem);
  floatx4 acc[M_REP * N_REP];
#pragma unroll
  for (int i = 0; i < M_REP * N_REP; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  const Dma d(by, bx, tid);
  constexpr int NH = GK / KH;  // half-tiles
#if YOUNG_PRIO
  if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);  // guide T5 static form
#endif
#if PREFETCH
  // Two K-half banks (even halves in bank 0, odd halves in bank 1), each double-buffered by
  // tile parity: a step refills the slot of ITS OWN bank that the previous step read, and reads
  // the other bank, so every ds_read provably misses the LDS-DMA just issued (the compiler can
  // then keep its counted waits instead of a vmcnt(0) before the first read of each step).
  // At half h the fragments of h are already in registers (read during h-1).
  half_t* bank0 = smem;             // [2][SLOT]: half 0 of tiles k%2
  half_t* bank1 = smem + 2 * SLOT;  // [2][SLOT]: half 1 of tiles k%2
  constexpr int NT = GK / (2 * KH);
  issue(A, B, d, 0, bank0, wave, lane);
  issue(A, B, d, 1, bank1, wave, lane);
  issue(A, B, d, 2, bank0 + SLOT, wave, lane);
  issue(A, B, d, 3, bank1 + SLOT, wave, lane);
  Frags f0, f1;
  tl::wait_vmcnt<12>();
  tl::barrier_raw();
  load_frags(bank0, bank0 + BM * KH, f0, wm, wn, lane);
  for (int k = 0; k < NT; ++k) {
    half_t* s0 = bank0 + (k & 1) * SLOT;
    half_t* s1 = bank1 + (k & 1) * SLOT;
    half_t* s0n = bank0 + ((k + 1) & 1) * SLOT;
    // even half 2k: f0 = half 0 of tile k; read half 1 (bank 1), refill bank 0 slot with tile k+2
    if (k + 1 < NT) tl::wait_vmcnt<8>(); else tl::wait_vmcnt<0>();
    tl::barrier_raw();
    __builtin_amdgcn_sched_barrier(0);
    if (k + 2 < NT) issue(A, B, d, 2 * (k + 2), s0, wave, lane);
    load_frags(s1, s1 + BM * KH, f1, wm, wn, lane);
    prio_on();
    mma(f0, acc);
    prio_off();
    interleave();
    // odd half 2k+1: f1 = half 1 of tile k; read half 0 of tile k+1 (bank 0), refill bank 1 slot
    if (k + 2 < NT) tl::wait_vmcnt<8>(); else if (k + 1 < NT) tl::wait_vmcnt<4>(); else tl::wait_vmcnt<0>();
    tl::barrier_raw();
    __builtin_amdgcn_sched_barrier(0);
    if (k + 2 < NT) issue(A, B, d, 2 * (k + 2) + 1, s1, wave, lane);
    if (k + 1 < NT) load_frags(s0n, s0n + BM * KH, f0, wm, wn, lane);
    prio_on();
    mma(f1, acc);
    prio_off();
    interleave();
  }
#else
  // current DSL schedule: wait for the slot, barrier, refill the slot read the step before,
  // read + MMA (unrolled 4x: compile-time slots, see above)
#pragma unroll
  for (int h = 0; h < 3; ++h) issue(A, B, d, h, smem + h * SLOT, wave, lane);
  for (int h0 = 0; h0 < NH; h0 += 4) {
#define NP_STEP(S)                                                                         \
  {                                                                                        \
    const int h = h0 + S;                                                                  \
    if (h + 2 < NH) tl::wait_vmcnt<8>();                                                   \
    else if (h + 1 < NH) tl::wait_vmcnt<4>();                                              \
    else tl::wait_vmcnt<0>();                                                              \
    tl::barrier_raw();                                                                     \
    if (h + 3 < NH) issue(A, B, d, h + 3, smem + ((S + 3) % 4) * SLOT, wave, lane);        \
    Frags f;                                                                               \
    load_frags(smem + S * SLOT, smem + S * SLOT + BM * KH, f, wm, wn, lane);               \
    prio_on();                                                                             \
    mma(f, acc);                                                                           \
    prio_off();                                                                            \
  }
    NP_STEP(0)
    NP_STEP(1)
    NP_STEP(2)
    NP_STEP(3)
#undef NP_STEP
  }
#endif
  // epilogue: fragments -> row-padded LDS tile -> 16-byte row stores
  tl::barrier_raw();
  half_t* Cs = smem;
  constexpr int LDC = BN + 8;
#pragma unroll
  for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni) {
      const floatx4 v = acc[mi * N_REP + ni];
      half_t o[4] = {(half_t)v[0], (half_t)v[1], (half_t)v[2], (half_t)v[3]};
      const int r = wm * WM + mi * 16 + (lane & 15), c = wn * WN + ni * 16 + 4 * (lane >> 4);
      tl::store_vec<half_t, 4>(&Cs[r * LDC + c], o);
    }
  tl::sync_threads();
#pragma unroll
  for (int i = 0; i < (BM * BN) / (512 * 8); ++i) {
    const int e = (i * 512 + tid) * 8, r = e / BN, c = e % BN;
    tl::copy_bytes<16>(&C[(long)(by * BM + r) * GN + bx * BN + c], &Cs[r * LDC + c]);
  }
}
