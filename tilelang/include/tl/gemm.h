// tl/gemm.h — CDNA4 MFMA tile GEMM micro-kernels (wave64).
//
// Counterpart of src/tl_templates/hip/gemm.h (CDNA3, 16x16x16 MFMA, kPack) and the
// Python MFMA emitter tilelang/intrinsics/mfma_macro_generator.py.  gfx950 specifics:
//   * v_mfma_f32_16x16x32_{f16,bf16}: 8 K-consecutive operands per lane (one ds_read_b128);
//   * MN-contiguous operands ([K][N] B, [K][M] A^T) are read with ds_read_b64_tr_b16
//     (hardware transpose) instead of scalar LDS gathers;
//   * operands are SWAPPED at issue (mfma(B, A)) so every lane holds a row segment of C:
//     C[m = lane&15][n = 4*(lane>>4) + v]  -> 8/16-byte vector epilogue stores and a
//     register-resident accumulator that can feed the next GEMM as its A operand (KPERM=1);
//   * LDS tiles are XOR-swizzled in 16-byte chunks: chunk' = chunk ^ gather(row bits),
//     encoded in a 32-bit SWZ (nibble cb = 1 + row bit XORed into chunk bit cb, 0 = none).
#pragma once

#include <type_traits>

// The T.gemm(valid_m= / valid_m_min=) wave guards are tested only when the argument is not its
// default, so the branch folds away at compile time otherwise: a kept early-return path forces
// the accumulator's initial values (T.clear zeros, fold_max's -m) to stay materialised in
// registers (FA fwd: 35 v_mov per KV tile; FA bwd dQ: 96 AGPR writes per tile).
// -DTL_GEMM_FOLD_DEFAULT_GUARD=0 restores the unconditional test (A/B only).
#ifndef TL_GEMM_FOLD_DEFAULT_GUARD
#define TL_GEMM_FOLD_DEFAULT_GUARD 1
#endif

namespace tl {

// the wave index: callers in loops pass the kernel's own (computed once before the loop); a
// readfirstlane inside the loop is convergent, so LLVM cannot hoist it or the swizzled LDS
// addresses derived from it (+35 VALU per GEMM main-loop iteration, see pipeline.py)
TL_DEVICE int wave_or(int wave_in) {
  return wave_in >= 0 ? wave_in : __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
}

template <uint32_t SWZ> TL_DEVICE int swz_term(int row) {
  int t = 0;
#pragma unroll
  for (int cb = 0; cb < 8; ++cb) {
    const int rb = (int)((SWZ >> (4 * cb)) & 15u);
    if (rb) t |= ((row >> (rb - 1)) & 1) << cb;
  }
  return t;
}

// element offset of (row, col) inside a swizzled [*][COLS] tile of T
// highest row bit (1-based) the swizzle code reads; 0 = unswizzled
template <uint32_t SWZ> constexpr int swz_row_bits() {
  int m = 0;
  for (int cb = 0; cb < 8; ++cb) m = ((SWZ >> (4 * cb)) & 15u) > (uint32_t)m ? (int)((SWZ >> (4 * cb)) & 15u) : m;
  return m;
}

template <typename T, int COLS, uint32_t SWZ> TL_DEVICE int swz_offset(int row, int col) {
  constexpr int EPC = 16 / (int)sizeof(T);
  if constexpr (SWZ == 0u) {
    return row * COLS + col;
  } else {
    return row * COLS + (((col / EPC) ^ swz_term<SWZ>(row)) * EPC) + (col % EPC);
  }
}

template <typename T> struct mfma_traits;

template <> struct mfma_traits<half_t> {
  typedef halfx8 frag;
  TL_DEVICE static floatx4 mma16(frag a, frag b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct mfma_traits<bfloat16_t> {
  typedef bf16x8 frag;
  TL_DEVICE static floatx4 mma16(frag a, frag b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};

// 8 consecutive elements of a row (K-contiguous operand): one ds_read_b128
template <typename T, int COLS, uint32_t SWZ>
TL_DEVICE typename mfma_traits<T>::frag ld_rows8(const T* base, int row, int col) {
  return *reinterpret_cast<const typename mfma_traits<T>::frag*>(base + swz_offset<T, COLS, SWZ>(row, col));
}

// 2x4 K-consecutive elements at cols col0 and col0+16 (k-permuted K-contiguous operand)
template <typename T, int COLS, uint32_t SWZ>
TL_DEVICE typename mfma_traits<T>::frag ld_rows4x2(const T* base, int row, int col0) {
  typedef typename mfma_traits<T>::frag F;
  shortx4 lo = *reinterpret_cast<const shortx4*>(base + swz_offset<T, COLS, SWZ>(row, col0));
  shortx4 hi = *reinterpret_cast<const shortx4*>(base + swz_offset<T, COLS, SWZ>(row, col0 + 16));
  shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(F, v);
}

// transposed read: lane (g=lane>>4, i=lane&15) receives column c0+i of rows r0+q (q=0..3)
// where each lane supplies the address of row rows_of(q) and columns c0 + 4*(i&3).
template <typename T, int COLS, uint32_t SWZ>
TL_DEVICE shortx4 ld_tr4(const T* base, int row, int col) {
  const T* p = base + swz_offset<T, COLS, SWZ>(row, col);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) shortx4*)((__attribute__((address_space(3))) char*)(p)));
}

// MN-contiguous operand fragment for MFMA column c (=lane&15) of tile column c0:
// KPERM=0: rows k0 + 8g + {0..7};   KPERM=1: rows k0 + 4g + {0..3} and k0 + 16 + 4g + {0..3}
template <typename T, int COLS, uint32_t SWZ, int KPERM>
TL_DEVICE typename mfma_traits<T>::frag ld_tr8(const T* base, int k0, int c0, int lane) {
  typedef typename mfma_traits<T>::frag F;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = KPERM ? (k0 + 4 * g + q) : (k0 + 8 * g + q);
  const int r1 = KPERM ? (r0 + 16) : (r0 + 4);
  shortx4 lo = ld_tr4<T, COLS, SWZ>(base, r0, c0 + 4 * p);
  shortx4 hi = ld_tr4<T, COLS, SWZ>(base, r1, c0 + 4 * p);
  shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(F, v);
}

// Operand fragment of an [MN][K] (K-contiguous) or [K][MN] (MN-contiguous) LDS tile for the
// 16-wide MFMA block starting at mn0 and K step k0.
template <typename T, int ROWS, int COLS, uint32_t SWZ, bool MN_CONTIG, int KPERM>
TL_DEVICE typename mfma_traits<T>::frag ld_operand(const T* base, int mn0, int k0, int lane) {
  if constexpr (!MN_CONTIG) {
    const int row = mn0 + (lane & 15);
    if constexpr (KPERM == 0) {
      return ld_rows8<T, COLS, SWZ>(base, row, k0 + 8 * (lane >> 4));
    } else {
      return ld_rows4x2<T, COLS, SWZ>(base, row, k0 + 4 * (lane >> 4));
    }
  } else {
    return ld_tr8<T, COLS, SWZ, KPERM>(base, k0, mn0, lane);
  }
}

// C[M x N] (+)= A * B for one block; each of the WARP_M*WARP_N waves owns a (M/WARP_M)x(N/WARP_N)
// sub-tile held in registers as floatx4 [M_REP][N_REP] (local index (mi*N_REP+ni)*4+v).
// A: LDS tile [M][K] (TA=false) or [K][M] (TA=true); B: [K][N] (TB=false) or [N][K] (TB=true).
template <typename T, int M, int N, int K, int WARP_M, int WARP_N, bool TA, bool TB, int A_COLS, uint32_t SWZ_A,
          int B_COLS, uint32_t SWZ_B>
TL_DEVICE void gemm_ss(const T* __restrict__ A, const T* __restrict__ B, float* __restrict__ C,
                       int m_limit = 0x3fffffff, int wave_in = -1) {
  typedef mfma_traits<T> MT;
  typedef typename MT::frag F;
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 16, N_REP = WN / 16, KSTEPS = K / 32;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && K % 32 == 0, "MFMA 16x16x32 tiling");
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  // T.gemm(valid_m=): a wave whose rows all lie at or past the tile's valid-row count issues
  // nothing (its accumulator rows are don't-care padding); uniform branch, folded when unused
  if ((!TL_GEMM_FOLD_DEFAULT_GUARD || m_limit < 0x3fffffff) && wm * WM >= m_limit) return;  // see gemm_rs
  floatx4* acc = reinterpret_cast<floatx4*>(C);
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) {
    F a[M_REP], b[N_REP];
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
      a[mi] = ld_operand<T, (TA ? K : M), A_COLS, SWZ_A, TA, 0>(A, wm * WM + mi * 16, kk * 32, lane);
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni)
      b[ni] = ld_operand<T, (TB ? N : K), B_COLS, SWZ_B, !TB, 0>(B, wn * WN + ni * 16, kk * 32, lane);
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni)
        acc[mi * N_REP + ni] = MT::mma16(b[ni], a[mi], acc[mi * N_REP + ni]);
  }
}

// ---------------------------------------------------------------------------
// Register-prefetched gemm_ss (the pipelined K-half schedule, transform/pipeline.py): the
// operand fragments of the NEXT K half are read from LDS while the MFMAs of the current half
// run on fragments read one phase earlier, so no MFMA waits on a ds_read issued after the
// phase's barrier.  gemm_ss == gemm_ss_load + gemm_ss_mma on one fragment set.
// ---------------------------------------------------------------------------
template <typename T, int M, int N, int K, int WARP_M, int WARP_N> struct ss_frags {
  static constexpr int M_REP = M / WARP_M / 16, N_REP = N / WARP_N / 16, KSTEPS = K / 32;
  typename mfma_traits<T>::frag a[KSTEPS][M_REP];
  typename mfma_traits<T>::frag b[KSTEPS][N_REP];
};

template <typename T, int M, int N, int K, int WARP_M, int WARP_N, bool TA, bool TB, int A_COLS, uint32_t SWZ_A,
          int B_COLS, uint32_t SWZ_B>
TL_DEVICE void gemm_ss_load(const T* __restrict__ A, const T* __restrict__ B,
                            ss_frags<T, M, N, K, WARP_M, WARP_N>& __restrict__ f, int wave) {
  // `wave` is the kernel's wave index (computed once, outside the loop): a readfirstlane here
  // is convergent, so LLVM keeps it -- and the swizzled addresses derived from it -- in the loop
  typedef ss_frags<T, M, N, K, WARP_M, WARP_N> Fr;
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && K % 32 == 0, "MFMA 16x16x32 tiling");
  const int lane = threadIdx.x & 63;
  const int wm = wave / WARP_N, wn = wave % WARP_N;
#pragma unroll
  for (int kk = 0; kk < Fr::KSTEPS; ++kk) {
#pragma unroll
    for (int mi = 0; mi < Fr::M_REP; ++mi)
      f.a[kk][mi] = ld_operand<T, (TA ? K : M), A_COLS, SWZ_A, TA, 0>(A, wm * WM + mi * 16, kk * 32, lane);
#pragma unroll
    for (int ni = 0; ni < Fr::N_REP; ++ni)
      f.b[kk][ni] = ld_operand<T, (TB ? N : K), B_COLS, SWZ_B, !TB, 0>(B, wn * WN + ni * 16, kk * 32, lane);
  }
}

// ds_read instructions gemm_ss_load issues (MN-contiguous operands use two ds_read_b64_tr_b16)
template <int M, int N, int K, int WARP_M, int WARP_N, bool TA, bool TB> struct ss_load_count {
  static constexpr int value = (K / 32) * ((M / WARP_M / 16) * (TA ? 2 : 1) + (N / WARP_N / 16) * (TB ? 1 : 2));
};

// MFMAs on a fragment set.  NLOAD > 0: the caller issued NLOAD ds_reads (the next half's
// gemm_ss_load) just before, in the same basic block: pin a 1 MFMA : 1 ds_read interleave so the
// reads drain under the matrix pipe instead of queueing in front of it (guide T19).
template <typename T, int M, int N, int K, int WARP_M, int WARP_N, int NLOAD>
TL_DEVICE void gemm_ss_mma(const ss_frags<T, M, N, K, WARP_M, WARP_N>& __restrict__ f, float* __restrict__ C) {
  typedef ss_frags<T, M, N, K, WARP_M, WARP_N> Fr;
  typedef mfma_traits<T> MT;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
#pragma unroll
  for (int kk = 0; kk < Fr::KSTEPS; ++kk)
#pragma unroll
    for (int ni = 0; ni < Fr::N_REP; ++ni)
#pragma unroll
      for (int mi = 0; mi < Fr::M_REP; ++mi)
        acc[mi * Fr::N_REP + ni] = MT::mma16(f.b[kk][ni], f.a[kk][mi], acc[mi * Fr::N_REP + ni]);
  if constexpr (NLOAD > 0) {
    constexpr int NMFMA = Fr::KSTEPS * Fr::M_REP * Fr::N_REP;
    constexpr int PAIRS = NLOAD < NMFMA ? NLOAD : NMFMA;
#pragma unroll
    for (int i = 0; i < PAIRS; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 ds_read
    }
    if constexpr (NMFMA > PAIRS) __builtin_amdgcn_sched_group_barrier(0x008, NMFMA - PAIRS, 0);
    if constexpr (NLOAD > PAIRS) __builtin_amdgcn_sched_group_barrier(0x100, NLOAD - PAIRS, 0);
  }
}

// A operand in registers (gemm_rs): a_regs holds the A fragment, 8 elements per (mi, kk) at
// a_regs + (mi*KSTEPS + kk)*8.  KPERM=1 when the fragment came from an accumulator layout.
//
// PIPE = G > 0 (pass config tl.gemm_rs_pipe): the B fragments stream through the MFMAs in groups
// of G: group g+1's ds_reads are pinned 1:1 (or 1 : reads-per-MFMA) between group g's MFMAs,
// across K steps too, so at most two groups are in flight.  Without it the compiler issues every
// read of a K step first and then waits for all of them: with 16 transposed reads (the PV GEMM of
// attention, 8 fragments x 2 ds_read_b64_tr_b16) that is more than the 15 the lgkmcnt counter can
// track, so the first MFMA waits on lgkmcnt(0) -- the whole K step's LDS latency, exposed.
template <typename T, int M, int N, int K, int WARP_M, int WARP_N, bool TB, int B_COLS, uint32_t SWZ_B, int KPERM,
          int PIPE = 0>
TL_DEVICE void gemm_rs(const T* __restrict__ a_regs, const T* __restrict__ B, float* __restrict__ C,
                       int wave_in = -1, int m_min = 0) {
  typedef mfma_traits<T> MT;
  typedef typename MT::frag F;
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 16, N_REP = WN / 16, KSTEPS = K / 32;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && K % 32 == 0, "MFMA 16x16x32 tiling");
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wn = wave % WARP_N;
  // T.gemm(valid_m_min=): a wave whose rows all lie below m_min has nothing to add (uniform branch)
  if ((!TL_GEMM_FOLD_DEFAULT_GUARD || m_min > 0) && (wave / WARP_N + 1) * WM <= m_min) return;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
  if constexpr (PIPE > 0 && N_REP % PIPE == 0 && KSTEPS * N_REP > PIPE) {
    constexpr int G = PIPE, NG = KSTEPS * N_REP / G;  // groups of G fragments, in (kk, ni) order
    constexpr int RPF = TB ? 1 : 2;                    // ds_reads per fragment
    F b[NG][G];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
#pragma unroll
      for (int j = 0; j < G; ++j) {
        const int q = g * G + j, kk = q / N_REP, ni = q % N_REP;
        b[g][j] = ld_operand<T, (TB ? N : K), B_COLS, SWZ_B, !TB, KPERM>(B, wn * WN + ni * 16, kk * 32, lane);
      }
      if (g > 0) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
          const int q = (g - 1) * G + j, kk = q / N_REP, ni = q % N_REP;
#pragma unroll
          for (int mi = 0; mi < M_REP; ++mi) {
            F a;
            __builtin_memcpy(&a, a_regs + (mi * KSTEPS + kk) * 8, sizeof(F));
            acc[mi * N_REP + ni] = MT::mma16(b[g - 1][j], a, acc[mi * N_REP + ni]);
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int q = (NG - 1) * G + j, kk = q / N_REP, ni = q % N_REP;
#pragma unroll
      for (int mi = 0; mi < M_REP; ++mi) {
        F a;
        __builtin_memcpy(&a, a_regs + (mi * KSTEPS + kk) * 8, sizeof(F));
        acc[mi * N_REP + ni] = MT::mma16(b[NG - 1][j], a, acc[mi * N_REP + ni]);
      }
    }
    // schedule: group 0's reads, then each later group's reads spread over the previous group's
    // MFMAs (M_REP MFMAs per fragment against RPF reads), then the last group's MFMAs
    constexpr int MF = G * M_REP, RD = G * RPF;
    __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
#pragma unroll
    for (int g = 1; g < NG; ++g) {
      if constexpr (MF >= RD) {
#pragma unroll
        for (int i = 0; i < RD; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, MF / RD, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (MF % RD) __builtin_amdgcn_sched_group_barrier(0x008, MF % RD, 0);
      } else {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, RD / MF, 0);
        }
        if constexpr (RD % MF) __builtin_amdgcn_sched_group_barrier(0x100, RD % MF, 0);
      }
    }
    __builtin_amdgcn_sched_group_barrier(0x008, MF, 0);
    return;
  }
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) {
    F b[N_REP];
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni)
      b[ni] = ld_operand<T, (TB ? N : K), B_COLS, SWZ_B, !TB, KPERM>(B, wn * WN + ni * 16, kk * 32, lane);
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi) {
      F a;
      __builtin_memcpy(&a, a_regs + (mi * KSTEPS + kk) * 8, sizeof(F));
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni)
        acc[mi * N_REP + ni] = MT::mma16(b[ni], a, acc[mi * N_REP + ni]);
    }
  }
}

// ---------------------------------------------------------------------------
// 8-bit (OCP fp8 e4m3 / e5m2) GEMM, both operands K-contiguous ([M][K] and [N][K] in LDS).
// K % 128 == 0: v_mfma_scale_f32_16x16x128_f8f6f4 with unit e8m0 scales (2x the bf16 MFMA
//               rate); each lane feeds 32 consecutive k (two ds_read_b128).  The operand
//               k-assignment only has to agree between A and B (verified on gfx950 with exact
//               integer data: csrc/probes/mfma_fp8_layout.hip).
// otherwise:    v_mfma_f32_16x16x32_{fp8,bf8}_{fp8,bf8}, 8 consecutive k per lane (ds_read_b64).
// ---------------------------------------------------------------------------
template <typename T> struct fp8_fmt;
template <> struct fp8_fmt<fp8_e4_t> { static constexpr int code = 0; };
template <> struct fp8_fmt<fp8_e5_t> { static constexpr int code = 1; };

template <typename TA, typename TB> TL_DEVICE floatx4 mma_f8_32(long a, long b, floatx4 c) {
  if constexpr (fp8_fmt<TA>::code == 0 && fp8_fmt<TB>::code == 0)
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0);
  else if constexpr (fp8_fmt<TA>::code == 0)
    return __builtin_amdgcn_mfma_f32_16x16x32_fp8_bf8(a, b, c, 0, 0, 0);
  else if constexpr (fp8_fmt<TB>::code == 0)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf8_fp8(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf8_bf8(a, b, c, 0, 0, 0);
}

template <int COLS, uint32_t SWZ>
TL_DEVICE intx8 ld_rows32_b8(const uint8_t* base, int row, int col) {
  intx4 lo = *reinterpret_cast<const intx4*>(base + swz_offset<uint8_t, COLS, SWZ>(row, col));
  intx4 hi = *reinterpret_cast<const intx4*>(base + swz_offset<uint8_t, COLS, SWZ>(row, col + 16));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <int COLS, uint32_t SWZ>
TL_DEVICE long ld_rows8_b8(const uint8_t* base, int row, int col) {
  return *reinterpret_cast<const long*>(base + swz_offset<uint8_t, COLS, SWZ>(row, col));
}

// MN-contiguous 8-bit operand ([K][N] in LDS) via ds_read_b64_tr_b8: in each 16-lane group, lane i
// supplies the address of row k0 + (i >> 1), columns n0 + 8 (i & 1) and receives column n0 + i of
// rows k0 .. k0 + 7, one byte per row in order (measured on gfx950:
// csrc/probes/ds_read_tr8_probe.hip, profiles/r6/ds_read_tr8_probe.log).  Lane group g = lane >> 4
// reads its own 8-row block, so lane (g, i) gets rows k0 + 8 g .. + 7 of column n0 + i -- the k
// assignment of the K-contiguous reads (8 consecutive k per lane group), as the MFMA needs.
template <int COLS, uint32_t SWZ>
TL_DEVICE long ld_tr8_b8(const uint8_t* base, int k0, int n0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  typedef int v2i __attribute__((ext_vector_type(2)));
  const uint8_t* p = base + swz_offset<uint8_t, COLS, SWZ>(k0 + 8 * g + (i >> 1), n0 + 8 * (i & 1));
  v2i v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (__attribute__((address_space(3))) v2i*)((__attribute__((address_space(3))) char*)(p)));
  return __builtin_bit_cast(long, v);
}

// the 32-byte operand of the scaled 16x16x128 MFMA from an MN-contiguous tile: lane group g needs
// rows k0 + 32 g .. + 31 of its column: four transposed reads of 8 rows (rows 32 g + 8 t of the
// read's lane group = its own group when the read's base row is k0 + 24 g + 8 t)
template <int COLS, uint32_t SWZ>
TL_DEVICE intx8 ld_tr32_b8(const uint8_t* base, int k0, int n0, int lane) {
  const int g = lane >> 4;
  long v[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) v[t] = ld_tr8_b8<COLS, SWZ>(base, k0 + 24 * g + 8 * t, n0, lane);
  typedef int v2i __attribute__((ext_vector_type(2)));
  const v2i a = __builtin_bit_cast(v2i, v[0]), b = __builtin_bit_cast(v2i, v[1]);
  const v2i c = __builtin_bit_cast(v2i, v[2]), d = __builtin_bit_cast(v2i, v[3]);
  return intx8{a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
}

// A: [M][K] (K contiguous), B: [N][K] (K contiguous, TB) or [K][N] (N contiguous, !TB: transposed
// LDS reads, ds_read_b64_tr_b8)
template <typename TA, typename TB, int M, int N, int K, int WARP_M, int WARP_N, int A_COLS, uint32_t SWZ_A,
          int B_COLS, uint32_t SWZ_B, bool B_KCONTIG = true>
TL_DEVICE void gemm_ss_f8(const TA* __restrict__ A_, const TB* __restrict__ B_, float* __restrict__ C,
                          int wave_in = -1) {
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 16, N_REP = WN / 16;
  const uint8_t* A = reinterpret_cast<const uint8_t*>(A_);
  const uint8_t* B = reinterpret_cast<const uint8_t*>(B_);
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  const int r = lane & 15, g = lane >> 4;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
  if constexpr (K % 128 == 0) {
#pragma unroll
    for (int kk = 0; kk < K / 128; ++kk) {
      intx8 a[M_REP], b[N_REP];
#pragma unroll
      for (int mi = 0; mi < M_REP; ++mi)
        a[mi] = ld_rows32_b8<A_COLS, SWZ_A>(A, wm * WM + mi * 16 + r, kk * 128 + 32 * g);
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni) {
        if constexpr (B_KCONTIG)
          b[ni] = ld_rows32_b8<B_COLS, SWZ_B>(B, wn * WN + ni * 16 + r, kk * 128 + 32 * g);
        else
          b[ni] = ld_tr32_b8<B_COLS, SWZ_B>(B, kk * 128, wn * WN + ni * 16, lane);
      }
#pragma unroll
      for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
        for (int ni = 0; ni < N_REP; ++ni)
          // scale operands 0: the compiler selects the unscaled v_mfma_f32_16x16x128_f8f6f4 (unit
          // scales; numerics in tests/test_gemm_phased.py), not the two-word v_mfma_scale form
          acc[mi * N_REP + ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              b[ni], a[mi], acc[mi * N_REP + ni], fp8_fmt<TB>::code, fp8_fmt<TA>::code, 0, 0, 0, 0);
    }
  } else {
    static_assert(K % 32 == 0, "fp8 MFMA needs K % 32 == 0");
#pragma unroll
    for (int kk = 0; kk < K / 32; ++kk) {
      long a[M_REP], b[N_REP];
#pragma unroll
      for (int mi = 0; mi < M_REP; ++mi) a[mi] = ld_rows8_b8<A_COLS, SWZ_A>(A, wm * WM + mi * 16 + r, kk * 32 + 8 * g);
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni) {
        if constexpr (B_KCONTIG)
          b[ni] = ld_rows8_b8<B_COLS, SWZ_B>(B, wn * WN + ni * 16 + r, kk * 32 + 8 * g);
        else
          b[ni] = ld_tr8_b8<B_COLS, SWZ_B>(B, kk * 32, wn * WN + ni * 16, lane);
      }
#pragma unroll
      for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
        for (int ni = 0; ni < N_REP; ++ni)
          acc[mi * N_REP + ni] = mma_f8_32<TB, TA>(b[ni], a[mi], acc[mi * N_REP + ni]);
    }
  }
}

}  // namespace tl

namespace tl {

// ---------------------------------------------------------------------------
// Block-scaled MX GEMM (OCP MX: one e8m0 scale per 32 K of each row), both operands
// K-contiguous byte tiles in LDS: fp8 rows hold K bytes, packed fp4 rows K/2 bytes.
// v_mfma_scale_f32_16x16x128_f8f6f4, lane l = (row r = l&15, group g = l>>4), one 128-K step,
// measured on gfx950 with exact data and per-lane scales (csrc/probes/mfma_scale_probe.hip):
//   fp8 : bytes 0-15 of the lane are k = 16g..16g+15, bytes 16-31 are k = 64+16g..64+16g+15;
//   fp4 : the 16 bytes are k = 32g..32g+31 (low nibble = even k);
//   scale: lane l's e8m0 byte (bits 7:0, opsel 0) scales K block g = k 32g..32g+31 of row r.
//   For fp8 block g therefore spans bytes 0-15 (g < 2) or 16-31 (g >= 2) of lane groups 2(g&1)
//   and 2(g&1)+1, not the scale lane's own bytes: the data is fetched in the hardware K order
//   above (two 16-byte reads at 16g and 64+16g) so contiguous MX blocks line up with the scales.
//   fp6 : packed 4 per 3 bytes (element k at bits 6k..6k+5 of the row), the 24 bytes at 24g
//         (= k 32g..32g+31, the fp4 order) in registers 0-5 -- three 8-byte reads.
// FMT codes: 0 e4m3, 1 e5m2, 2 e2m3, 3 e3m2, 4 e2m1.  Operands are swapped at issue like gemm_ss.
// ---------------------------------------------------------------------------
template <int FMT> struct mx_fmt {
  static constexpr int lane_bytes = FMT == 4 ? 16 : (FMT == 2 || FMT == 3) ? 24 : 32;
  static constexpr int step_bytes = lane_bytes * 4;  // bytes of one 128-K step of a row
  static constexpr int nreads = FMT == 4 ? 1 : (FMT == 2 || FMT == 3) ? 3 : 2;
};
// byte column (in the 128-K step) of a lane group's read j
template <int FMT> TL_DEVICE constexpr int mx_read_col(int g, int j) {
  return mx_fmt<FMT>::lane_bytes == 24 ? 24 * g + 8 * j : 16 * g + 64 * j;
}

// bcol0: byte column of the 128-K step in the row
template <int FMT, int COLS, uint32_t SWZ>
TL_DEVICE intx8 ld_mx_operand(const uint8_t* base, int row, int bcol0, int g) {
  if constexpr (mx_fmt<FMT>::lane_bytes == 32) {
    intx4 lo = *reinterpret_cast<const intx4*>(base + swz_offset<uint8_t, COLS, SWZ>(row, bcol0 + 16 * g));
    intx4 hi = *reinterpret_cast<const intx4*>(base + swz_offset<uint8_t, COLS, SWZ>(row, bcol0 + 64 + 16 * g));
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  } else {
    intx4 lo = *reinterpret_cast<const intx4*>(base + swz_offset<uint8_t, COLS, SWZ>(row, bcol0 + 16 * g));
    intx4 z = {0, 0, 0, 0};
    return __builtin_shufflevector(lo, z, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// Scaled MFMA with the scale bytes picked by op_sel (2-bit byte select per scale operand; the
// builtin needs immediates, the switch folds once the fragment loops are unrolled).
#define TL_MXS_CASE(OB, OA) \
  case OB * 4 + OA:         \
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b, a, c, FB, FA, OB, sb, OA, sa);
template <int FA, int FB>
TL_DEVICE floatx4 mfma_mx_sel(intx8 b, intx8 a, floatx4 c, int sb, int sa, int ob, int oa) {
  switch (ob * 4 + oa) {
    TL_MXS_CASE(0, 0) TL_MXS_CASE(0, 1) TL_MXS_CASE(0, 2) TL_MXS_CASE(0, 3)
    TL_MXS_CASE(1, 0) TL_MXS_CASE(1, 1) TL_MXS_CASE(1, 2) TL_MXS_CASE(1, 3)
    TL_MXS_CASE(2, 0) TL_MXS_CASE(2, 1) TL_MXS_CASE(2, 2) TL_MXS_CASE(2, 3)
    TL_MXS_CASE(3, 0) TL_MXS_CASE(3, 1) TL_MXS_CASE(3, 2) TL_MXS_CASE(3, 3)
  }
  return c;
}
#undef TL_MXS_CASE

// Pre-shuffled scale tile of R rows (T.gemm_scaled(scale_layout="preshuffled")): row = 16 f + r,
// scale column kb = 4 kk + g; byte ((((kk * R/64 + f/4) * 4 + g) * 16 + r) * 4 + f % 4.  Lane (r, g)
// then finds the scales of 4 consecutive 16-row fragments in one dword (one ds_read_b32 instead
// of four ds_read_u8) and the MFMA's op_sel picks fragment f % 4's byte.
template <int FA, int FB, int M, int N, int K, int WARP_M, int WARP_N, int A_COLS, uint32_t SWZ_A, int B_COLS,
          uint32_t SWZ_B, int SA_STRIDE, int SB_STRIDE, int SCALE_PS = 0>
TL_DEVICE void gemm_ss_mx(const void* __restrict__ A_, const void* __restrict__ B_, const void* __restrict__ SA_,
                          const void* __restrict__ SB_, float* __restrict__ C, int wave_in = -1) {
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 16, N_REP = WN / 16;
  constexpr int BA = mx_fmt<FA>::lane_bytes, BB = mx_fmt<FB>::lane_bytes;  // bytes per lane per step
  static_assert(WM % 16 == 0 && WN % 16 == 0 && K % 128 == 0, "scaled MFMA 16x16x128 tiling");
  const uint8_t* A = reinterpret_cast<const uint8_t*>(A_);
  const uint8_t* B = reinterpret_cast<const uint8_t*>(B_);
  const uint8_t* SA = reinterpret_cast<const uint8_t*>(SA_);
  const uint8_t* SB = reinterpret_cast<const uint8_t*>(SB_);
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  const int r = lane & 15, g = lane >> 4;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
  // The operand with fewer fragments per wave stays in registers for the 128-K step; the other is
  // streamed one fragment ahead of its MFMAs.  Holding both (M_REP + N_REP fragments + scales next
  // to the 128-register accumulator of a 256x256 / 8-wave tile) reached 256 VGPRs and the compiler
  // re-read A between MFMA groups behind lgkmcnt(0) waits.
  // Addresses: the swizzle reads row bits 0..3 only (static_assert), so a lane's swizzled byte
  // offsets are the same for every 16-row fragment; fragment i is i * 16 rows further on, an
  // immediate of the ds_read.  Written as swz_offset(row, col) per fragment the compiler rebuilt
  // each address from three registers every K step (~60 VALU adds per step, half the loop's VALU).
  static_assert(swz_row_bits<SWZ_A>() <= 4 && swz_row_bits<SWZ_B>() <= 4, "MX swizzle must use row bits 0..3");
  constexpr bool HOLD_B = N_REP <= M_REP;
  constexpr int NH = HOLD_B ? N_REP : M_REP, NS = HOLD_B ? M_REP : N_REP;
  constexpr int KS = K / 128;
  int oa[KS][3], ob[KS][3];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk)
#pragma unroll
    for (int h = 0; h < 3; ++h) {
      oa[kk][h] = swz_offset<uint8_t, A_COLS, SWZ_A>(r, kk * 4 * BA + mx_read_col<FA>(g, h));
      ob[kk][h] = swz_offset<uint8_t, B_COLS, SWZ_B>(r, kk * 4 * BB + mx_read_col<FB>(g, h));
    }
  const uint8_t* Aw = A + wm * WM * A_COLS;
  const uint8_t* Bw = B + wn * WN * B_COLS;
  static_assert(!SCALE_PS || (WM % 64 == 0 && WN % 64 == 0), "pre-shuffled scales: 64-row warp tiles");
  const uint8_t* SAw = SCALE_PS ? SA + (wm * WM / 64) * 256 + (g * 16 + r) * 4 : SA + (wm * WM + r) * SA_STRIDE + g;
  const uint8_t* SBw = SCALE_PS ? SB + (wn * WN / 64) * 256 + (g * 16 + r) * 4 : SB + (wn * WN + r) * SB_STRIDE + g;
  auto frag = [&](const uint8_t* base, int cols, const int (&o)[3], int i, int lane_bytes) -> intx8 {
    const uint8_t* p = base + i * 16 * cols;
    if (lane_bytes == 24) {  // fp6: 3 x 8 bytes (8-byte aligned, never across a 16-byte chunk)
      intx2 a = *reinterpret_cast<const intx2*>(p + o[0]);
      intx2 b = *reinterpret_cast<const intx2*>(p + o[1]);
      intx2 c = *reinterpret_cast<const intx2*>(p + o[2]);
      return intx8{a.x, a.y, b.x, b.y, c.x, c.y, 0, 0};
    }
    intx4 lo = *reinterpret_cast<const intx4*>(p + o[0]);
    intx4 hi = lane_bytes == 32 ? *reinterpret_cast<const intx4*>(p + o[1]) : intx4{0, 0, 0, 0};
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  };
  auto ld_scale = [&](const uint8_t* w, int rows, int stride, int i, int kk) -> int {
    if constexpr (SCALE_PS) return *reinterpret_cast<const int*>(w + (i >> 2) * 256 + kk * rows * 4);
    return (int)w[i * 16 * stride + kk * 4];
  };
  auto ld_a = [&](int i, int kk, int& sc) -> intx8 {
    sc = ld_scale(SAw, M, SA_STRIDE, i, kk);
    return frag(Aw, A_COLS, oa[kk], i, BA);
  };
  auto ld_b = [&](int i, int kk, int& sc) -> intx8 {
    sc = ld_scale(SBw, N, SB_STRIDE, i, kk);
    return frag(Bw, B_COLS, ob[kk], i, BB);
  };
  auto ld_held = [&](int i, int kk, int& sc) -> intx8 { return HOLD_B ? ld_b(i, kk, sc) : ld_a(i, kk, sc); };
  auto ld_stream = [&](int i, int kk, int& sc) -> intx8 { return HOLD_B ? ld_a(i, kk, sc) : ld_b(i, kk, sc); };
  // one streamed fragment in flight ahead of its MFMAs: distances 0-3 measured within 0.5 % of each
  // other once the addresses were immediates (profiles/r3/s3/lowp/mx_pd_ab_after_addr.log)
  constexpr int PD = NS < 1 ? NS : 1;
#pragma unroll
  for (int kk = 0; kk < K / 128; ++kk) {
    intx8 h[NH], sv[NS];
    int sh[NH], ss[NS];
#pragma unroll
    for (int i = 0; i < NH; ++i) h[i] = ld_held(i, kk, sh[i]);
#pragma unroll
    for (int j = 0; j < PD; ++j) sv[j] = ld_stream(j, kk, ss[j]);
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      if (j + PD < NS) sv[j + PD] = ld_stream(j + PD, kk, ss[j + PD]);
#pragma unroll
      for (int i = 0; i < NH; ++i) {
        const int mi = HOLD_B ? j : i, ni = HOLD_B ? i : j;
        const intx8 av = HOLD_B ? sv[j] : h[i], bv = HOLD_B ? h[i] : sv[j];
        const int sav = HOLD_B ? ss[j] : sh[i], sbv = HOLD_B ? sh[i] : ss[j];
        acc[mi * N_REP + ni] = mfma_mx_sel<FA, FB>(bv, av, acc[mi * N_REP + ni], sbv, sav, SCALE_PS ? ni & 3 : 0,
                                                   SCALE_PS ? mi & 3 : 0);
      }
    }
  }
}

}  // namespace tl

namespace tl {

// ---------------------------------------------------------------------------
// 32x32 MFMA tiles (v_mfma_f32_32x32x16_{f16,bf16}, v_mfma_i32_32x32x32_i8) and the 16x16 int8 /
// fp32 forms.  Operand maps (swapped issue, as gemm_ss): lane l holds operand rows (m or n)
// l & 31 and 8 (16-bit) / 16 (8-bit) consecutive k starting at (l >> 5) * 8 / 16; the accumulator
// (16 registers) is C[m = l & 31][n = (v & 3) + 8 (v >> 2) + 4 (l >> 5)].
// ---------------------------------------------------------------------------
template <typename T> struct mfma32_traits;
template <> struct mfma32_traits<half_t> {
  typedef halfx8 frag;
  TL_DEVICE static floatx16 mma(frag a, frag b, floatx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
};
template <> struct mfma32_traits<bfloat16_t> {
  typedef bf16x8 frag;
  TL_DEVICE static floatx16 mma(frag a, frag b, floatx16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

// MN-contiguous operand of the 32x32x16 MFMA: lane (g = l >> 4, i = l & 15) needs column
// c0 + 16 (g & 1) + i, rows k0 + 8 (g >> 1) + 0..7: two ds_read_b64_tr_b16 of 4 rows each.
// KPERM=1 (the A operand is a 32x32 accumulator, layout.mfma._mfma_a_fragment32): rows
// k0 + 4 (g >> 1) + 0..3 and k0 + 8 + 4 (g >> 1) + 0..3 -- still two 4-row transposed reads.
template <typename T, int COLS, uint32_t SWZ, int KPERM = 0>
TL_DEVICE typename mfma32_traits<T>::frag ld_tr8_32(const T* base, int k0, int c0, int lane) {
  typedef typename mfma32_traits<T>::frag F;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int r0 = KPERM ? (k0 + 4 * (g >> 1) + q) : (k0 + 8 * (g >> 1) + q);
  const int c = c0 + 16 * (g & 1) + 4 * p;
  shortx4 lo = ld_tr4<T, COLS, SWZ>(base, r0, c);
  shortx4 hi = ld_tr4<T, COLS, SWZ>(base, r0 + (KPERM ? 8 : 4), c);
  shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(F, v);
}

template <typename T, int ROWS, int COLS, uint32_t SWZ, bool MN_CONTIG, int KPERM = 0>
TL_DEVICE typename mfma32_traits<T>::frag ld_operand32(const T* base, int mn0, int k0, int lane) {
  if constexpr (!MN_CONTIG) {
    if constexpr (KPERM == 0) {
      return *reinterpret_cast<const typename mfma32_traits<T>::frag*>(
          base + swz_offset<T, COLS, SWZ>(mn0 + (lane & 31), k0 + 8 * (lane >> 5)));
    } else {  // k0 + 4h + 0..3 and k0 + 8 + 4h + 0..3
      typedef typename mfma32_traits<T>::frag F;
      const int row = mn0 + (lane & 31), c = k0 + 4 * (lane >> 5);
      shortx4 lo = *reinterpret_cast<const shortx4*>(base + swz_offset<T, COLS, SWZ>(row, c));
      shortx4 hi = *reinterpret_cast<const shortx4*>(base + swz_offset<T, COLS, SWZ>(row, c + 8));
      shortx8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      return __builtin_bit_cast(F, v);
    }
  } else {
    return ld_tr8_32<T, COLS, SWZ, KPERM>(base, k0, mn0, lane);
  }
}

template <typename T, int M, int N, int K, int WARP_M, int WARP_N, bool TA, bool TB, int A_COLS, uint32_t SWZ_A,
          int B_COLS, uint32_t SWZ_B>
TL_DEVICE void gemm_ss_32(const T* __restrict__ A, const T* __restrict__ B, float* __restrict__ C,
                          int m_limit = 0x3fffffff, int wave_in = -1) {
  typedef mfma32_traits<T> MT;
  typedef typename MT::frag F;
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 32, N_REP = WN / 32, KSTEPS = K / 16;
  static_assert(WM % 32 == 0 && WN % 32 == 0 && K % 16 == 0, "MFMA 32x32x16 tiling");
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  if ((!TL_GEMM_FOLD_DEFAULT_GUARD || m_limit < 0x3fffffff) && wm * WM >= m_limit) return;  // valid_m
  floatx16* acc = reinterpret_cast<floatx16*>(C);
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) {
    F a[M_REP], b[N_REP];
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
      a[mi] = ld_operand32<T, (TA ? K : M), A_COLS, SWZ_A, TA>(A, wm * WM + mi * 32, kk * 16, lane);
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni)
      b[ni] = ld_operand32<T, (TB ? N : K), B_COLS, SWZ_B, !TB>(B, wn * WN + ni * 32, kk * 16, lane);
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni)
        acc[mi * N_REP + ni] = MT::mma(b[ni], a[mi], acc[mi * N_REP + ni]);
  }
}

// A operand in registers, 32x32x16 MFMA: a_regs holds 8 elements per (mi, kk) at
// a_regs + (mi*KSTEPS + kk)*8 (KSTEPS = K/16).  KPERM=1 when the fragment is a 32x32
// accumulator (FlashAttention's P): its k order is matched by the B read (ld_tr8_32<KPERM>).
// With one query row per lane, the softmax row reductions of such a kernel are in-register
// except one lane^32 exchange, and a 32-cycle MFMA leaves 24 of its cycles to the VALU (8 of
// 16 for 16x16x32): the exp/max/sum stream of the softmax fits in the matrix pipe's shadow.
template <typename T, int M, int N, int K, int WARP_M, int WARP_N, bool TB, int B_COLS, uint32_t SWZ_B, int KPERM>
TL_DEVICE void gemm_rs_32(const T* __restrict__ a_regs, const T* __restrict__ B, float* __restrict__ C,
                          int wave_in = -1) {
  typedef mfma32_traits<T> MT;
  typedef typename MT::frag F;
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 32, N_REP = WN / 32, KSTEPS = K / 16;
  static_assert(WM % 32 == 0 && WN % 32 == 0 && K % 16 == 0, "MFMA 32x32x16 tiling");
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wn = wave % WARP_N;
  floatx16* acc = reinterpret_cast<floatx16*>(C);
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) {
    F b[N_REP];
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni)
      b[ni] = ld_operand32<T, (TB ? N : K), B_COLS, SWZ_B, !TB, KPERM>(B, wn * WN + ni * 32, kk * 16, lane);
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi) {
      F a;
      __builtin_memcpy(&a, a_regs + (mi * KSTEPS + kk) * 8, sizeof(F));
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni)
        acc[mi * N_REP + ni] = MT::mma(b[ni], a, acc[mi * N_REP + ni]);
    }
  }
}

// int8 x int8 -> int32, both operands K-contiguous ([M][K] and [N][K] bytes in LDS).
// MS = 16: v_mfma_i32_16x16x64_i8 (lane: row l & 15, 16 bytes at k = 16 (l >> 4));
// MS = 32: v_mfma_i32_32x32x32_i8 (lane: row l & 31, 16 bytes at k = 16 (l >> 5)).
template <int MS, int M, int N, int K, int WARP_M, int WARP_N, int A_COLS, uint32_t SWZ_A, int B_COLS,
          uint32_t SWZ_B>
TL_DEVICE void gemm_ss_i8(const int8_t* __restrict__ A_, const int8_t* __restrict__ B_, int* __restrict__ C,
                          int wave_in = -1) {
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / MS, N_REP = WN / MS, KS = MS == 16 ? 64 : 32;
  static_assert(WM % MS == 0 && WN % MS == 0 && K % KS == 0, "int8 MFMA tiling");
  const uint8_t* A = reinterpret_cast<const uint8_t*>(A_);
  const uint8_t* B = reinterpret_cast<const uint8_t*>(B_);
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  const int r = lane & (MS - 1), g = MS == 16 ? (lane >> 4) : (lane >> 5);
#pragma unroll
  for (int kk = 0; kk < K / KS; ++kk) {
    intx4 a[M_REP], b[N_REP];
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
      a[mi] = *reinterpret_cast<const intx4*>(A + swz_offset<uint8_t, A_COLS, SWZ_A>(wm * WM + mi * MS + r,
                                                                                       kk * KS + 16 * g));
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni)
      b[ni] = *reinterpret_cast<const intx4*>(B + swz_offset<uint8_t, B_COLS, SWZ_B>(wn * WN + ni * MS + r,
                                                                                       kk * KS + 16 * g));
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni) {
        if constexpr (MS == 16) {
          intx4* acc = reinterpret_cast<intx4*>(C);
          acc[mi * N_REP + ni] = __builtin_amdgcn_mfma_i32_16x16x64_i8(b[ni], a[mi], acc[mi * N_REP + ni], 0, 0, 0);
        } else {
          intx16* acc = reinterpret_cast<intx16*>(C);
          acc[mi * N_REP + ni] = __builtin_amdgcn_mfma_i32_32x32x32_i8(b[ni], a[mi], acc[mi * N_REP + ni], 0, 0, 0);
        }
      }
  }
}

// fp32 x fp32 -> fp32 (exact f32 fmaf chain, the f32 VALU rate): v_mfma_f32_16x16x4_f32,
// lane l holds A[m = l & 15][k = l >> 4] and B[k = l >> 4][n = l & 15]; any operand layout.
template <int M, int N, int K, int WARP_M, int WARP_N, bool TA, bool TB, int A_COLS, int B_COLS>
TL_DEVICE void gemm_ss_f32(const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C,
                           int wave_in = -1) {
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 16, N_REP = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && K % 4 == 0, "MFMA 16x16x4 f32 tiling");
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  const int r = lane & 15, g = lane >> 4;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
#pragma unroll 4
  for (int kk = 0; kk < K / 4; ++kk) {
    float a[M_REP], b[N_REP];
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi) {
      const int m = wm * WM + mi * 16 + r, k = kk * 4 + g;
      a[mi] = TA ? A[k * A_COLS + m] : A[m * A_COLS + k];
    }
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni) {
      const int n = wn * WN + ni * 16 + r, k = kk * 4 + g;
      b[ni] = TB ? B[n * B_COLS + k] : B[k * B_COLS + n];
    }
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni)
        acc[mi * N_REP + ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(b[ni], a[mi], acc[mi * N_REP + ni], 0, 0, 0);
  }
}

}  // namespace tl

namespace tl {

// ---------------------------------------------------------------------------
// Single MFMA on per-thread register arrays, for the user-level intrinsic emitter
// (tilelang/intrinsics/mfma_macro_generator.py).  Standard (unswapped) operand maps:
//   a: lane l holds A[row = l & 15][k = K_PER * (l >> 4) + 0 .. K_PER-1]
//   b: lane l holds B[k = K_PER * (l >> 4) + 0 .. K_PER-1][col = l & 15]
//   c: lane l holds C[row = 4 * (l >> 4) + v][col = l & 15], v = 0..3
// K_PER = 8 (f16 / bf16, 16x16x32) or 16 (int8, 16x16x64, int32 accumulator).
// ---------------------------------------------------------------------------
template <typename T> TL_DEVICE void mfma_16x16(float* c, const T* a, const T* b) {
  typedef typename mfma_traits<T>::frag F;
  F av = *reinterpret_cast<const F*>(a);
  F bv = *reinterpret_cast<const F*>(b);
  floatx4 cv = *reinterpret_cast<floatx4*>(c);
  cv = mfma_traits<T>::mma16(av, bv, cv);
  *reinterpret_cast<floatx4*>(c) = cv;
}

TL_DEVICE void mfma_16x16(int* c, const int8_t* a, const int8_t* b) {
  intx4 av = *reinterpret_cast<const intx4*>(a);
  intx4 bv = *reinterpret_cast<const intx4*>(b);
  intx4 cv = *reinterpret_cast<intx4*>(c);
  cv = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, cv, 0, 0, 0);
  *reinterpret_cast<intx4*>(c) = cv;
}

// General form for the emitter: MS x MS tiles (16 or 32), KPER consecutive k per lane, standard
// operand order mfma(A, B) (no swap):
//   MS = 16: lane l holds A[l & 15][KPER (l >> 4) + j], B[KPER (l >> 4) + j][l & 15];
//            C[4 (l >> 4) + v][l & 15], v < 4
//   MS = 32: lane l holds A[l & 31][KPER (l >> 5) + j], B[KPER (l >> 5) + j][l & 31];
//            C[8 (v >> 2) + 4 (l >> 5) + (v & 3)][l & 31], v < 16
// Instructions: f16/bf16 KPER 8 (16x16x32, 32x32x16); int8 KPER 16 (16x16x64, 32x32x32); OCP fp8
// (e4m3fn / e5m2, any mix) KPER 8 (16x16x32, 32x32x16) or KPER 32 (the f8f6f4 16x16x128 / 32x32x64
// forms with unit e8m0 scales, 2x the rate; their in-lane k order is a fixed permutation applied
// to A and B alike, so the contraction is unchanged); fp32 KPER 1 (16x16x4, 32x32x2).
template <typename T> struct emit_kind { static constexpr int v = 0; };
template <> struct emit_kind<half_t> { static constexpr int v = 1; };
template <> struct emit_kind<bfloat16_t> { static constexpr int v = 1; };
template <> struct emit_kind<int8_t> { static constexpr int v = 2; };
template <> struct emit_kind<fp8_e4_t> { static constexpr int v = 3; };
template <> struct emit_kind<fp8_e5_t> { static constexpr int v = 3; };
template <> struct emit_kind<float> { static constexpr int v = 4; };

template <typename TA, typename TB> TL_DEVICE floatx16 mma_f8_32x32(long a, long b, floatx16 c) {
  if constexpr (fp8_fmt<TA>::code == 0 && fp8_fmt<TB>::code == 0)
    return __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(a, b, c, 0, 0, 0);
  else if constexpr (fp8_fmt<TA>::code == 0)
    return __builtin_amdgcn_mfma_f32_32x32x16_fp8_bf8(a, b, c, 0, 0, 0);
  else if constexpr (fp8_fmt<TB>::code == 0)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf8_fp8(a, b, c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf8_bf8(a, b, c, 0, 0, 0);
}

template <int MS, int KPER, typename TA, typename TB, typename TC>
TL_DEVICE void mfma_emit(TC* c, const TA* a, const TB* b) {
  constexpr int K = emit_kind<TA>::v;
  static_assert(K != 0 && K == emit_kind<TB>::v, "mfma_emit: unsupported operand types");
  static_assert(MS == 16 || MS == 32, "mfma_emit: 16x16 or 32x32 tiles");
  typedef typename std::conditional<MS == 16, floatx4, floatx16>::type FAcc;
  if constexpr (K == 1) {
    static_assert(KPER == 8, "f16/bf16 MFMA: 8 k per lane");
    static_assert(std::is_same<TA, TB>::value, "f16/bf16 MFMA: same operand type");
    if constexpr (MS == 16) {
      typedef typename mfma_traits<TA>::frag F;
      floatx4 cv = *reinterpret_cast<floatx4*>(c);
      cv = mfma_traits<TA>::mma16(*reinterpret_cast<const F*>(a), *reinterpret_cast<const F*>(b), cv);
      *reinterpret_cast<floatx4*>(c) = cv;
    } else {
      typedef typename mfma32_traits<TA>::frag F;
      floatx16 cv = *reinterpret_cast<floatx16*>(c);
      cv = mfma32_traits<TA>::mma(*reinterpret_cast<const F*>(a), *reinterpret_cast<const F*>(b), cv);
      *reinterpret_cast<floatx16*>(c) = cv;
    }
  } else if constexpr (K == 2) {
    static_assert(KPER == 16, "int8 MFMA: 16 k per lane");
    intx4 av = *reinterpret_cast<const intx4*>(a), bv = *reinterpret_cast<const intx4*>(b);
    if constexpr (MS == 16) {
      intx4 cv = *reinterpret_cast<intx4*>(c);
      *reinterpret_cast<intx4*>(c) = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, cv, 0, 0, 0);
    } else {
      intx16 cv = *reinterpret_cast<intx16*>(c);
      *reinterpret_cast<intx16*>(c) = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, cv, 0, 0, 0);
    }
  } else if constexpr (K == 3) {
    FAcc cv = *reinterpret_cast<FAcc*>(c);
    if constexpr (KPER == 8) {
      const long av = *reinterpret_cast<const long*>(a), bv = *reinterpret_cast<const long*>(b);
      if constexpr (MS == 16)
        cv = mma_f8_32<TA, TB>(av, bv, cv);
      else
        cv = mma_f8_32x32<TA, TB>(av, bv, cv);
    } else {
      static_assert(KPER == 32, "fp8 MFMA: 8 or 32 k per lane");
      const intx8 av = *reinterpret_cast<const intx8*>(a), bv = *reinterpret_cast<const intx8*>(b);
      if constexpr (MS == 16)
        cv = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, cv, fp8_fmt<TA>::code, fp8_fmt<TB>::code, 0,
                                                              0, 0, 0);
      else
        cv = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, cv, fp8_fmt<TA>::code, fp8_fmt<TB>::code, 0,
                                                             0, 0, 0);
    }
    *reinterpret_cast<FAcc*>(c) = cv;
  } else {
    static_assert(KPER == 1, "fp32 MFMA: 1 k per lane");
    FAcc cv = *reinterpret_cast<FAcc*>(c);
    if constexpr (MS == 16)
      cv = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], cv, 0, 0, 0);
    else
      cv = __builtin_amdgcn_mfma_f32_32x32x2f32(a[0], b[0], cv, 0, 0, 0);
    *reinterpret_cast<FAcc*>(c) = cv;
  }
}

// contiguous register run <- LDS / global (16-byte aligned runs: ds_read_b128 / global_load_dwordx4)
template <typename T, int N> TL_DEVICE void ld_run(T* dst, const T* src) {
  constexpr int BYTES = N * (int)sizeof(T);
  if constexpr (BYTES % 16 == 0) {
#pragma unroll
    for (int i = 0; i < BYTES / 16; ++i)
      reinterpret_cast<intx4*>(dst)[i] = reinterpret_cast<const intx4*>(src)[i];
  } else if constexpr (BYTES == 8) {
    *reinterpret_cast<long*>(dst) = *reinterpret_cast<const long*>(src);
  } else if constexpr (BYTES == 4) {
    *reinterpret_cast<int*>(dst) = *reinterpret_cast<const int*>(src);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) dst[i] = src[i];
  }
}

}  // namespace tl


namespace tl {

// ---------------------------------------------------------------------------------------------
// 2:4 structured-sparse A: v_smfmac_f32_16x16x64_{f16,bf16} (T.gemm_sp; reference
// src/op/gemm_sp.cc:147 + src/tl_templates/cuda/gemm_sp*.h, which use NVIDIA mma.sp).
// Operand map measured on gfx950 (scripts/probes/smfmac_map.hip): per 64-wide K step, lane
// (i = l&15, g = l>>4) supplies the 8 kept A values of original K [16g, 16g+16) of row i (8
// consecutive compressed elements = one ds_read_b128), their 2-bit in-group positions in the low
// 16 bits of the index VGPR (value v at bits 2v), and 16 B values whose elements 0..7 / 8..15
// are the dense 16x16x32 B fragments of K steps k0 and k0+32.  Issued as smfmac(A, B): C is in
// the direct MFMA layout C[4g + v][i].
template <typename T> struct smfmac_traits;
template <> struct smfmac_traits<half_t> {
  typedef half_t bfrag __attribute__((ext_vector_type(16)));
  TL_DEVICE static floatx4 mma(halfx8 a, bfrag b, floatx4 c, int idx) {
    return __builtin_amdgcn_smfmac_f32_16x16x64_f16(a, b, c, idx, 0, 0);
  }
};
template <> struct smfmac_traits<bfloat16_t> {
  typedef bfloat16_t bfrag __attribute__((ext_vector_type(16)));
  TL_DEVICE static floatx4 mma(bf16x8 a, bfrag b, floatx4 c, int idx) {
    return __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c, idx, 0, 0);
  }
};

// A_sp: LDS [M][K/2] (TA=false) or [K/2][M] (TA=true); E: [M][E_COLS] int16 (LDS or global);
// B: [K][N] (TB=false) or [N][K] (TB=true).  C: floatx4 [M_REP][N_REP] per wave, direct layout.
template <typename T, int M, int N, int K, int WARP_M, int WARP_N, bool TA, bool TB, int A_COLS, uint32_t SWZ_A,
          int E_COLS, int B_COLS, uint32_t SWZ_B>
TL_DEVICE void gemm_sp_ss(const T* __restrict__ A, const int16_t* __restrict__ E, const T* __restrict__ B,
                          float* __restrict__ C, int wave_in = -1) {
  typedef smfmac_traits<T> ST;
  typedef typename mfma_traits<T>::frag F;
  typedef typename ST::bfrag BF;
  constexpr int WM = M / WARP_M, WN = N / WARP_N;
  constexpr int M_REP = WM / 16, N_REP = WN / 16, KSTEPS = K / 64;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && K % 64 == 0, "smfmac 16x16x64 tiling");
  const int lane = threadIdx.x & 63;
  const int wave = wave_or(wave_in);
  const int wm = wave / WARP_N, wn = wave % WARP_N;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
#pragma unroll
  for (int kk = 0; kk < KSTEPS; ++kk) {
    F a[M_REP];
    int idx[M_REP];
    BF b[N_REP];
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi) {
      const int m0 = wm * WM + mi * 16;
      a[mi] = ld_operand<T, (TA ? K / 2 : M), A_COLS, SWZ_A, TA, 0>(A, m0, kk * 32, lane);
      idx[mi] = (int)(uint16_t)E[(m0 + (lane & 15)) * E_COLS + kk * 4 + (lane >> 4)];
    }
#pragma unroll
    for (int ni = 0; ni < N_REP; ++ni) {
      const int n0 = wn * WN + ni * 16;
      F lo = ld_operand<T, (TB ? N : K), B_COLS, SWZ_B, !TB, 0>(B, n0, kk * 64, lane);
      F hi = ld_operand<T, (TB ? N : K), B_COLS, SWZ_B, !TB, 0>(B, n0, kk * 64 + 32, lane);
      b[ni] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    }
#pragma unroll
    for (int mi = 0; mi < M_REP; ++mi)
#pragma unroll
      for (int ni = 0; ni < N_REP; ++ni)
        acc[mi * N_REP + ni] = ST::mma(a[mi], b[ni], acc[mi * N_REP + ni], idx[mi]);
  }
}

}  // namespace tl
