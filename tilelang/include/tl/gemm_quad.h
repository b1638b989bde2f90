// tl/gemm_quad.h — whole-K-loop "quadrant" GEMM schedule for the 256x256 NT tile with 128-byte K
// tiles (K = 64 fp16/bf16, or K = 128 fp8 on the scaled 16x16x128 MFMA) on gfx950.
//
// Selected by the software-pipeline pass (transform/pipeline.py, _quad_schedule) for the canonical
//     for k in T.Pipelined(K / 64, num_stages=2):
//         T.copy(A[m0:m0+256, k*64:+64], A_s); T.copy(B[n0:n0+256, k*64:+64], B_s)
//         T.gemm(A_s, B_s, C, transpose_B=True)            # 512 threads, 4x2 waves
// The accumulator layout is tl::gemm_ss's (wave (wm, wn) = (wave / 2, wave % 2) owns the
// contiguous 64x128 piece, acc[mi * 8 + ni]), so the DSL's epilogue is unchanged.
//
// Schedule (MI355X guide, "The 256^2 8-phase template", T2-T5; measured against the K-half
// schedule of pipeline.py in scripts/proto/gemm_8ph_ab.py):
//   * a K tile is four phases; phase (qa, qb) computes, on every wave, the 32x64 quadrant
//     rows wm*64 + qa*32 + [0, 32) x cols wn*128 + qb*64 + [0, 64): 16 MFMAs 16x16x32 (fp8: 8
//     scaled 16x16x128 MFMAs of twice the cycles -- the same MFMA time per byte of tile).
//   * LDS holds two K tiles as eight [128][64] half-tile slots: A half qa = block rows
//     {wm*64 + qa*32 + r} (four 32-row groups), B half qb = block cols {wn*128 + qb*64 + c}
//     (two 64-col groups), gathered by the per-lane LDS-DMA source address; 16-byte chunks are
//     XOR-swizzled by (row >> 1) & 7, conflict-free for the ds_read_b128 operand pattern.
//   * quadrant order (0,0) (1,0) (1,1) (0,1) reads A0+B0 / A1 / B1 / nothing; a barrier after
//     the second and the fourth phase; each half-tile is restaged into a slot whose last read
//     precedes the barrier just passed (B1 of tile t+1 in phase 0; A0, B0, A1 of tile t+2 in
//     phases 2-3), and one counted vmcnt(6) per K tile keeps three half-tiles in flight.
// Requirements (checked by the pass): A [.., K] and B [.., K] K-contiguous global tensors with
// the whole 256 x (K-tile n_tiles) blocks in bounds, 16-bit or fp8 elements, 512 threads.
#pragma once

namespace tl {
namespace quad {

// K-tile geometry in bytes: every row of a K tile is 128 bytes (64 fp16/bf16 or 128 fp8 elements),
// eight 16-byte chunks; a half-tile slot is 128 rows (16 KiB)
template <typename T> struct geo {
  static constexpr int ES = (int)sizeof(T);
  static constexpr int KE = 128 / ES;     // elements of a K-tile row
  static constexpr int CE = 16 / ES;      // elements of a 16-byte chunk
  static constexpr int HALF = 128 * KE;   // elements of a half-tile slot
};

// operand fragments of one K tile: two 16x16x32 fp16/bf16 fragments (one 16-byte read each), or
// ONE 32-byte fp8 fragment of the scaled 16x16x128 MFMA (its two 16-byte reads land in the two
// halves of the 8-register tuple the MFMA takes: no copies)
template <typename T, bool F8 = sizeof(T) == 1> struct qfrag {
  typedef typename mfma_traits<T>::frag F;
  static constexpr int KK = 2;
};
template <typename T> struct qfrag<T, true> {
  typedef intx8 F;
  static constexpr int KK = 1;
};

TL_DEVICE void bar() { asm volatile("s_barrier" ::: "memory"); }
TL_DEVICE const int* no_rows() { return nullptr; }  // dense A: no row list

// The arguments are block-uniform by construction, but values the compiler cannot prove
// uniform (e.g. an expert id loaded from a device table) would put the buffer resources in VGPRs
// and wrap every LDS-DMA in a readfirstlane waterfall loop: make them scalar.
TL_DEVICE int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
template <typename P> TL_DEVICE P* uni_ptr(P* p) {
  const unsigned long long v = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (P*)(((unsigned long long)hi << 32) | lo);
}

// fragments i = 0..N-1 of LDS rows r0 + 16 i + (lane & 15), chunks cx[0] / cx[1] of the K tile
template <typename T, int SLOT_OFF, int N>
TL_DEVICE void read_rows(const T* lds, typename qfrag<T>::F (&f)[N][qfrag<T>::KK], int r0, int lrow,
                         const int (&cx)[2]) {
  typedef typename qfrag<T>::F F;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const T* p = lds + SLOT_OFF + (r0 + i * 16) * geo<T>::KE + lrow;
    if constexpr (qfrag<T>::KK == 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) f[i][kk] = *reinterpret_cast<const F*>(p + cx[kk]);
    } else {
      const intx4 lo = *reinterpret_cast<const intx4*>(p + cx[0]);
      const intx4 hi = *reinterpret_cast<const intx4*>(p + cx[1]);
      f[i][0] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  }
}

// acc[BASE + mi * RS + ni] += A fragment mi x B fragment ni over the K tile: two 16x16x32 MFMAs
// (kk outer, so consecutive MFMAs hit different accumulators), or for fp8 ONE 16x16x128 f8f6f4
// MFMA (the same chunk permutation of K on both operands).  Scale operands 0 select the unscaled
// v_mfma_f32_16x16x128_f8f6f4; the unit-scale (127) form is the two-word v_mfma_scale, whose
// register constraints spilled ~130 VGPRs of this loop (256 + spills vs 223).
template <typename T, int BASE, int RS, int MR, int NR>
TL_DEVICE void mma_blk(const typename qfrag<T>::F (&a)[MR][qfrag<T>::KK],
                       const typename qfrag<T>::F (&b)[NR][qfrag<T>::KK], floatx4* acc) {
  if constexpr (qfrag<T>::KK == 1) {
#pragma unroll
    for (int mi = 0; mi < MR; ++mi)
#pragma unroll
      for (int ni = 0; ni < NR; ++ni) {
        floatx4& c = acc[BASE + mi * RS + ni];
        c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(b[ni][0], a[mi][0], c, fp8_fmt<T>::code,
                                                              fp8_fmt<T>::code, 0, 0, 0, 0);
      }
  } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int mi = 0; mi < MR; ++mi)
#pragma unroll
        for (int ni = 0; ni < NR; ++ni) {
          floatx4& c = acc[BASE + mi * RS + ni];
          c = mfma_traits<T>::mma16(b[ni][kk], a[mi][kk], c);
        }
  }
}

}  // namespace quad

// The loop, generalised:
//   GATHER: A rows come from the index list `rows` (the tile's 256 rows, then EXT rows) -- or,
//     with `rows` null, are row0 + 0..255+EXT: A is the tensor base, `a_rows` its row count; a
//     negative / out-of-range row reads zeros (the buffer resource's range check), as
//     T.gather_rows and the pipeline's out-of-range LDS-DMA.
//   EXT (> 0, 32): a 32 x 256 extension GEMM of the extra EXT rows on the SAME B tile, result in
//     Cx with tl::gemm_ss's 1x8-wave (FullCol) layout; its rows are staged one DMA per thread per
//     K tile (waves 4-7 duplicate waves 0-3: the same bytes to the same LDS, so every wave counts
//     the same DMAs) and multiplied in phase 1, where both B halves of the tile are resident.
//   m_limit: T.gemm(valid_m=): waves whose 64 rows all lie at or past it skip their reads and
//     MFMAs (not the DMAs or barriers); the extension runs only if m_limit > 256.
//   BROWS: B's rows are b_row0 + 0..255 of the tensor B (its base), range-checked against b_rows
//     (ragged N: rows past the tensor read zeros).
//   KTAIL: the last K tile runs past the rows' end k_len (elements, k_len * sizeof(T) % 16 == 0):
//     its 16-byte chunks at or past k_len read zeros (the lane's offset is replaced by the buffer
//     resource's range for that tile only), so a ragged K needs no padded copy.
// Every zero-filled load uses an offset equal to its resource's range (not a wrapping sentinel):
// out of range whether or not the hardware adds the scalar offset before the range check.
template <typename T, bool GATHER, int EXT, bool BROWS = false, bool KTAIL = false>
TL_DEVICE void gemm_quad_nt_x(const T* __restrict__ A, int lda, const int* __restrict__ rows, int row0, int a_rows,
                              const T* __restrict__ B, int ldb, int n_tiles, T* lds_a, T* lds_b, T* lds_x,
                              float* __restrict__ C, float* __restrict__ Cx, int m_limit, int wave, int b_row0 = 0,
                              int b_rows = 0, int k_len = 0) {
  using namespace quad;
  typedef typename qfrag<T>::F F;
  constexpr int KE = geo<T>::KE, CE = geo<T>::CE, HALF = geo<T>::HALF;
  static_assert(EXT == 0 || EXT == 32, "extension rows: 0 or 32");
  A = uni_ptr(A);
  B = uni_ptr(B);
  lda = uni(lda);
  ldb = uni(ldb);
  n_tiles = uni(n_tiles);
  row0 = uni(row0);
  a_rows = uni(a_rows);
  m_limit = uni(m_limit);
  b_row0 = uni(b_row0);
  b_rows = uni(b_rows);
  k_len = uni(k_len);
  constexpr int ES = (int)sizeof(T);
  floatx4* acc = reinterpret_cast<floatx4*>(C);
  const int NT = n_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;
  // wave-uniform guards; the loop is instantiated per (live, xlive) combination below so no
  // branch splits a phase
  const bool live = wm * 64 < m_limit;
  const bool xlive = EXT > 0 && m_limit > 256;

  // LDS-DMA: a half-tile is 1024 16-byte chunks, chunk q = j*512 + tid (j = 0, 1) -> LDS row
  // j*64 + rr, position tid & 7 holding global chunk (tid & 7) ^ ((row >> 1) & 7).
  //   A half qa: LDS row j*64 + rr = block row (2j + (rr >> 5)) * 64 + qa * 32 + (rr & 31)
  //   B half qb: LDS row j*64 + rr = block col j*128 + qb*64 + rr
  // dense A: ONE per-lane offset, the (slot, j, tile) parts in the scalar offset; gathered A: one
  // per-lane offset per (qa, j) from the row list
  const int rr = tid >> 3;
  const int dc = (tid & 7) ^ ((tid >> 4) & 7);
  uint32_t voffa[2][2];
  __amdgpu_buffer_rsrc_t ra;
  uint32_t ra_n;  // the A resource's range in bytes: an offset equal to it reads zeros
  if constexpr (GATHER) {
    ra_n = (uint32_t)(a_rows * lda * ES);
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int br = (2 * j + (rr >> 5)) * 64 + qa * 32 + (rr & 31);
        const int src = rows ? rows[br] : row0 + br;
        voffa[qa][j] = (src >= 0 && src < a_rows) ? (uint32_t)((src * lda + dc * CE) * ES) : ra_n;
      }
    ra = make_rsrc(A, ra_n);
  } else {
    ra_n = (uint32_t)(((255 + EXT) * lda + KE * NT) * ES);
    const uint32_t v = (uint32_t)((((rr >> 5) * 64 + (rr & 31)) * lda + dc * CE) * ES);
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int j = 0; j < 2; ++j) voffa[qa][j] = v;
    ra = make_rsrc(A, ra_n);
  }
  uint32_t voffx = 0;
  if constexpr (EXT > 0) {
    const int xr = (tid & 255) >> 3;
    if constexpr (GATHER) {
      const int src = rows ? rows[256 + xr] : row0 + 256 + xr;
      voffx = (src >= 0 && src < a_rows) ? (uint32_t)((src * lda + dc * CE) * ES) : ra_n;
    } else {
      voffx = (uint32_t)(((256 + xr) * lda + dc * CE) * ES);
    }
  }
  // B: one per-lane offset (slot and half rows in the scalar offset), or per (half, j) row offsets
  // range-checked against b_rows (BROWS; B is then the tensor base and rows start at b_row0)
  uint32_t voffb[2][2];
  uint32_t rb_n;
  if constexpr (BROWS) {
    rb_n = (uint32_t)(b_rows * ldb * ES);
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int src = b_row0 + j * 128 + qb * 64 + rr;
        voffb[qb][j] = src < b_rows ? (uint32_t)((src * ldb + dc * CE) * ES) : rb_n;
      }
  } else {
    rb_n = (uint32_t)((255 * ldb + KE * NT) * ES);
    const uint32_t v = (uint32_t)((rr * ldb + dc * CE) * ES);
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int j = 0; j < 2; ++j) voffb[qb][j] = v;
  }
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, rb_n);
  // KTAIL: the offsets of the LAST K tile, computed once: a lane whose chunk lies at or past k_len
  // reads zeros there (the chunk index is per lane); stage() picks them with a uniform branch on
  // the tile, so the other tiles' DMAs carry no per-lane select
  const bool chunk_in = !KTAIL || (NT - 1) * KE + dc * CE < k_len;
  uint32_t voffa_t[2][2], voffb_t[2][2], voffx_t = ra_n;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      voffa_t[q][j] = chunk_in ? voffa[q][j] : ra_n;
      voffb_t[q][j] = chunk_in ? voffb[q][j] : rb_n;
    }
  if constexpr (EXT > 0) voffx_t = chunk_in ? voffx : ra_n;
  // each wave's 64 lanes fill 1 KiB of a slot per DMA (lane-linear destination)
  T* da = lds_a + wave * 8 * KE;
  T* db = lds_b + wave * 8 * KE;
  // slot s of buffer b: A slots (s = 0, 1) in lds_a, B slots (s = 2, 3) in lds_b
  auto stage_with = [&](int buf, int slot, int tile, const uint32_t (&va)[2][2], const uint32_t (&vb)[2][2]) {
    const int kb = tile * 128;  // bytes
    if (slot < 2) {
      T* l = da + (buf * 2 + slot) * HALF;
      const int s0 = GATHER ? kb : kb + (slot * 32) * lda * ES;
      const int s1 = GATHER ? kb : kb + (128 + slot * 32) * lda * ES;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)l, 16, va[slot][0], s0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(l + 64 * KE), 16, va[slot][1], s1, 0, 0);
    } else {
      T* l = db + (buf * 2 + slot - 2) * HALF;
      const int q = slot - 2;
      const int s0 = BROWS ? kb : kb + (q * 64) * ldb * ES;
      const int s1 = BROWS ? kb : kb + (128 + q * 64) * ldb * ES;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)l, 16, vb[q][0], s0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)(l + 64 * KE), 16, vb[q][1], s1, 0, 0);
    }
  };
  auto stage = [&](int buf, int slot, int tile) {
    if constexpr (KTAIL) {
      if (tile == NT - 1) {
        stage_with(buf, slot, tile, voffa_t, voffb_t);
        return;
      }
    }
    stage_with(buf, slot, tile, voffa, voffb);
  };
  auto stage_x = [&](int buf, int tile) {
    if constexpr (EXT > 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(lds_x + buf * 32 * KE + (wave & 3) * 8 * KE), 16,
                                                (KTAIL && tile == NT - 1) ? voffx_t : voffx, tile * 128, 0, 0);
  };
  constexpr int XW = EXT > 0 ? 1 : 0;  // extension DMAs per thread per K tile
  // operand reads: LDS row r0 + (lane & 15), chunk kk*4 + (lane >> 4), swizzled by (lane >> 1) & 7
  const int lrow = (lane & 15) * KE;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {((lane >> 4) ^ sw) * CE, ((4 + (lane >> 4)) ^ sw) * CE};
  // extension operands of wave w: B cols w*32 + [0, 32) = half qb = (w >> 1) & 1, LDS rows
  // (w >> 2) * 64 + (w & 1) * 32 + [0, 32) of that slot
  const int xqb = (wave >> 1) & 1;
  const int xrow = ((wave >> 2) * 64 + (wave & 1) * 32) * KE;

  // prologue: tile 0 (+ its extension rows) and what P1-P3 of tile -1 stage: tile 1's A0,
  // B0 + extension, A1
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  stage(0, 3, 0);
  stage_x(0, 0);
  if (NT > 1) {
    stage(1, 0, 1);
    stage(1, 2, 1);
    stage_x(1, 1);
    stage(1, 1, 1);
    wait_vmcnt<6 + XW>();
  } else {
    wait_vmcnt<0>();
  }
  bar();

  constexpr int KK = qfrag<T>::KK;
  F fa0[2][KK], fa1[2][KK], fb[4][KK];
  // the younger half of the workgroup (waves 4-7) at issue priority 1 for the loop (guide T5
  // static form: +0.5 %, profiles/r5/proto_8pb_single.log)
  if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  // quadrant order (0,0) (1,0) (1,1) (0,1) -- reads A0+B0 / A1 (+ extension) / B1 / nothing;
  // a barrier after P1 and after P3 only (two per K tile: +2 % over one per phase,
  // profiles/r5/proto_8pb_merge.log); restaging after the barrier that retires a slot's reads:
  // P0 B1 of tile t+1, P2 A0 + B0 (+ extension), P3 A1 of tile t+2
#define TL_QUAD_PHASE(BUF, P, T_)                                                              \
  {                                                                                            \
    constexpr int SA = (BUF) * 2 * HALF;                                                       \
    if constexpr (P == 0) {                                                                    \
      if constexpr (LIVE_) {                                                                   \
        read_rows<T, SA>(lds_a, fa0, wm * 32, lrow, cx);                                       \
        read_rows<T, SA>(lds_b, fb, wn * 64, lrow, cx);                                        \
      }                                                                                        \
      if ((T_) + 1 < NT) stage((BUF) ^ 1, 3, (T_) + 1);                                        \
      if constexpr (LIVE_) mma_blk<T, 0, 8>(fa0, fb, acc);                                     \
    } else if constexpr (P == 1) {                                                             \
      if constexpr (LIVE_) read_rows<T, SA + HALF>(lds_a, fa1, wm * 32, lrow, cx);             \
      if constexpr (LIVE_) mma_blk<T, 16, 8>(fa1, fb, acc);                                    \
      if constexpr (EXT > 0) {                                                                 \
        if constexpr (XLIVE_) {                                                                \
          F xa[2][KK], xb[2][KK];                                                              \
          read_rows<T, 0>(lds_x + (BUF) * 32 * KE, xa, 0, lrow, cx);                           \
          read_rows<T, 0>(lds_b + (SA + xqb * HALF) + xrow, xb, 0, lrow, cx);                  \
          mma_blk<T, 0, 2>(xa, xb, reinterpret_cast<floatx4*>(Cx));                            \
        }                                                                                      \
      }                                                                                        \
    } else if constexpr (P == 2) {                                                             \
      if constexpr (LIVE_) read_rows<T, SA + HALF>(lds_b, fb, wn * 64, lrow, cx);              \
      if ((T_) + 2 < NT) {                                                                     \
        stage(BUF, 0, (T_) + 2);                                                               \
        stage(BUF, 2, (T_) + 2);                                                               \
        stage_x(BUF, (T_) + 2);                                                                \
      }                                                                                        \
      if constexpr (LIVE_) mma_blk<T, 20, 8>(fa1, fb, acc);                                    \
    } else {                                                                                   \
      if ((T_) + 2 < NT) stage(BUF, 1, (T_) + 2);                                              \
      if constexpr (LIVE_) mma_blk<T, 4, 8>(fa0, fb, acc);                                     \
      if ((T_) + 2 < NT) wait_vmcnt<6 + XW>();                                                 \
      else if ((T_) + 1 < NT) wait_vmcnt<0>();                                                 \
    }                                                                                          \
    if constexpr (P == 1 || P == 3) bar();                                                     \
  }

#define TL_QUAD_LOOP(L_, X_)                                                                   \
  {                                                                                            \
    constexpr bool LIVE_ = L_, XLIVE_ = X_;                                                    \
    /* never unrolled: a compile-time K of 2-16 tiles was unrolled whole and spilled          \
       (16-40 VGPRs; fp8 K = 1024: 110 -> 83 us) */                                             \
    _Pragma("nounroll") for (int t = 0; t < NT; t += 2) {                                      \
      TL_QUAD_PHASE(0, 0, t)                                                                   \
      TL_QUAD_PHASE(0, 1, t)                                                                   \
      TL_QUAD_PHASE(0, 2, t)                                                                   \
      TL_QUAD_PHASE(0, 3, t)                                                                   \
      if (t + 1 < NT) {                                                                        \
        TL_QUAD_PHASE(1, 0, t + 1)                                                             \
        TL_QUAD_PHASE(1, 1, t + 1)                                                             \
        TL_QUAD_PHASE(1, 2, t + 1)                                                             \
        TL_QUAD_PHASE(1, 3, t + 1)                                                             \
      }                                                                                        \
    }                                                                                          \
  }
  if (live) {
    if (EXT > 0 && xlive) TL_QUAD_LOOP(true, EXT > 0)
    else TL_QUAD_LOOP(true, false)
  } else {
    TL_QUAD_LOOP(false, false)
  }
#undef TL_QUAD_LOOP
#undef TL_QUAD_PHASE
  __builtin_amdgcn_s_setprio(0);
}

// Dense form: A = element (m0, 0) of the block's rows (row stride lda), B = element (n0, 0)
// (row stride ldb); lds_a / lds_b: 64 KiB each (2 stages x [256][64]); C: the wave's gemm_ss
// accumulator (32 floatx4).  Ends with every LDS-DMA retired and a barrier passed.
template <typename T>
TL_DEVICE void gemm_quad_nt(const T* __restrict__ A, int lda, const T* __restrict__ B, int ldb, int n_tiles,
                            T* lds_a, T* lds_b, float* __restrict__ C, int wave, int m_limit = 0x3fffffff) {
  gemm_quad_nt_x<T, false, 0>(A, lda, nullptr, 0, 0, B, ldb, n_tiles, lds_a, lds_b, nullptr, C, nullptr, m_limit,
                              wave);
}

}  // namespace tl
