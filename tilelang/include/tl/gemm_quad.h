// tl/gemm_quad.h — whole-K-loop "quadrant" GEMM schedule for the 256x256x64 NT tile (gfx950).
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
//     rows wm*64 + qa*32 + [0, 32) x cols wn*128 + qb*64 + [0, 64): 16 MFMAs 16x16x32.
//   * LDS holds two K tiles as eight [128][64] half-tile slots: A half qa = block rows
//     {wm*64 + qa*32 + r} (four 32-row groups), B half qb = block cols {wn*128 + qb*64 + c}
//     (two 64-col groups), gathered by the per-lane LDS-DMA source address; 16-byte chunks are
//     XOR-swizzled by (row >> 1) & 7, conflict-free for the ds_read_b128 operand pattern.
//   * quadrant order (0,0) (1,0) (1,1) (0,1) reads A0+B0 / A1 / B1 / nothing; a barrier after
//     the second and the fourth phase; each half-tile is restaged into a slot whose last read
//     precedes the barrier just passed (B1 of tile t+1 in phase 0; A0, B0, A1 of tile t+2 in
//     phases 2-3), and one counted vmcnt(6) per K tile keeps three half-tiles in flight.
// Requirements (checked by the pass): A [.., K] and B [.., K] K-contiguous global tensors with
// the whole 256 x (64 n_tiles) blocks in bounds, 16-bit elements, 512 threads.
#pragma once

namespace tl {
namespace quad {

constexpr int HALF = 128 * 64;  // elements of one half-tile slot (16 KiB)

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

template <typename T, int SLOT_OFF>
TL_DEVICE void read_a(const T* lds, typename mfma_traits<T>::frag (&a)[2][2], int wm, int lrow,
                      const int (&cx)[2]) {
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      a[mi][kk] = *reinterpret_cast<const typename mfma_traits<T>::frag*>(lds + SLOT_OFF + (wm * 32 + mi * 16) * 64 +
                                                                          lrow + cx[kk]);
}

template <typename T, int SLOT_OFF>
TL_DEVICE void read_b(const T* lds, typename mfma_traits<T>::frag (&b)[4][2], int wn, int lrow,
                      const int (&cx)[2]) {
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      b[ni][kk] = *reinterpret_cast<const typename mfma_traits<T>::frag*>(lds + SLOT_OFF + (wn * 64 + ni * 16) * 64 +
                                                                          lrow + cx[kk]);
}

template <typename T, int QA, int QB>
TL_DEVICE void mma(const typename mfma_traits<T>::frag (&a)[2][2], const typename mfma_traits<T>::frag (&b)[4][2],
                   floatx4* acc) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        floatx4& c = acc[(QA * 2 + mi) * 8 + QB * 4 + ni];
        c = mfma_traits<T>::mma16(b[ni][kk], a[mi][kk], c);
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
template <typename T, bool GATHER, int EXT>
TL_DEVICE void gemm_quad_nt_x(const T* __restrict__ A, int lda, const int* __restrict__ rows, int row0, int a_rows,
                              const T* __restrict__ B, int ldb, int n_tiles, T* lds_a, T* lds_b, T* lds_x,
                              float* __restrict__ C, float* __restrict__ Cx, int m_limit, int wave) {
  using namespace quad;
  typedef typename mfma_traits<T>::frag F;
  static_assert(EXT == 0 || EXT == 32, "extension rows: 0 or 32");
  A = uni_ptr(A);
  B = uni_ptr(B);
  lda = uni(lda);
  ldb = uni(ldb);
  n_tiles = uni(n_tiles);
  row0 = uni(row0);
  a_rows = uni(a_rows);
  m_limit = uni(m_limit);
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
  if constexpr (GATHER) {
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int br = (2 * j + (rr >> 5)) * 64 + qa * 32 + (rr & 31);
        const int src = rows ? rows[br] : row0 + br;
        voffa[qa][j] = (src >= 0 && src < a_rows) ? (uint32_t)((src * lda + dc * 8) * ES) : 0xFFFFFFF0u;
      }
    ra = make_rsrc(A, (uint32_t)(a_rows * lda * ES));
  } else {
    const uint32_t v = (uint32_t)((((rr >> 5) * 64 + (rr & 31)) * lda + dc * 8) * ES);
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int j = 0; j < 2; ++j) voffa[qa][j] = v;
    ra = make_rsrc(A, (uint32_t)(((255 + EXT) * lda + 64 * NT) * ES));
  }
  uint32_t voffx = 0;
  if constexpr (EXT > 0) {
    const int xr = (tid & 255) >> 3;
    if constexpr (GATHER) {
      const int src = rows ? rows[256 + xr] : row0 + 256 + xr;
      voffx = (src >= 0 && src < a_rows) ? (uint32_t)((src * lda + dc * 8) * ES) : 0xFFFFFFF0u;
    } else {
      voffx = (uint32_t)(((256 + xr) * lda + dc * 8) * ES);
    }
  }
  const uint32_t voffb = (uint32_t)((rr * ldb + dc * 8) * ES);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, (uint32_t)((255 * ldb + 64 * NT) * ES));
  T* da = lds_a + wave * 512;
  T* db = lds_b + wave * 512;
  // slot s of buffer b: A slots (s = 0, 1) in lds_a, B slots (s = 2, 3) in lds_b
  auto stage = [&](int buf, int slot, int tile) {
    const int kb = tile * 64 * ES;
    if (slot < 2) {
      T* l = da + (buf * 2 + slot) * HALF;
      const int s0 = GATHER ? kb : kb + (slot * 32) * lda * ES;
      const int s1 = GATHER ? kb : kb + (128 + slot * 32) * lda * ES;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)l, 16, voffa[slot][0], s0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(l + 4096), 16, voffa[slot][1], s1, 0, 0);
    } else {
      T* l = db + (buf * 2 + slot - 2) * HALF;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)l, 16, voffb, kb + ((slot - 2) * 64) * ldb * ES,
                                                0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)(l + 4096), 16, voffb,
                                                kb + (128 + (slot - 2) * 64) * ldb * ES, 0, 0);
    }
  };
  auto stage_x = [&](int buf, int tile) {
    if constexpr (EXT > 0)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(lds_x + buf * 2048 + (wave & 3) * 512), 16, voffx,
                                                tile * 64 * ES, 0, 0);
  };
  constexpr int XW = EXT > 0 ? 1 : 0;  // extension DMAs per thread per K tile
  // operand reads: LDS row r0 + (lane & 15), chunk kk*4 + (lane >> 4), swizzled by (lane >> 1) & 7
  const int lrow = (lane & 15) * 64;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {((lane >> 4) ^ sw) * 8, ((4 + (lane >> 4)) ^ sw) * 8};
  // extension operands of wave w: B cols w*32 + [0, 32) = half qb = (w >> 1) & 1, LDS rows
  // (w >> 2) * 64 + (w & 1) * 32 + [0, 32) of that slot
  const int xqb = (wave >> 1) & 1;
  const int xrow = ((wave >> 2) * 64 + (wave & 1) * 32) * 64;

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

  F fa0[2][2], fa1[2][2], fb[4][2];
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
      if constexpr (LIVE_) {                                                                              \
        read_a<T, SA>(lds_a, fa0, wm, lrow, cx);                                               \
        read_b<T, SA>(lds_b, fb, wn, lrow, cx);                                                \
      }                                                                                        \
      if ((T_) + 1 < NT) stage((BUF) ^ 1, 3, (T_) + 1);                                        \
      if constexpr (LIVE_) mma<T, 0, 0>(fa0, fb, acc);                                                    \
    } else if constexpr (P == 1) {                                                             \
      if constexpr (LIVE_) read_a<T, SA + HALF>(lds_a, fa1, wm, lrow, cx);                                \
      if constexpr (LIVE_) mma<T, 1, 0>(fa1, fb, acc);                                                    \
      if constexpr (EXT > 0) {                                                                 \
        if constexpr (XLIVE_) {                                                                           \
          F xa[2][2], xb[2][2];                                                                \
          const T* xs = lds_x + (BUF) * 2048;                                                  \
          const T* bs = lds_b + (SA + xqb * HALF) + xrow;                                      \
          _Pragma("unroll") for (int i = 0; i < 2; ++i)                                        \
          _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) {                                   \
            xa[i][kk] = *reinterpret_cast<const F*>(xs + i * 16 * 64 + lrow + cx[kk]);          \
            xb[i][kk] = *reinterpret_cast<const F*>(bs + i * 16 * 64 + lrow + cx[kk]);          \
          }                                                                                    \
          floatx4* accx = reinterpret_cast<floatx4*>(Cx);                                      \
          _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                     \
          _Pragma("unroll") for (int mi = 0; mi < 2; ++mi)                                     \
          _Pragma("unroll") for (int ni = 0; ni < 2; ++ni)                                     \
            accx[mi * 2 + ni] = mfma_traits<T>::mma16(xb[ni][kk], xa[mi][kk], accx[mi * 2 + ni]); \
        }                                                                                      \
      }                                                                                        \
    } else if constexpr (P == 2) {                                                             \
      if constexpr (LIVE_) read_b<T, SA + HALF>(lds_b, fb, wn, lrow, cx);                                 \
      if ((T_) + 2 < NT) {                                                                     \
        stage(BUF, 0, (T_) + 2);                                                               \
        stage(BUF, 2, (T_) + 2);                                                               \
        stage_x(BUF, (T_) + 2);                                                                \
      }                                                                                        \
      if constexpr (LIVE_) mma<T, 1, 1>(fa1, fb, acc);                                                    \
    } else {                                                                                   \
      if ((T_) + 2 < NT) stage(BUF, 1, (T_) + 2);                                              \
      if constexpr (LIVE_) mma<T, 0, 1>(fa0, fb, acc);                                                    \
      if ((T_) + 2 < NT) wait_vmcnt<6 + XW>();                                                 \
      else if ((T_) + 1 < NT) wait_vmcnt<0>();                                                 \
    }                                                                                          \
    if constexpr (P == 1 || P == 3) bar();                                                     \
  }

#define TL_QUAD_LOOP(L_, X_)                                                                   \
  {                                                                                            \
    constexpr bool LIVE_ = L_, XLIVE_ = X_;                                                    \
    for (int t = 0; t < NT; t += 2) {                                                          \
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
