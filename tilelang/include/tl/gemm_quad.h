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
//   * quadrant order (0,0) (1,0) (1,1) (0,1) reads A0+B0 / A1 / B1 / nothing; each phase
//     restages ONE half-tile into a slot whose last read was in an earlier phase (P0: B1 of
//     tile t+1; P1-P3: A0 / B0 / A1 of tile t+2) and one counted vmcnt(6) per K tile keeps three
//     half-tiles in flight across the raw barriers.
// Requirements (checked by the pass): A [.., K] and B [.., K] K-contiguous global tensors with
// the whole 256 x (64 n_tiles) blocks in bounds, 16-bit elements, 512 threads.
#pragma once

namespace tl {
namespace quad {

constexpr int HALF = 128 * 64;  // elements of one half-tile slot (16 KiB)

TL_DEVICE void bar() { asm volatile("s_barrier" ::: "memory"); }

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

// A: element (m0, 0) of the block's rows (row stride lda); B: element (n0, 0) (row stride ldb);
// lds: 64 KiB (2 stages x [256][64]) for the A slots and 64 KiB for the B slots; C: the wave's
// gemm_ss accumulator (32 floatx4).  Ends with every LDS-DMA retired and a barrier passed.
template <typename T>
TL_DEVICE void gemm_quad_nt(const T* __restrict__ A, int lda, const T* __restrict__ B, int ldb, int n_tiles,
                            T* lds_a, T* lds_b, float* __restrict__ C, int wave) {
  using namespace quad;
  typedef typename mfma_traits<T>::frag F;
  floatx4* acc = reinterpret_cast<floatx4*>(C);
  const int NT = n_tiles;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wm = wave >> 1, wn = wave & 1;

  // LDS-DMA: a half-tile is 1024 16-byte chunks, chunk q = j*512 + tid (j = 0, 1) -> LDS row
  // j*64 + rr, position tid & 7 holding global chunk (tid & 7) ^ ((row >> 1) & 7).
  //   A half qa: LDS row j*64 + rr = block row (2j + (rr >> 5)) * 64 + qa * 32 + (rr & 31)
  //   B half qb: LDS row j*64 + rr = block col j*128 + qb*64 + rr
  // so ONE per-lane offset per operand; the (slot, j, tile) parts go to the scalar offset
  const int rr = tid >> 3;
  const int dc = (tid & 7) ^ ((tid >> 4) & 7);
  const uint32_t voffa = (uint32_t)((((rr >> 5) * 64 + (rr & 31)) * lda + dc * 8) * (int)sizeof(T));
  const uint32_t voffb = (uint32_t)((rr * ldb + dc * 8) * (int)sizeof(T));
  const __amdgpu_buffer_rsrc_t ra = make_rsrc(A, (uint32_t)((255 * lda + 64 * NT) * (int)sizeof(T)));
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(B, (uint32_t)((255 * ldb + 64 * NT) * (int)sizeof(T)));
  T* da = lds_a + wave * 512;
  T* db = lds_b + wave * 512;
  // slot s of buffer b: A slots (s = 0, 1) in lds_a, B slots (s = 2, 3) in lds_b
  auto stage = [&](int buf, int slot, int tile) {
    const int kb = tile * 64 * (int)sizeof(T);
    if (slot < 2) {
      T* l = da + (buf * 2 + slot) * HALF;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)l, 16, voffa, kb + (slot * 32) * lda * (int)sizeof(T),
                                                0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void_t*)(l + 4096), 16, voffa,
                                                kb + (128 + slot * 32) * lda * (int)sizeof(T), 0, 0);
    } else {
      T* l = db + (buf * 2 + slot - 2) * HALF;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)l, 16, voffb, kb + ((slot - 2) * 64) * ldb * (int)sizeof(T),
                                                0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void_t*)(l + 4096), 16, voffb,
                                                kb + (128 + (slot - 2) * 64) * ldb * (int)sizeof(T), 0, 0);
    }
  };
  // operand reads: LDS row r0 + (lane & 15), chunk kk*4 + (lane >> 4), swizzled by (lane >> 1) & 7
  const int lrow = (lane & 15) * 64;
  const int sw = (lane >> 1) & 7;
  const int cx[2] = {((lane >> 4) ^ sw) * 8, ((4 + (lane >> 4)) ^ sw) * 8};

  // prologue: tile 0 (all four slots) and tile 1's A0 / B0 / A1 (what P1-P3 of tile -1 stage)
  stage(0, 0, 0);
  stage(0, 2, 0);
  stage(0, 1, 0);
  stage(0, 3, 0);
  if (NT > 1) {
    stage(1, 0, 1);
    stage(1, 2, 1);
    stage(1, 1, 1);
    wait_vmcnt<6>();
  } else {
    wait_vmcnt<0>();
  }
  bar();

  F fa0[2][2], fa1[2][2], fb[4][2];
#define TL_QUAD_PHASE(BUF, P, T_)                                                              \
  {                                                                                            \
    constexpr int SA = (BUF) * 2 * HALF;                                                       \
    if constexpr (P == 0) {                                                                    \
      read_a<T, SA>(lds_a, fa0, wm, lrow, cx);                                                 \
      read_b<T, SA>(lds_b, fb, wn, lrow, cx);                                                  \
      if ((T_) + 1 < NT) stage((BUF) ^ 1, 3, (T_) + 1);                                        \
      mma<T, 0, 0>(fa0, fb, acc);                                                              \
    } else if constexpr (P == 1) {                                                             \
      read_a<T, SA + HALF>(lds_a, fa1, wm, lrow, cx);                                          \
      if ((T_) + 2 < NT) stage(BUF, 0, (T_) + 2);                                              \
      mma<T, 1, 0>(fa1, fb, acc);                                                              \
    } else if constexpr (P == 2) {                                                             \
      read_b<T, SA + HALF>(lds_b, fb, wn, lrow, cx);                                           \
      if ((T_) + 2 < NT) stage(BUF, 2, (T_) + 2);                                              \
      mma<T, 1, 1>(fa1, fb, acc);                                                              \
    } else {                                                                                   \
      if ((T_) + 2 < NT) stage(BUF, 1, (T_) + 2);                                              \
      mma<T, 0, 1>(fa0, fb, acc);                                                              \
      if ((T_) + 2 < NT) wait_vmcnt<6>();                                                      \
      else if ((T_) + 1 < NT) wait_vmcnt<0>();                                                 \
    }                                                                                          \
    bar();                                                                                     \
  }

  for (int t = 0; t < NT; t += 2) {
    TL_QUAD_PHASE(0, 0, t)
    TL_QUAD_PHASE(0, 1, t)
    TL_QUAD_PHASE(0, 2, t)
    TL_QUAD_PHASE(0, 3, t)
    if (t + 1 < NT) {
      TL_QUAD_PHASE(1, 0, t + 1)
      TL_QUAD_PHASE(1, 1, t + 1)
      TL_QUAD_PHASE(1, 2, t + 1)
      TL_QUAD_PHASE(1, 3, t + 1)
    }
  }
#undef TL_QUAD_PHASE
}

}  // namespace tl
