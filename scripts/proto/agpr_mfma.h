// generated: MFMA 16x16x32 on literal accumulator registers a[R:R+3] (R = 4k), with the
// registers as clobbers (so the kernel descriptor allocates them and the compiler keeps out)
#pragma once
namespace tl { namespace agpr {
template <int R> struct acc;
template <> struct acc<0> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[0:3], %0, %1, a[0:3]" :: "v"(b), "v"(a) : "a0", "a1", "a2", "a3"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[0:3], %0, %1, a[0:3]" :: "v"(b), "v"(a) : "a0", "a1", "a2", "a3"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a0, 0\n\tv_accvgpr_write_b32 a1, 0\n\tv_accvgpr_write_b32 a2, 0\n\tv_accvgpr_write_b32 a3, 0" ::: "a0", "a1", "a2", "a3"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a0, %0\n\tv_accvgpr_write_b32 a1, %1\n\tv_accvgpr_write_b32 a2, %2\n\tv_accvgpr_write_b32 a3, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a0", "a1", "a2", "a3"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a0\n\tv_accvgpr_read_b32 %1, a1\n\tv_accvgpr_read_b32 %2, a2\n\tv_accvgpr_read_b32 %3, a3" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<4> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[4:7], %0, %1, a[4:7]" :: "v"(b), "v"(a) : "a4", "a5", "a6", "a7"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[4:7], %0, %1, a[4:7]" :: "v"(b), "v"(a) : "a4", "a5", "a6", "a7"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a4, 0\n\tv_accvgpr_write_b32 a5, 0\n\tv_accvgpr_write_b32 a6, 0\n\tv_accvgpr_write_b32 a7, 0" ::: "a4", "a5", "a6", "a7"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a4, %0\n\tv_accvgpr_write_b32 a5, %1\n\tv_accvgpr_write_b32 a6, %2\n\tv_accvgpr_write_b32 a7, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a4", "a5", "a6", "a7"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a4\n\tv_accvgpr_read_b32 %1, a5\n\tv_accvgpr_read_b32 %2, a6\n\tv_accvgpr_read_b32 %3, a7" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<8> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[8:11], %0, %1, a[8:11]" :: "v"(b), "v"(a) : "a8", "a9", "a10", "a11"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[8:11], %0, %1, a[8:11]" :: "v"(b), "v"(a) : "a8", "a9", "a10", "a11"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a8, 0\n\tv_accvgpr_write_b32 a9, 0\n\tv_accvgpr_write_b32 a10, 0\n\tv_accvgpr_write_b32 a11, 0" ::: "a8", "a9", "a10", "a11"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a8, %0\n\tv_accvgpr_write_b32 a9, %1\n\tv_accvgpr_write_b32 a10, %2\n\tv_accvgpr_write_b32 a11, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a8", "a9", "a10", "a11"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a8\n\tv_accvgpr_read_b32 %1, a9\n\tv_accvgpr_read_b32 %2, a10\n\tv_accvgpr_read_b32 %3, a11" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<12> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[12:15], %0, %1, a[12:15]" :: "v"(b), "v"(a) : "a12", "a13", "a14", "a15"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[12:15], %0, %1, a[12:15]" :: "v"(b), "v"(a) : "a12", "a13", "a14", "a15"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a12, 0\n\tv_accvgpr_write_b32 a13, 0\n\tv_accvgpr_write_b32 a14, 0\n\tv_accvgpr_write_b32 a15, 0" ::: "a12", "a13", "a14", "a15"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a12, %0\n\tv_accvgpr_write_b32 a13, %1\n\tv_accvgpr_write_b32 a14, %2\n\tv_accvgpr_write_b32 a15, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a12", "a13", "a14", "a15"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a12\n\tv_accvgpr_read_b32 %1, a13\n\tv_accvgpr_read_b32 %2, a14\n\tv_accvgpr_read_b32 %3, a15" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<16> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[16:19], %0, %1, a[16:19]" :: "v"(b), "v"(a) : "a16", "a17", "a18", "a19"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[16:19], %0, %1, a[16:19]" :: "v"(b), "v"(a) : "a16", "a17", "a18", "a19"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a16, 0\n\tv_accvgpr_write_b32 a17, 0\n\tv_accvgpr_write_b32 a18, 0\n\tv_accvgpr_write_b32 a19, 0" ::: "a16", "a17", "a18", "a19"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a16, %0\n\tv_accvgpr_write_b32 a17, %1\n\tv_accvgpr_write_b32 a18, %2\n\tv_accvgpr_write_b32 a19, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a16", "a17", "a18", "a19"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a16\n\tv_accvgpr_read_b32 %1, a17\n\tv_accvgpr_read_b32 %2, a18\n\tv_accvgpr_read_b32 %3, a19" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<20> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[20:23], %0, %1, a[20:23]" :: "v"(b), "v"(a) : "a20", "a21", "a22", "a23"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[20:23], %0, %1, a[20:23]" :: "v"(b), "v"(a) : "a20", "a21", "a22", "a23"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a20, 0\n\tv_accvgpr_write_b32 a21, 0\n\tv_accvgpr_write_b32 a22, 0\n\tv_accvgpr_write_b32 a23, 0" ::: "a20", "a21", "a22", "a23"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a20, %0\n\tv_accvgpr_write_b32 a21, %1\n\tv_accvgpr_write_b32 a22, %2\n\tv_accvgpr_write_b32 a23, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a20", "a21", "a22", "a23"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a20\n\tv_accvgpr_read_b32 %1, a21\n\tv_accvgpr_read_b32 %2, a22\n\tv_accvgpr_read_b32 %3, a23" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<24> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[24:27], %0, %1, a[24:27]" :: "v"(b), "v"(a) : "a24", "a25", "a26", "a27"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[24:27], %0, %1, a[24:27]" :: "v"(b), "v"(a) : "a24", "a25", "a26", "a27"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a24, 0\n\tv_accvgpr_write_b32 a25, 0\n\tv_accvgpr_write_b32 a26, 0\n\tv_accvgpr_write_b32 a27, 0" ::: "a24", "a25", "a26", "a27"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a24, %0\n\tv_accvgpr_write_b32 a25, %1\n\tv_accvgpr_write_b32 a26, %2\n\tv_accvgpr_write_b32 a27, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a24", "a25", "a26", "a27"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a24\n\tv_accvgpr_read_b32 %1, a25\n\tv_accvgpr_read_b32 %2, a26\n\tv_accvgpr_read_b32 %3, a27" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<28> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[28:31], %0, %1, a[28:31]" :: "v"(b), "v"(a) : "a28", "a29", "a30", "a31"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[28:31], %0, %1, a[28:31]" :: "v"(b), "v"(a) : "a28", "a29", "a30", "a31"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a28, 0\n\tv_accvgpr_write_b32 a29, 0\n\tv_accvgpr_write_b32 a30, 0\n\tv_accvgpr_write_b32 a31, 0" ::: "a28", "a29", "a30", "a31"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a28, %0\n\tv_accvgpr_write_b32 a29, %1\n\tv_accvgpr_write_b32 a30, %2\n\tv_accvgpr_write_b32 a31, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a28", "a29", "a30", "a31"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a28\n\tv_accvgpr_read_b32 %1, a29\n\tv_accvgpr_read_b32 %2, a30\n\tv_accvgpr_read_b32 %3, a31" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<32> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[32:35], %0, %1, a[32:35]" :: "v"(b), "v"(a) : "a32", "a33", "a34", "a35"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[32:35], %0, %1, a[32:35]" :: "v"(b), "v"(a) : "a32", "a33", "a34", "a35"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a32, 0\n\tv_accvgpr_write_b32 a33, 0\n\tv_accvgpr_write_b32 a34, 0\n\tv_accvgpr_write_b32 a35, 0" ::: "a32", "a33", "a34", "a35"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a32, %0\n\tv_accvgpr_write_b32 a33, %1\n\tv_accvgpr_write_b32 a34, %2\n\tv_accvgpr_write_b32 a35, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a32", "a33", "a34", "a35"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a32\n\tv_accvgpr_read_b32 %1, a33\n\tv_accvgpr_read_b32 %2, a34\n\tv_accvgpr_read_b32 %3, a35" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<36> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[36:39], %0, %1, a[36:39]" :: "v"(b), "v"(a) : "a36", "a37", "a38", "a39"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[36:39], %0, %1, a[36:39]" :: "v"(b), "v"(a) : "a36", "a37", "a38", "a39"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a36, 0\n\tv_accvgpr_write_b32 a37, 0\n\tv_accvgpr_write_b32 a38, 0\n\tv_accvgpr_write_b32 a39, 0" ::: "a36", "a37", "a38", "a39"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a36, %0\n\tv_accvgpr_write_b32 a37, %1\n\tv_accvgpr_write_b32 a38, %2\n\tv_accvgpr_write_b32 a39, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a36", "a37", "a38", "a39"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a36\n\tv_accvgpr_read_b32 %1, a37\n\tv_accvgpr_read_b32 %2, a38\n\tv_accvgpr_read_b32 %3, a39" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<40> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[40:43], %0, %1, a[40:43]" :: "v"(b), "v"(a) : "a40", "a41", "a42", "a43"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[40:43], %0, %1, a[40:43]" :: "v"(b), "v"(a) : "a40", "a41", "a42", "a43"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a40, 0\n\tv_accvgpr_write_b32 a41, 0\n\tv_accvgpr_write_b32 a42, 0\n\tv_accvgpr_write_b32 a43, 0" ::: "a40", "a41", "a42", "a43"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a40, %0\n\tv_accvgpr_write_b32 a41, %1\n\tv_accvgpr_write_b32 a42, %2\n\tv_accvgpr_write_b32 a43, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a40", "a41", "a42", "a43"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a40\n\tv_accvgpr_read_b32 %1, a41\n\tv_accvgpr_read_b32 %2, a42\n\tv_accvgpr_read_b32 %3, a43" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<44> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[44:47], %0, %1, a[44:47]" :: "v"(b), "v"(a) : "a44", "a45", "a46", "a47"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[44:47], %0, %1, a[44:47]" :: "v"(b), "v"(a) : "a44", "a45", "a46", "a47"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a44, 0\n\tv_accvgpr_write_b32 a45, 0\n\tv_accvgpr_write_b32 a46, 0\n\tv_accvgpr_write_b32 a47, 0" ::: "a44", "a45", "a46", "a47"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a44, %0\n\tv_accvgpr_write_b32 a45, %1\n\tv_accvgpr_write_b32 a46, %2\n\tv_accvgpr_write_b32 a47, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a44", "a45", "a46", "a47"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a44\n\tv_accvgpr_read_b32 %1, a45\n\tv_accvgpr_read_b32 %2, a46\n\tv_accvgpr_read_b32 %3, a47" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<48> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[48:51], %0, %1, a[48:51]" :: "v"(b), "v"(a) : "a48", "a49", "a50", "a51"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[48:51], %0, %1, a[48:51]" :: "v"(b), "v"(a) : "a48", "a49", "a50", "a51"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a48, 0\n\tv_accvgpr_write_b32 a49, 0\n\tv_accvgpr_write_b32 a50, 0\n\tv_accvgpr_write_b32 a51, 0" ::: "a48", "a49", "a50", "a51"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a48, %0\n\tv_accvgpr_write_b32 a49, %1\n\tv_accvgpr_write_b32 a50, %2\n\tv_accvgpr_write_b32 a51, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a48", "a49", "a50", "a51"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a48\n\tv_accvgpr_read_b32 %1, a49\n\tv_accvgpr_read_b32 %2, a50\n\tv_accvgpr_read_b32 %3, a51" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<52> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[52:55], %0, %1, a[52:55]" :: "v"(b), "v"(a) : "a52", "a53", "a54", "a55"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[52:55], %0, %1, a[52:55]" :: "v"(b), "v"(a) : "a52", "a53", "a54", "a55"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a52, 0\n\tv_accvgpr_write_b32 a53, 0\n\tv_accvgpr_write_b32 a54, 0\n\tv_accvgpr_write_b32 a55, 0" ::: "a52", "a53", "a54", "a55"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a52, %0\n\tv_accvgpr_write_b32 a53, %1\n\tv_accvgpr_write_b32 a54, %2\n\tv_accvgpr_write_b32 a55, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a52", "a53", "a54", "a55"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a52\n\tv_accvgpr_read_b32 %1, a53\n\tv_accvgpr_read_b32 %2, a54\n\tv_accvgpr_read_b32 %3, a55" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<56> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[56:59], %0, %1, a[56:59]" :: "v"(b), "v"(a) : "a56", "a57", "a58", "a59"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[56:59], %0, %1, a[56:59]" :: "v"(b), "v"(a) : "a56", "a57", "a58", "a59"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a56, 0\n\tv_accvgpr_write_b32 a57, 0\n\tv_accvgpr_write_b32 a58, 0\n\tv_accvgpr_write_b32 a59, 0" ::: "a56", "a57", "a58", "a59"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a56, %0\n\tv_accvgpr_write_b32 a57, %1\n\tv_accvgpr_write_b32 a58, %2\n\tv_accvgpr_write_b32 a59, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a56", "a57", "a58", "a59"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a56\n\tv_accvgpr_read_b32 %1, a57\n\tv_accvgpr_read_b32 %2, a58\n\tv_accvgpr_read_b32 %3, a59" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<60> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[60:63], %0, %1, a[60:63]" :: "v"(b), "v"(a) : "a60", "a61", "a62", "a63"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[60:63], %0, %1, a[60:63]" :: "v"(b), "v"(a) : "a60", "a61", "a62", "a63"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a60, 0\n\tv_accvgpr_write_b32 a61, 0\n\tv_accvgpr_write_b32 a62, 0\n\tv_accvgpr_write_b32 a63, 0" ::: "a60", "a61", "a62", "a63"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a60, %0\n\tv_accvgpr_write_b32 a61, %1\n\tv_accvgpr_write_b32 a62, %2\n\tv_accvgpr_write_b32 a63, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a60", "a61", "a62", "a63"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a60\n\tv_accvgpr_read_b32 %1, a61\n\tv_accvgpr_read_b32 %2, a62\n\tv_accvgpr_read_b32 %3, a63" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<64> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[64:67], %0, %1, a[64:67]" :: "v"(b), "v"(a) : "a64", "a65", "a66", "a67"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[64:67], %0, %1, a[64:67]" :: "v"(b), "v"(a) : "a64", "a65", "a66", "a67"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a64, 0\n\tv_accvgpr_write_b32 a65, 0\n\tv_accvgpr_write_b32 a66, 0\n\tv_accvgpr_write_b32 a67, 0" ::: "a64", "a65", "a66", "a67"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a64, %0\n\tv_accvgpr_write_b32 a65, %1\n\tv_accvgpr_write_b32 a66, %2\n\tv_accvgpr_write_b32 a67, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a64", "a65", "a66", "a67"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a64\n\tv_accvgpr_read_b32 %1, a65\n\tv_accvgpr_read_b32 %2, a66\n\tv_accvgpr_read_b32 %3, a67" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<68> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[68:71], %0, %1, a[68:71]" :: "v"(b), "v"(a) : "a68", "a69", "a70", "a71"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[68:71], %0, %1, a[68:71]" :: "v"(b), "v"(a) : "a68", "a69", "a70", "a71"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a68, 0\n\tv_accvgpr_write_b32 a69, 0\n\tv_accvgpr_write_b32 a70, 0\n\tv_accvgpr_write_b32 a71, 0" ::: "a68", "a69", "a70", "a71"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a68, %0\n\tv_accvgpr_write_b32 a69, %1\n\tv_accvgpr_write_b32 a70, %2\n\tv_accvgpr_write_b32 a71, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a68", "a69", "a70", "a71"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a68\n\tv_accvgpr_read_b32 %1, a69\n\tv_accvgpr_read_b32 %2, a70\n\tv_accvgpr_read_b32 %3, a71" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<72> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[72:75], %0, %1, a[72:75]" :: "v"(b), "v"(a) : "a72", "a73", "a74", "a75"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[72:75], %0, %1, a[72:75]" :: "v"(b), "v"(a) : "a72", "a73", "a74", "a75"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a72, 0\n\tv_accvgpr_write_b32 a73, 0\n\tv_accvgpr_write_b32 a74, 0\n\tv_accvgpr_write_b32 a75, 0" ::: "a72", "a73", "a74", "a75"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a72, %0\n\tv_accvgpr_write_b32 a73, %1\n\tv_accvgpr_write_b32 a74, %2\n\tv_accvgpr_write_b32 a75, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a72", "a73", "a74", "a75"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a72\n\tv_accvgpr_read_b32 %1, a73\n\tv_accvgpr_read_b32 %2, a74\n\tv_accvgpr_read_b32 %3, a75" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<76> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[76:79], %0, %1, a[76:79]" :: "v"(b), "v"(a) : "a76", "a77", "a78", "a79"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[76:79], %0, %1, a[76:79]" :: "v"(b), "v"(a) : "a76", "a77", "a78", "a79"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a76, 0\n\tv_accvgpr_write_b32 a77, 0\n\tv_accvgpr_write_b32 a78, 0\n\tv_accvgpr_write_b32 a79, 0" ::: "a76", "a77", "a78", "a79"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a76, %0\n\tv_accvgpr_write_b32 a77, %1\n\tv_accvgpr_write_b32 a78, %2\n\tv_accvgpr_write_b32 a79, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a76", "a77", "a78", "a79"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a76\n\tv_accvgpr_read_b32 %1, a77\n\tv_accvgpr_read_b32 %2, a78\n\tv_accvgpr_read_b32 %3, a79" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<80> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[80:83], %0, %1, a[80:83]" :: "v"(b), "v"(a) : "a80", "a81", "a82", "a83"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[80:83], %0, %1, a[80:83]" :: "v"(b), "v"(a) : "a80", "a81", "a82", "a83"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a80, 0\n\tv_accvgpr_write_b32 a81, 0\n\tv_accvgpr_write_b32 a82, 0\n\tv_accvgpr_write_b32 a83, 0" ::: "a80", "a81", "a82", "a83"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a80, %0\n\tv_accvgpr_write_b32 a81, %1\n\tv_accvgpr_write_b32 a82, %2\n\tv_accvgpr_write_b32 a83, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a80", "a81", "a82", "a83"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a80\n\tv_accvgpr_read_b32 %1, a81\n\tv_accvgpr_read_b32 %2, a82\n\tv_accvgpr_read_b32 %3, a83" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<84> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[84:87], %0, %1, a[84:87]" :: "v"(b), "v"(a) : "a84", "a85", "a86", "a87"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[84:87], %0, %1, a[84:87]" :: "v"(b), "v"(a) : "a84", "a85", "a86", "a87"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a84, 0\n\tv_accvgpr_write_b32 a85, 0\n\tv_accvgpr_write_b32 a86, 0\n\tv_accvgpr_write_b32 a87, 0" ::: "a84", "a85", "a86", "a87"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a84, %0\n\tv_accvgpr_write_b32 a85, %1\n\tv_accvgpr_write_b32 a86, %2\n\tv_accvgpr_write_b32 a87, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a84", "a85", "a86", "a87"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a84\n\tv_accvgpr_read_b32 %1, a85\n\tv_accvgpr_read_b32 %2, a86\n\tv_accvgpr_read_b32 %3, a87" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<88> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[88:91], %0, %1, a[88:91]" :: "v"(b), "v"(a) : "a88", "a89", "a90", "a91"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[88:91], %0, %1, a[88:91]" :: "v"(b), "v"(a) : "a88", "a89", "a90", "a91"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a88, 0\n\tv_accvgpr_write_b32 a89, 0\n\tv_accvgpr_write_b32 a90, 0\n\tv_accvgpr_write_b32 a91, 0" ::: "a88", "a89", "a90", "a91"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a88, %0\n\tv_accvgpr_write_b32 a89, %1\n\tv_accvgpr_write_b32 a90, %2\n\tv_accvgpr_write_b32 a91, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a88", "a89", "a90", "a91"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a88\n\tv_accvgpr_read_b32 %1, a89\n\tv_accvgpr_read_b32 %2, a90\n\tv_accvgpr_read_b32 %3, a91" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<92> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[92:95], %0, %1, a[92:95]" :: "v"(b), "v"(a) : "a92", "a93", "a94", "a95"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[92:95], %0, %1, a[92:95]" :: "v"(b), "v"(a) : "a92", "a93", "a94", "a95"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a92, 0\n\tv_accvgpr_write_b32 a93, 0\n\tv_accvgpr_write_b32 a94, 0\n\tv_accvgpr_write_b32 a95, 0" ::: "a92", "a93", "a94", "a95"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a92, %0\n\tv_accvgpr_write_b32 a93, %1\n\tv_accvgpr_write_b32 a94, %2\n\tv_accvgpr_write_b32 a95, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a92", "a93", "a94", "a95"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a92\n\tv_accvgpr_read_b32 %1, a93\n\tv_accvgpr_read_b32 %2, a94\n\tv_accvgpr_read_b32 %3, a95" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<96> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[96:99], %0, %1, a[96:99]" :: "v"(b), "v"(a) : "a96", "a97", "a98", "a99"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[96:99], %0, %1, a[96:99]" :: "v"(b), "v"(a) : "a96", "a97", "a98", "a99"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a96, 0\n\tv_accvgpr_write_b32 a97, 0\n\tv_accvgpr_write_b32 a98, 0\n\tv_accvgpr_write_b32 a99, 0" ::: "a96", "a97", "a98", "a99"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a96, %0\n\tv_accvgpr_write_b32 a97, %1\n\tv_accvgpr_write_b32 a98, %2\n\tv_accvgpr_write_b32 a99, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a96", "a97", "a98", "a99"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a96\n\tv_accvgpr_read_b32 %1, a97\n\tv_accvgpr_read_b32 %2, a98\n\tv_accvgpr_read_b32 %3, a99" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<100> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[100:103], %0, %1, a[100:103]" :: "v"(b), "v"(a) : "a100", "a101", "a102", "a103"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[100:103], %0, %1, a[100:103]" :: "v"(b), "v"(a) : "a100", "a101", "a102", "a103"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a100, 0\n\tv_accvgpr_write_b32 a101, 0\n\tv_accvgpr_write_b32 a102, 0\n\tv_accvgpr_write_b32 a103, 0" ::: "a100", "a101", "a102", "a103"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a100, %0\n\tv_accvgpr_write_b32 a101, %1\n\tv_accvgpr_write_b32 a102, %2\n\tv_accvgpr_write_b32 a103, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a100", "a101", "a102", "a103"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a100\n\tv_accvgpr_read_b32 %1, a101\n\tv_accvgpr_read_b32 %2, a102\n\tv_accvgpr_read_b32 %3, a103" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<104> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[104:107], %0, %1, a[104:107]" :: "v"(b), "v"(a) : "a104", "a105", "a106", "a107"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[104:107], %0, %1, a[104:107]" :: "v"(b), "v"(a) : "a104", "a105", "a106", "a107"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a104, 0\n\tv_accvgpr_write_b32 a105, 0\n\tv_accvgpr_write_b32 a106, 0\n\tv_accvgpr_write_b32 a107, 0" ::: "a104", "a105", "a106", "a107"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a104, %0\n\tv_accvgpr_write_b32 a105, %1\n\tv_accvgpr_write_b32 a106, %2\n\tv_accvgpr_write_b32 a107, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a104", "a105", "a106", "a107"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a104\n\tv_accvgpr_read_b32 %1, a105\n\tv_accvgpr_read_b32 %2, a106\n\tv_accvgpr_read_b32 %3, a107" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<108> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[108:111], %0, %1, a[108:111]" :: "v"(b), "v"(a) : "a108", "a109", "a110", "a111"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[108:111], %0, %1, a[108:111]" :: "v"(b), "v"(a) : "a108", "a109", "a110", "a111"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a108, 0\n\tv_accvgpr_write_b32 a109, 0\n\tv_accvgpr_write_b32 a110, 0\n\tv_accvgpr_write_b32 a111, 0" ::: "a108", "a109", "a110", "a111"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a108, %0\n\tv_accvgpr_write_b32 a109, %1\n\tv_accvgpr_write_b32 a110, %2\n\tv_accvgpr_write_b32 a111, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a108", "a109", "a110", "a111"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a108\n\tv_accvgpr_read_b32 %1, a109\n\tv_accvgpr_read_b32 %2, a110\n\tv_accvgpr_read_b32 %3, a111" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<112> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[112:115], %0, %1, a[112:115]" :: "v"(b), "v"(a) : "a112", "a113", "a114", "a115"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[112:115], %0, %1, a[112:115]" :: "v"(b), "v"(a) : "a112", "a113", "a114", "a115"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a112, 0\n\tv_accvgpr_write_b32 a113, 0\n\tv_accvgpr_write_b32 a114, 0\n\tv_accvgpr_write_b32 a115, 0" ::: "a112", "a113", "a114", "a115"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a112, %0\n\tv_accvgpr_write_b32 a113, %1\n\tv_accvgpr_write_b32 a114, %2\n\tv_accvgpr_write_b32 a115, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a112", "a113", "a114", "a115"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a112\n\tv_accvgpr_read_b32 %1, a113\n\tv_accvgpr_read_b32 %2, a114\n\tv_accvgpr_read_b32 %3, a115" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<116> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[116:119], %0, %1, a[116:119]" :: "v"(b), "v"(a) : "a116", "a117", "a118", "a119"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[116:119], %0, %1, a[116:119]" :: "v"(b), "v"(a) : "a116", "a117", "a118", "a119"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a116, 0\n\tv_accvgpr_write_b32 a117, 0\n\tv_accvgpr_write_b32 a118, 0\n\tv_accvgpr_write_b32 a119, 0" ::: "a116", "a117", "a118", "a119"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a116, %0\n\tv_accvgpr_write_b32 a117, %1\n\tv_accvgpr_write_b32 a118, %2\n\tv_accvgpr_write_b32 a119, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a116", "a117", "a118", "a119"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a116\n\tv_accvgpr_read_b32 %1, a117\n\tv_accvgpr_read_b32 %2, a118\n\tv_accvgpr_read_b32 %3, a119" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<120> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[120:123], %0, %1, a[120:123]" :: "v"(b), "v"(a) : "a120", "a121", "a122", "a123"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[120:123], %0, %1, a[120:123]" :: "v"(b), "v"(a) : "a120", "a121", "a122", "a123"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a120, 0\n\tv_accvgpr_write_b32 a121, 0\n\tv_accvgpr_write_b32 a122, 0\n\tv_accvgpr_write_b32 a123, 0" ::: "a120", "a121", "a122", "a123"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a120, %0\n\tv_accvgpr_write_b32 a121, %1\n\tv_accvgpr_write_b32 a122, %2\n\tv_accvgpr_write_b32 a123, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a120", "a121", "a122", "a123"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a120\n\tv_accvgpr_read_b32 %1, a121\n\tv_accvgpr_read_b32 %2, a122\n\tv_accvgpr_read_b32 %3, a123" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<124> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[124:127], %0, %1, a[124:127]" :: "v"(b), "v"(a) : "a124", "a125", "a126", "a127"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[124:127], %0, %1, a[124:127]" :: "v"(b), "v"(a) : "a124", "a125", "a126", "a127"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a124, 0\n\tv_accvgpr_write_b32 a125, 0\n\tv_accvgpr_write_b32 a126, 0\n\tv_accvgpr_write_b32 a127, 0" ::: "a124", "a125", "a126", "a127"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a124, %0\n\tv_accvgpr_write_b32 a125, %1\n\tv_accvgpr_write_b32 a126, %2\n\tv_accvgpr_write_b32 a127, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a124", "a125", "a126", "a127"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a124\n\tv_accvgpr_read_b32 %1, a125\n\tv_accvgpr_read_b32 %2, a126\n\tv_accvgpr_read_b32 %3, a127" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<128> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[128:131], %0, %1, a[128:131]" :: "v"(b), "v"(a) : "a128", "a129", "a130", "a131"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[128:131], %0, %1, a[128:131]" :: "v"(b), "v"(a) : "a128", "a129", "a130", "a131"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a128, 0\n\tv_accvgpr_write_b32 a129, 0\n\tv_accvgpr_write_b32 a130, 0\n\tv_accvgpr_write_b32 a131, 0" ::: "a128", "a129", "a130", "a131"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a128, %0\n\tv_accvgpr_write_b32 a129, %1\n\tv_accvgpr_write_b32 a130, %2\n\tv_accvgpr_write_b32 a131, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a128", "a129", "a130", "a131"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a128\n\tv_accvgpr_read_b32 %1, a129\n\tv_accvgpr_read_b32 %2, a130\n\tv_accvgpr_read_b32 %3, a131" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<132> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[132:135], %0, %1, a[132:135]" :: "v"(b), "v"(a) : "a132", "a133", "a134", "a135"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[132:135], %0, %1, a[132:135]" :: "v"(b), "v"(a) : "a132", "a133", "a134", "a135"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a132, 0\n\tv_accvgpr_write_b32 a133, 0\n\tv_accvgpr_write_b32 a134, 0\n\tv_accvgpr_write_b32 a135, 0" ::: "a132", "a133", "a134", "a135"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a132, %0\n\tv_accvgpr_write_b32 a133, %1\n\tv_accvgpr_write_b32 a134, %2\n\tv_accvgpr_write_b32 a135, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a132", "a133", "a134", "a135"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a132\n\tv_accvgpr_read_b32 %1, a133\n\tv_accvgpr_read_b32 %2, a134\n\tv_accvgpr_read_b32 %3, a135" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<136> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[136:139], %0, %1, a[136:139]" :: "v"(b), "v"(a) : "a136", "a137", "a138", "a139"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[136:139], %0, %1, a[136:139]" :: "v"(b), "v"(a) : "a136", "a137", "a138", "a139"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a136, 0\n\tv_accvgpr_write_b32 a137, 0\n\tv_accvgpr_write_b32 a138, 0\n\tv_accvgpr_write_b32 a139, 0" ::: "a136", "a137", "a138", "a139"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a136, %0\n\tv_accvgpr_write_b32 a137, %1\n\tv_accvgpr_write_b32 a138, %2\n\tv_accvgpr_write_b32 a139, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a136", "a137", "a138", "a139"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a136\n\tv_accvgpr_read_b32 %1, a137\n\tv_accvgpr_read_b32 %2, a138\n\tv_accvgpr_read_b32 %3, a139" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<140> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[140:143], %0, %1, a[140:143]" :: "v"(b), "v"(a) : "a140", "a141", "a142", "a143"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[140:143], %0, %1, a[140:143]" :: "v"(b), "v"(a) : "a140", "a141", "a142", "a143"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a140, 0\n\tv_accvgpr_write_b32 a141, 0\n\tv_accvgpr_write_b32 a142, 0\n\tv_accvgpr_write_b32 a143, 0" ::: "a140", "a141", "a142", "a143"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a140, %0\n\tv_accvgpr_write_b32 a141, %1\n\tv_accvgpr_write_b32 a142, %2\n\tv_accvgpr_write_b32 a143, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a140", "a141", "a142", "a143"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a140\n\tv_accvgpr_read_b32 %1, a141\n\tv_accvgpr_read_b32 %2, a142\n\tv_accvgpr_read_b32 %3, a143" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<144> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[144:147], %0, %1, a[144:147]" :: "v"(b), "v"(a) : "a144", "a145", "a146", "a147"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[144:147], %0, %1, a[144:147]" :: "v"(b), "v"(a) : "a144", "a145", "a146", "a147"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a144, 0\n\tv_accvgpr_write_b32 a145, 0\n\tv_accvgpr_write_b32 a146, 0\n\tv_accvgpr_write_b32 a147, 0" ::: "a144", "a145", "a146", "a147"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a144, %0\n\tv_accvgpr_write_b32 a145, %1\n\tv_accvgpr_write_b32 a146, %2\n\tv_accvgpr_write_b32 a147, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a144", "a145", "a146", "a147"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a144\n\tv_accvgpr_read_b32 %1, a145\n\tv_accvgpr_read_b32 %2, a146\n\tv_accvgpr_read_b32 %3, a147" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<148> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[148:151], %0, %1, a[148:151]" :: "v"(b), "v"(a) : "a148", "a149", "a150", "a151"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[148:151], %0, %1, a[148:151]" :: "v"(b), "v"(a) : "a148", "a149", "a150", "a151"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a148, 0\n\tv_accvgpr_write_b32 a149, 0\n\tv_accvgpr_write_b32 a150, 0\n\tv_accvgpr_write_b32 a151, 0" ::: "a148", "a149", "a150", "a151"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a148, %0\n\tv_accvgpr_write_b32 a149, %1\n\tv_accvgpr_write_b32 a150, %2\n\tv_accvgpr_write_b32 a151, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a148", "a149", "a150", "a151"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a148\n\tv_accvgpr_read_b32 %1, a149\n\tv_accvgpr_read_b32 %2, a150\n\tv_accvgpr_read_b32 %3, a151" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<152> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[152:155], %0, %1, a[152:155]" :: "v"(b), "v"(a) : "a152", "a153", "a154", "a155"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[152:155], %0, %1, a[152:155]" :: "v"(b), "v"(a) : "a152", "a153", "a154", "a155"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a152, 0\n\tv_accvgpr_write_b32 a153, 0\n\tv_accvgpr_write_b32 a154, 0\n\tv_accvgpr_write_b32 a155, 0" ::: "a152", "a153", "a154", "a155"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a152, %0\n\tv_accvgpr_write_b32 a153, %1\n\tv_accvgpr_write_b32 a154, %2\n\tv_accvgpr_write_b32 a155, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a152", "a153", "a154", "a155"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a152\n\tv_accvgpr_read_b32 %1, a153\n\tv_accvgpr_read_b32 %2, a154\n\tv_accvgpr_read_b32 %3, a155" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<156> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[156:159], %0, %1, a[156:159]" :: "v"(b), "v"(a) : "a156", "a157", "a158", "a159"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[156:159], %0, %1, a[156:159]" :: "v"(b), "v"(a) : "a156", "a157", "a158", "a159"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a156, 0\n\tv_accvgpr_write_b32 a157, 0\n\tv_accvgpr_write_b32 a158, 0\n\tv_accvgpr_write_b32 a159, 0" ::: "a156", "a157", "a158", "a159"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a156, %0\n\tv_accvgpr_write_b32 a157, %1\n\tv_accvgpr_write_b32 a158, %2\n\tv_accvgpr_write_b32 a159, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a156", "a157", "a158", "a159"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a156\n\tv_accvgpr_read_b32 %1, a157\n\tv_accvgpr_read_b32 %2, a158\n\tv_accvgpr_read_b32 %3, a159" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<160> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[160:163], %0, %1, a[160:163]" :: "v"(b), "v"(a) : "a160", "a161", "a162", "a163"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[160:163], %0, %1, a[160:163]" :: "v"(b), "v"(a) : "a160", "a161", "a162", "a163"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a160, 0\n\tv_accvgpr_write_b32 a161, 0\n\tv_accvgpr_write_b32 a162, 0\n\tv_accvgpr_write_b32 a163, 0" ::: "a160", "a161", "a162", "a163"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a160, %0\n\tv_accvgpr_write_b32 a161, %1\n\tv_accvgpr_write_b32 a162, %2\n\tv_accvgpr_write_b32 a163, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a160", "a161", "a162", "a163"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a160\n\tv_accvgpr_read_b32 %1, a161\n\tv_accvgpr_read_b32 %2, a162\n\tv_accvgpr_read_b32 %3, a163" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<164> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[164:167], %0, %1, a[164:167]" :: "v"(b), "v"(a) : "a164", "a165", "a166", "a167"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[164:167], %0, %1, a[164:167]" :: "v"(b), "v"(a) : "a164", "a165", "a166", "a167"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a164, 0\n\tv_accvgpr_write_b32 a165, 0\n\tv_accvgpr_write_b32 a166, 0\n\tv_accvgpr_write_b32 a167, 0" ::: "a164", "a165", "a166", "a167"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a164, %0\n\tv_accvgpr_write_b32 a165, %1\n\tv_accvgpr_write_b32 a166, %2\n\tv_accvgpr_write_b32 a167, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a164", "a165", "a166", "a167"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a164\n\tv_accvgpr_read_b32 %1, a165\n\tv_accvgpr_read_b32 %2, a166\n\tv_accvgpr_read_b32 %3, a167" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<168> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[168:171], %0, %1, a[168:171]" :: "v"(b), "v"(a) : "a168", "a169", "a170", "a171"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[168:171], %0, %1, a[168:171]" :: "v"(b), "v"(a) : "a168", "a169", "a170", "a171"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a168, 0\n\tv_accvgpr_write_b32 a169, 0\n\tv_accvgpr_write_b32 a170, 0\n\tv_accvgpr_write_b32 a171, 0" ::: "a168", "a169", "a170", "a171"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a168, %0\n\tv_accvgpr_write_b32 a169, %1\n\tv_accvgpr_write_b32 a170, %2\n\tv_accvgpr_write_b32 a171, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a168", "a169", "a170", "a171"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a168\n\tv_accvgpr_read_b32 %1, a169\n\tv_accvgpr_read_b32 %2, a170\n\tv_accvgpr_read_b32 %3, a171" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<172> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[172:175], %0, %1, a[172:175]" :: "v"(b), "v"(a) : "a172", "a173", "a174", "a175"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[172:175], %0, %1, a[172:175]" :: "v"(b), "v"(a) : "a172", "a173", "a174", "a175"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a172, 0\n\tv_accvgpr_write_b32 a173, 0\n\tv_accvgpr_write_b32 a174, 0\n\tv_accvgpr_write_b32 a175, 0" ::: "a172", "a173", "a174", "a175"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a172, %0\n\tv_accvgpr_write_b32 a173, %1\n\tv_accvgpr_write_b32 a174, %2\n\tv_accvgpr_write_b32 a175, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a172", "a173", "a174", "a175"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a172\n\tv_accvgpr_read_b32 %1, a173\n\tv_accvgpr_read_b32 %2, a174\n\tv_accvgpr_read_b32 %3, a175" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<176> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[176:179], %0, %1, a[176:179]" :: "v"(b), "v"(a) : "a176", "a177", "a178", "a179"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[176:179], %0, %1, a[176:179]" :: "v"(b), "v"(a) : "a176", "a177", "a178", "a179"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a176, 0\n\tv_accvgpr_write_b32 a177, 0\n\tv_accvgpr_write_b32 a178, 0\n\tv_accvgpr_write_b32 a179, 0" ::: "a176", "a177", "a178", "a179"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a176, %0\n\tv_accvgpr_write_b32 a177, %1\n\tv_accvgpr_write_b32 a178, %2\n\tv_accvgpr_write_b32 a179, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a176", "a177", "a178", "a179"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a176\n\tv_accvgpr_read_b32 %1, a177\n\tv_accvgpr_read_b32 %2, a178\n\tv_accvgpr_read_b32 %3, a179" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<180> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[180:183], %0, %1, a[180:183]" :: "v"(b), "v"(a) : "a180", "a181", "a182", "a183"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[180:183], %0, %1, a[180:183]" :: "v"(b), "v"(a) : "a180", "a181", "a182", "a183"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a180, 0\n\tv_accvgpr_write_b32 a181, 0\n\tv_accvgpr_write_b32 a182, 0\n\tv_accvgpr_write_b32 a183, 0" ::: "a180", "a181", "a182", "a183"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a180, %0\n\tv_accvgpr_write_b32 a181, %1\n\tv_accvgpr_write_b32 a182, %2\n\tv_accvgpr_write_b32 a183, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a180", "a181", "a182", "a183"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a180\n\tv_accvgpr_read_b32 %1, a181\n\tv_accvgpr_read_b32 %2, a182\n\tv_accvgpr_read_b32 %3, a183" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<184> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[184:187], %0, %1, a[184:187]" :: "v"(b), "v"(a) : "a184", "a185", "a186", "a187"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[184:187], %0, %1, a[184:187]" :: "v"(b), "v"(a) : "a184", "a185", "a186", "a187"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a184, 0\n\tv_accvgpr_write_b32 a185, 0\n\tv_accvgpr_write_b32 a186, 0\n\tv_accvgpr_write_b32 a187, 0" ::: "a184", "a185", "a186", "a187"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a184, %0\n\tv_accvgpr_write_b32 a185, %1\n\tv_accvgpr_write_b32 a186, %2\n\tv_accvgpr_write_b32 a187, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a184", "a185", "a186", "a187"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a184\n\tv_accvgpr_read_b32 %1, a185\n\tv_accvgpr_read_b32 %2, a186\n\tv_accvgpr_read_b32 %3, a187" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<188> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[188:191], %0, %1, a[188:191]" :: "v"(b), "v"(a) : "a188", "a189", "a190", "a191"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[188:191], %0, %1, a[188:191]" :: "v"(b), "v"(a) : "a188", "a189", "a190", "a191"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a188, 0\n\tv_accvgpr_write_b32 a189, 0\n\tv_accvgpr_write_b32 a190, 0\n\tv_accvgpr_write_b32 a191, 0" ::: "a188", "a189", "a190", "a191"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a188, %0\n\tv_accvgpr_write_b32 a189, %1\n\tv_accvgpr_write_b32 a190, %2\n\tv_accvgpr_write_b32 a191, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a188", "a189", "a190", "a191"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a188\n\tv_accvgpr_read_b32 %1, a189\n\tv_accvgpr_read_b32 %2, a190\n\tv_accvgpr_read_b32 %3, a191" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<192> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[192:195], %0, %1, a[192:195]" :: "v"(b), "v"(a) : "a192", "a193", "a194", "a195"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[192:195], %0, %1, a[192:195]" :: "v"(b), "v"(a) : "a192", "a193", "a194", "a195"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a192, 0\n\tv_accvgpr_write_b32 a193, 0\n\tv_accvgpr_write_b32 a194, 0\n\tv_accvgpr_write_b32 a195, 0" ::: "a192", "a193", "a194", "a195"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a192, %0\n\tv_accvgpr_write_b32 a193, %1\n\tv_accvgpr_write_b32 a194, %2\n\tv_accvgpr_write_b32 a195, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a192", "a193", "a194", "a195"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a192\n\tv_accvgpr_read_b32 %1, a193\n\tv_accvgpr_read_b32 %2, a194\n\tv_accvgpr_read_b32 %3, a195" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<196> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[196:199], %0, %1, a[196:199]" :: "v"(b), "v"(a) : "a196", "a197", "a198", "a199"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[196:199], %0, %1, a[196:199]" :: "v"(b), "v"(a) : "a196", "a197", "a198", "a199"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a196, 0\n\tv_accvgpr_write_b32 a197, 0\n\tv_accvgpr_write_b32 a198, 0\n\tv_accvgpr_write_b32 a199, 0" ::: "a196", "a197", "a198", "a199"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a196, %0\n\tv_accvgpr_write_b32 a197, %1\n\tv_accvgpr_write_b32 a198, %2\n\tv_accvgpr_write_b32 a199, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a196", "a197", "a198", "a199"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a196\n\tv_accvgpr_read_b32 %1, a197\n\tv_accvgpr_read_b32 %2, a198\n\tv_accvgpr_read_b32 %3, a199" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<200> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[200:203], %0, %1, a[200:203]" :: "v"(b), "v"(a) : "a200", "a201", "a202", "a203"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[200:203], %0, %1, a[200:203]" :: "v"(b), "v"(a) : "a200", "a201", "a202", "a203"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a200, 0\n\tv_accvgpr_write_b32 a201, 0\n\tv_accvgpr_write_b32 a202, 0\n\tv_accvgpr_write_b32 a203, 0" ::: "a200", "a201", "a202", "a203"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a200, %0\n\tv_accvgpr_write_b32 a201, %1\n\tv_accvgpr_write_b32 a202, %2\n\tv_accvgpr_write_b32 a203, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a200", "a201", "a202", "a203"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a200\n\tv_accvgpr_read_b32 %1, a201\n\tv_accvgpr_read_b32 %2, a202\n\tv_accvgpr_read_b32 %3, a203" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<204> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[204:207], %0, %1, a[204:207]" :: "v"(b), "v"(a) : "a204", "a205", "a206", "a207"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[204:207], %0, %1, a[204:207]" :: "v"(b), "v"(a) : "a204", "a205", "a206", "a207"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a204, 0\n\tv_accvgpr_write_b32 a205, 0\n\tv_accvgpr_write_b32 a206, 0\n\tv_accvgpr_write_b32 a207, 0" ::: "a204", "a205", "a206", "a207"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a204, %0\n\tv_accvgpr_write_b32 a205, %1\n\tv_accvgpr_write_b32 a206, %2\n\tv_accvgpr_write_b32 a207, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a204", "a205", "a206", "a207"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a204\n\tv_accvgpr_read_b32 %1, a205\n\tv_accvgpr_read_b32 %2, a206\n\tv_accvgpr_read_b32 %3, a207" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<208> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[208:211], %0, %1, a[208:211]" :: "v"(b), "v"(a) : "a208", "a209", "a210", "a211"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[208:211], %0, %1, a[208:211]" :: "v"(b), "v"(a) : "a208", "a209", "a210", "a211"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a208, 0\n\tv_accvgpr_write_b32 a209, 0\n\tv_accvgpr_write_b32 a210, 0\n\tv_accvgpr_write_b32 a211, 0" ::: "a208", "a209", "a210", "a211"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a208, %0\n\tv_accvgpr_write_b32 a209, %1\n\tv_accvgpr_write_b32 a210, %2\n\tv_accvgpr_write_b32 a211, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a208", "a209", "a210", "a211"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a208\n\tv_accvgpr_read_b32 %1, a209\n\tv_accvgpr_read_b32 %2, a210\n\tv_accvgpr_read_b32 %3, a211" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<212> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[212:215], %0, %1, a[212:215]" :: "v"(b), "v"(a) : "a212", "a213", "a214", "a215"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[212:215], %0, %1, a[212:215]" :: "v"(b), "v"(a) : "a212", "a213", "a214", "a215"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a212, 0\n\tv_accvgpr_write_b32 a213, 0\n\tv_accvgpr_write_b32 a214, 0\n\tv_accvgpr_write_b32 a215, 0" ::: "a212", "a213", "a214", "a215"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a212, %0\n\tv_accvgpr_write_b32 a213, %1\n\tv_accvgpr_write_b32 a214, %2\n\tv_accvgpr_write_b32 a215, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a212", "a213", "a214", "a215"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a212\n\tv_accvgpr_read_b32 %1, a213\n\tv_accvgpr_read_b32 %2, a214\n\tv_accvgpr_read_b32 %3, a215" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<216> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[216:219], %0, %1, a[216:219]" :: "v"(b), "v"(a) : "a216", "a217", "a218", "a219"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[216:219], %0, %1, a[216:219]" :: "v"(b), "v"(a) : "a216", "a217", "a218", "a219"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a216, 0\n\tv_accvgpr_write_b32 a217, 0\n\tv_accvgpr_write_b32 a218, 0\n\tv_accvgpr_write_b32 a219, 0" ::: "a216", "a217", "a218", "a219"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a216, %0\n\tv_accvgpr_write_b32 a217, %1\n\tv_accvgpr_write_b32 a218, %2\n\tv_accvgpr_write_b32 a219, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a216", "a217", "a218", "a219"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a216\n\tv_accvgpr_read_b32 %1, a217\n\tv_accvgpr_read_b32 %2, a218\n\tv_accvgpr_read_b32 %3, a219" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<220> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[220:223], %0, %1, a[220:223]" :: "v"(b), "v"(a) : "a220", "a221", "a222", "a223"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[220:223], %0, %1, a[220:223]" :: "v"(b), "v"(a) : "a220", "a221", "a222", "a223"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a220, 0\n\tv_accvgpr_write_b32 a221, 0\n\tv_accvgpr_write_b32 a222, 0\n\tv_accvgpr_write_b32 a223, 0" ::: "a220", "a221", "a222", "a223"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a220, %0\n\tv_accvgpr_write_b32 a221, %1\n\tv_accvgpr_write_b32 a222, %2\n\tv_accvgpr_write_b32 a223, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a220", "a221", "a222", "a223"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a220\n\tv_accvgpr_read_b32 %1, a221\n\tv_accvgpr_read_b32 %2, a222\n\tv_accvgpr_read_b32 %3, a223" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<224> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[224:227], %0, %1, a[224:227]" :: "v"(b), "v"(a) : "a224", "a225", "a226", "a227"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[224:227], %0, %1, a[224:227]" :: "v"(b), "v"(a) : "a224", "a225", "a226", "a227"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a224, 0\n\tv_accvgpr_write_b32 a225, 0\n\tv_accvgpr_write_b32 a226, 0\n\tv_accvgpr_write_b32 a227, 0" ::: "a224", "a225", "a226", "a227"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a224, %0\n\tv_accvgpr_write_b32 a225, %1\n\tv_accvgpr_write_b32 a226, %2\n\tv_accvgpr_write_b32 a227, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a224", "a225", "a226", "a227"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a224\n\tv_accvgpr_read_b32 %1, a225\n\tv_accvgpr_read_b32 %2, a226\n\tv_accvgpr_read_b32 %3, a227" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<228> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[228:231], %0, %1, a[228:231]" :: "v"(b), "v"(a) : "a228", "a229", "a230", "a231"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[228:231], %0, %1, a[228:231]" :: "v"(b), "v"(a) : "a228", "a229", "a230", "a231"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a228, 0\n\tv_accvgpr_write_b32 a229, 0\n\tv_accvgpr_write_b32 a230, 0\n\tv_accvgpr_write_b32 a231, 0" ::: "a228", "a229", "a230", "a231"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a228, %0\n\tv_accvgpr_write_b32 a229, %1\n\tv_accvgpr_write_b32 a230, %2\n\tv_accvgpr_write_b32 a231, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a228", "a229", "a230", "a231"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a228\n\tv_accvgpr_read_b32 %1, a229\n\tv_accvgpr_read_b32 %2, a230\n\tv_accvgpr_read_b32 %3, a231" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<232> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[232:235], %0, %1, a[232:235]" :: "v"(b), "v"(a) : "a232", "a233", "a234", "a235"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[232:235], %0, %1, a[232:235]" :: "v"(b), "v"(a) : "a232", "a233", "a234", "a235"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a232, 0\n\tv_accvgpr_write_b32 a233, 0\n\tv_accvgpr_write_b32 a234, 0\n\tv_accvgpr_write_b32 a235, 0" ::: "a232", "a233", "a234", "a235"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a232, %0\n\tv_accvgpr_write_b32 a233, %1\n\tv_accvgpr_write_b32 a234, %2\n\tv_accvgpr_write_b32 a235, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a232", "a233", "a234", "a235"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a232\n\tv_accvgpr_read_b32 %1, a233\n\tv_accvgpr_read_b32 %2, a234\n\tv_accvgpr_read_b32 %3, a235" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<236> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[236:239], %0, %1, a[236:239]" :: "v"(b), "v"(a) : "a236", "a237", "a238", "a239"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[236:239], %0, %1, a[236:239]" :: "v"(b), "v"(a) : "a236", "a237", "a238", "a239"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a236, 0\n\tv_accvgpr_write_b32 a237, 0\n\tv_accvgpr_write_b32 a238, 0\n\tv_accvgpr_write_b32 a239, 0" ::: "a236", "a237", "a238", "a239"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a236, %0\n\tv_accvgpr_write_b32 a237, %1\n\tv_accvgpr_write_b32 a238, %2\n\tv_accvgpr_write_b32 a239, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a236", "a237", "a238", "a239"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a236\n\tv_accvgpr_read_b32 %1, a237\n\tv_accvgpr_read_b32 %2, a238\n\tv_accvgpr_read_b32 %3, a239" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<240> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[240:243], %0, %1, a[240:243]" :: "v"(b), "v"(a) : "a240", "a241", "a242", "a243"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[240:243], %0, %1, a[240:243]" :: "v"(b), "v"(a) : "a240", "a241", "a242", "a243"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a240, 0\n\tv_accvgpr_write_b32 a241, 0\n\tv_accvgpr_write_b32 a242, 0\n\tv_accvgpr_write_b32 a243, 0" ::: "a240", "a241", "a242", "a243"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a240, %0\n\tv_accvgpr_write_b32 a241, %1\n\tv_accvgpr_write_b32 a242, %2\n\tv_accvgpr_write_b32 a243, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a240", "a241", "a242", "a243"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a240\n\tv_accvgpr_read_b32 %1, a241\n\tv_accvgpr_read_b32 %2, a242\n\tv_accvgpr_read_b32 %3, a243" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<244> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[244:247], %0, %1, a[244:247]" :: "v"(b), "v"(a) : "a244", "a245", "a246", "a247"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[244:247], %0, %1, a[244:247]" :: "v"(b), "v"(a) : "a244", "a245", "a246", "a247"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a244, 0\n\tv_accvgpr_write_b32 a245, 0\n\tv_accvgpr_write_b32 a246, 0\n\tv_accvgpr_write_b32 a247, 0" ::: "a244", "a245", "a246", "a247"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a244, %0\n\tv_accvgpr_write_b32 a245, %1\n\tv_accvgpr_write_b32 a246, %2\n\tv_accvgpr_write_b32 a247, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a244", "a245", "a246", "a247"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a244\n\tv_accvgpr_read_b32 %1, a245\n\tv_accvgpr_read_b32 %2, a246\n\tv_accvgpr_read_b32 %3, a247" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<248> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[248:251], %0, %1, a[248:251]" :: "v"(b), "v"(a) : "a248", "a249", "a250", "a251"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[248:251], %0, %1, a[248:251]" :: "v"(b), "v"(a) : "a248", "a249", "a250", "a251"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a248, 0\n\tv_accvgpr_write_b32 a249, 0\n\tv_accvgpr_write_b32 a250, 0\n\tv_accvgpr_write_b32 a251, 0" ::: "a248", "a249", "a250", "a251"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a248, %0\n\tv_accvgpr_write_b32 a249, %1\n\tv_accvgpr_write_b32 a250, %2\n\tv_accvgpr_write_b32 a251, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a248", "a249", "a250", "a251"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a248\n\tv_accvgpr_read_b32 %1, a249\n\tv_accvgpr_read_b32 %2, a250\n\tv_accvgpr_read_b32 %3, a251" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
template <> struct acc<252> {
  TL_DEVICE static void mma(const halfx8& b, const halfx8& a) { asm volatile("v_mfma_f32_16x16x32_f16 a[252:255], %0, %1, a[252:255]" :: "v"(b), "v"(a) : "a252", "a253", "a254", "a255"); }
  TL_DEVICE static void mma(const bf16x8& b, const bf16x8& a) { asm volatile("v_mfma_f32_16x16x32_bf16 a[252:255], %0, %1, a[252:255]" :: "v"(b), "v"(a) : "a252", "a253", "a254", "a255"); }
  TL_DEVICE static void zero() { asm volatile("v_accvgpr_write_b32 a252, 0\n\tv_accvgpr_write_b32 a253, 0\n\tv_accvgpr_write_b32 a254, 0\n\tv_accvgpr_write_b32 a255, 0" ::: "a252", "a253", "a254", "a255"); }
  TL_DEVICE static void load(const floatx4& v) { asm volatile("v_accvgpr_write_b32 a252, %0\n\tv_accvgpr_write_b32 a253, %1\n\tv_accvgpr_write_b32 a254, %2\n\tv_accvgpr_write_b32 a255, %3" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]) : "a252", "a253", "a254", "a255"); }
  TL_DEVICE static floatx4 read() { float x0, x1, x2, x3; asm volatile("v_accvgpr_read_b32 %0, a252\n\tv_accvgpr_read_b32 %1, a253\n\tv_accvgpr_read_b32 %2, a254\n\tv_accvgpr_read_b32 %3, a255" : "=v"(x0), "=v"(x1), "=v"(x2), "=v"(x3)); return floatx4{x0, x1, x2, x3}; }
};
} }  // namespace tl::agpr
