// tl/fp8.h — OCP fp8 (e4m3fn / e5m2) types for gfx950.
//
// The reference's AMD path uses MI300 "fnuz" encodings (src/tl_templates/hip/hip_fp8.h:5-10);
// gfx950 implements OCP e4m3fn/e5m2 in hardware (v_cvt_pk_fp8_f32, v_cvt_f32_fp8, and the
// fp8 MFMA / scaled MFMA operand formats), so these wrappers map 1:1 to those instructions.
#pragma once

namespace tl {

struct fp8_e4_t {
  uint8_t v;
  fp8_e4_t() = default;
  TL_DEVICE explicit fp8_e4_t(float f) {
    v = (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(f, f, 0, false) & 0xff);
  }
  TL_DEVICE operator float() const { return __builtin_amdgcn_cvt_f32_fp8((int)v, 0); }
};

struct fp8_e5_t {
  uint8_t v;
  fp8_e5_t() = default;
  TL_DEVICE explicit fp8_e5_t(float f) {
    v = (uint8_t)(__builtin_amdgcn_cvt_pk_bf8_f32(f, f, 0, false) & 0xff);
  }
  TL_DEVICE operator float() const { return __builtin_amdgcn_cvt_f32_bf8((int)v, 0); }
};

// pack 4 floats into 4 e4m3 bytes (one dword) with two v_cvt_pk_fp8_f32
TL_DEVICE uint32_t pack4_e4m3(float a, float b, float c, float d) {
  int r = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  r = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, r, true);
  return (uint32_t)r;
}

// e8m0 block scale (MX): 2^(e-127)
TL_DEVICE float e8m0_to_float(uint8_t e) { return __builtin_bit_cast(float, (uint32_t)e << 23); }

}  // namespace tl

typedef tl::fp8_e4_t fp8_e4_t;
typedef tl::fp8_e5_t fp8_e5_t;
