// tl/math.h — scalar math used by lowered kernels.
//
// Precise variants call OCML (__ocml_*_f32) directly: clang's __builtin_tanhf & co. become LLVM
// intrinsics that the AMDGPU backend cannot always lower ("no libcall available for ftanh").
// The "fast" variants map to the gfx950 transcendental unit (v_exp_f32 computes 2^x, v_log_f32
// log2, v_rcp_f32, v_rsq_f32).
// Reference: src/target/intrin_rule_hip.cc:134-171 (HIPMath / HIPFastMath dispatch).
#pragma once

namespace tl {

#define TL_F32(x) static_cast<float>(x)

template <typename T> TL_DEVICE T exp(T x) { return (T)__ocml_exp_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T exp2(T x) { return (T)__ocml_exp2_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T exp10(T x) { return (T)__ocml_exp10_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T log(T x) { return (T)__ocml_log_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T log2(T x) { return (T)__ocml_log2_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T log10(T x) { return (T)__ocml_log10_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T log1p(T x) { return (T)__ocml_log1p_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T expm1(T x) { return (T)__ocml_expm1_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T sqrt(T x) { return (T)__builtin_sqrtf(TL_F32(x)); }
template <typename T> TL_DEVICE T rsqrt(T x) { return (T)(1.0f / __builtin_sqrtf(TL_F32(x))); }
template <typename T> TL_DEVICE T rcp(T x) { return (T)(1.0f / TL_F32(x)); }
template <typename T> TL_DEVICE T sin(T x) { return (T)__ocml_sin_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T cos(T x) { return (T)__ocml_cos_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T tan(T x) { return (T)__ocml_tan_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T asin(T x) { return (T)__ocml_asin_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T acos(T x) { return (T)__ocml_acos_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T atan(T x) { return (T)__ocml_atan_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T sinh(T x) { return (T)__ocml_sinh_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T cosh(T x) { return (T)__ocml_cosh_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T tanh(T x) { return (T)__ocml_tanh_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T erf(T x) { return (T)__ocml_erf_f32(TL_F32(x)); }
template <typename T> TL_DEVICE T floor(T x) { return (T)__builtin_floorf(TL_F32(x)); }
template <typename T> TL_DEVICE T ceil(T x) { return (T)__builtin_ceilf(TL_F32(x)); }
template <typename T> TL_DEVICE T trunc(T x) { return (T)__builtin_truncf(TL_F32(x)); }
template <typename T> TL_DEVICE T round(T x) { return (T)__builtin_roundf(TL_F32(x)); }
template <typename T> TL_DEVICE T nearbyint(T x) { return (T)__builtin_rintf(TL_F32(x)); }
template <typename T> TL_DEVICE T sigmoid(T x) { return (T)(1.0f / (1.0f + __builtin_expf(-TL_F32(x)))); }
template <typename T> TL_DEVICE T abs(T x) { return x < (T)0 ? (T)(-x) : x; }
TL_DEVICE float abs(float x) { return __builtin_fabsf(x); }
template <typename T, typename U> TL_DEVICE T pow(T x, U y) { return (T)__builtin_powf(TL_F32(x), TL_F32(y)); }
template <typename T, typename U> TL_DEVICE T fmod(T x, U y) { return (T)__builtin_fmodf(TL_F32(x), TL_F32(y)); }
template <typename T, typename U> TL_DEVICE T atan2(T y, U x) { return (T)__builtin_atan2f(TL_F32(y), TL_F32(x)); }
template <typename T> TL_DEVICE T fma(T a, T b, T c) { return (T)__builtin_fmaf(TL_F32(a), TL_F32(b), TL_F32(c)); }
template <typename T> TL_DEVICE bool isnan(T x) { return __builtin_isnan(TL_F32(x)); }
template <typename T> TL_DEVICE bool isinf(T x) { return __builtin_isinf(TL_F32(x)); }
template <typename T> TL_DEVICE bool isfinite(T x) { return __builtin_isfinite(TL_F32(x)); }

// hardware transcendental unit (fast math)
TL_DEVICE float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
TL_DEVICE float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
TL_DEVICE float fast_exp10(float x) { return __builtin_amdgcn_exp2f(x * 3.321928094887362f); }
TL_DEVICE float fast_log2(float x) { return __builtin_amdgcn_logf(x); }
TL_DEVICE float fast_log(float x) { return __builtin_amdgcn_logf(x) * 0.6931471805599453f; }
TL_DEVICE float fast_log10(float x) { return __builtin_amdgcn_logf(x) * 0.30102999566398120f; }
TL_DEVICE float fast_sin(float x) { return __builtin_amdgcn_sinf(x * 0.15915494309189535f); }
TL_DEVICE float fast_cos(float x) { return __builtin_amdgcn_cosf(x * 0.15915494309189535f); }
TL_DEVICE float fast_tan(float x) { return fast_sin(x) / fast_cos(x); }
template <typename T> TL_DEVICE T fast_exp(T x) { return (T)fast_exp(TL_F32(x)); }
template <typename T> TL_DEVICE T fast_exp2(T x) { return (T)fast_exp2(TL_F32(x)); }
template <typename T> TL_DEVICE T fast_log(T x) { return (T)fast_log(TL_F32(x)); }
template <typename T> TL_DEVICE T fast_log2(T x) { return (T)fast_log2(TL_F32(x)); }

#undef TL_F32

}  // namespace tl
