// tl/reduce.h — wave64 cross-lane reductions and shuffles.
//
// Reference: src/tl_templates/hip/reduce.h (AllReduce with xor shuffles below 64 lanes and
// LDS above).  gfx950 specifics: xor-32 uses v_permlane32_swap and xor-16 v_permlane16_swap
// (VALU, no LDS traffic); smaller strides use DPP-backed __shfl_xor (ds_bpermute fallback).
#pragma once

namespace tl {

struct SumOp { template <typename T> TL_DEVICE T operator()(T a, T b) const { return a + b; } };
struct MaxOp { template <typename T> TL_DEVICE T operator()(T a, T b) const { return max_(a, b); } };
struct MinOp { template <typename T> TL_DEVICE T operator()(T a, T b) const { return min_(a, b); } };
struct BitAndOp { template <typename T> TL_DEVICE T operator()(T a, T b) const { return a & b; } };
struct BitOrOp { template <typename T> TL_DEVICE T operator()(T a, T b) const { return a | b; } };
struct BitXorOp { template <typename T> TL_DEVICE T operator()(T a, T b) const { return a ^ b; } };

template <typename T> TL_DEVICE uint32_t as_u32(T v) {
  static_assert(sizeof(T) <= 4, "32-bit shuffle");
  uint32_t u = 0;
  __builtin_memcpy(&u, &v, sizeof(T));
  return u;
}
template <typename T> TL_DEVICE T from_u32(uint32_t u) {
  T v;
  __builtin_memcpy(&v, &u, sizeof(T));
  return v;
}

TL_DEVICE bool __lane_id_lt32() { return (threadIdx.x & 32) == 0; }

// value of lane (lane ^ MASK)
template <int MASK, typename T> TL_DEVICE T shfl_xor_c(T v) {
  if constexpr (sizeof(T) == 8) {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
    lo = as_u32(shfl_xor_c<MASK>(lo));
    hi = as_u32(shfl_xor_c<MASK>(hi));
    u = ((uint64_t)hi << 32) | lo;
    T r;
    __builtin_memcpy(&r, &u, 8);
    return r;
  } else {
    const uint32_t u = as_u32(v);
    if constexpr (MASK == 32) {
      auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
      return from_u32<T>(__lane_id_lt32() ? r[1] : r[0]);
    } else if constexpr (MASK == 16) {
      auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
      return from_u32<T>((threadIdx.x & 16) == 0 ? r[1] : r[0]);
    } else {
      return from_u32<T>((uint32_t)__shfl_xor((int)u, MASK, 64));
    }
  }
}

template <typename T> TL_DEVICE T shfl_xor(T v, int mask, int width = 64) {
  if constexpr (sizeof(T) < 4) {
    return from_u32<T>((uint32_t)__shfl_xor((int)as_u32(v), mask, width));
  } else if constexpr (sizeof(T) == 4) {
    return from_u32<T>((uint32_t)__shfl_xor((int)as_u32(v), mask, width));
  } else {
    return __shfl_xor(v, mask, width);
  }
}
template <typename T> TL_DEVICE T shfl_down(T v, int d, int width = 64) {
  return from_u32<T>((uint32_t)__shfl_down((int)as_u32(v), d, width));
}
template <typename T> TL_DEVICE T shfl_up(T v, int d, int width = 64) {
  return from_u32<T>((uint32_t)__shfl_up((int)as_u32(v), d, width));
}
template <typename T> TL_DEVICE T shfl(T v, int src, int width = 64) {
  return from_u32<T>((uint32_t)__shfl((int)as_u32(v), src, width));
}

// all-reduce over the lane bits selected by MASKBITS (a set of xor strides, each a power of 2)
// xor-32 / xor-16 step of a commutative reduction: one v_permlane{32,16}_swap leaves {own, partner}
// in its two results (which is which depends on the lane's half), and op(r0, r1) is the same
// either way, so no per-lane select is needed.
template <int MASK, typename Op, typename T> TL_DEVICE T swap_step(Op op, T v) {
  if constexpr (sizeof(T) == 4) {
    const uint32_t u = as_u32(v);
    auto r = MASK == 32 ? __builtin_amdgcn_permlane32_swap(u, u, false, false)
                        : __builtin_amdgcn_permlane16_swap(u, u, false, false);
    return op(from_u32<T>(r[0]), from_u32<T>(r[1]));
  } else {
    return op(v, shfl_xor_c<MASK>(v));
  }
}

template <typename Op, int MASKBITS, typename T> TL_DEVICE T lane_allreduce(T v) {
  Op op;
  if constexpr ((MASKBITS & 32) != 0) v = swap_step<32>(op, v);
  if constexpr ((MASKBITS & 16) != 0) v = swap_step<16>(op, v);
  if constexpr ((MASKBITS & 8) != 0) v = op(v, shfl_xor_c<8>(v));
  if constexpr ((MASKBITS & 4) != 0) v = op(v, shfl_xor_c<4>(v));
  if constexpr ((MASKBITS & 2) != 0) v = op(v, shfl_xor_c<2>(v));
  if constexpr ((MASKBITS & 1) != 0) v = op(v, shfl_xor_c<1>(v));
  return v;
}

template <typename Op, typename T> TL_DEVICE T wave_allreduce(T v) { return lane_allreduce<Op, 63>(v); }
template <typename T> TL_DEVICE T wave_reduce_sum(T v) { return wave_allreduce<SumOp>(v); }
template <typename T> TL_DEVICE T wave_reduce_max(T v) { return wave_allreduce<MaxOp>(v); }
template <typename T> TL_DEVICE T wave_reduce_min(T v) { return wave_allreduce<MinOp>(v); }
template <typename T> TL_DEVICE T wave_reduce_bitand(T v) { return wave_allreduce<BitAndOp>(v); }
template <typename T> TL_DEVICE T wave_reduce_bitor(T v) { return wave_allreduce<BitOrOp>(v); }
template <typename T> TL_DEVICE T wave_reduce_bitxor(T v) { return wave_allreduce<BitXorOp>(v); }

}  // namespace tl
