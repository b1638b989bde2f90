// tl/atomic.h — global / LDS atomics for gfx950.
//
// Counterpart of src/tl_templates/cuda/atomic.h (the reference's HIP path only has a scalar
// AtomicAdd in hip/common.h).  gfx950 executes float atomics at the memory side
// (global_atomic_add_f32, global_atomic_pk_add_{bf16,f16}); agent scope is the default.
#pragma once

namespace tl {

template <typename T, typename V> TL_DEVICE T atomic_add(T* addr, V val) {
  return atomicAdd(addr, static_cast<T>(val));
}
TL_DEVICE half_t atomic_add(half_t* addr, float val) {
  // no scalar f16 atomic add on gfx950: CAS loop on the containing dword
  uintptr_t a = reinterpret_cast<uintptr_t>(addr);
  uint32_t* base = reinterpret_cast<uint32_t*>(a & ~uintptr_t(3));
  const int shift = (a & 2) ? 16 : 0;
  uint32_t old = *base, assumed;
  do {
    assumed = old;
    uint16_t h = (uint16_t)(assumed >> shift);
    half_t hv = __builtin_bit_cast(half_t, h);
    half_t nv = (half_t)((float)hv + val);
    uint32_t nu = (assumed & ~(0xffffu << shift)) | ((uint32_t)__builtin_bit_cast(uint16_t, nv) << shift);
    old = atomicCAS(base, assumed, nu);
  } while (old != assumed);
  return __builtin_bit_cast(half_t, (uint16_t)(old >> shift));
}
TL_DEVICE bfloat16_t atomic_add(bfloat16_t* addr, float val) {
  uintptr_t a = reinterpret_cast<uintptr_t>(addr);
  uint32_t* base = reinterpret_cast<uint32_t*>(a & ~uintptr_t(3));
  const int shift = (a & 2) ? 16 : 0;
  uint32_t old = *base, assumed;
  do {
    assumed = old;
    uint16_t h = (uint16_t)(assumed >> shift);
    bfloat16_t hv = __builtin_bit_cast(bfloat16_t, h);
    bfloat16_t nv = (bfloat16_t)((float)hv + val);
    uint32_t nu = (assumed & ~(0xffffu << shift)) | ((uint32_t)__builtin_bit_cast(uint16_t, nv) << shift);
    old = atomicCAS(base, assumed, nu);
  } while (old != assumed);
  return __builtin_bit_cast(bfloat16_t, (uint16_t)(old >> shift));
}

template <typename T, typename V> TL_DEVICE T atomic_max(T* addr, V val) {
  return atomicMax(addr, static_cast<T>(val));
}
template <typename T, typename V> TL_DEVICE T atomic_min(T* addr, V val) {
  return atomicMin(addr, static_cast<T>(val));
}
TL_DEVICE float atomic_max(float* addr, float val) {
  // sign-aware integer trick: monotone mapping of floats onto ints
  if (val >= 0.0f) return __int_as_float(atomicMax(reinterpret_cast<int*>(addr), __float_as_int(val)));
  return __uint_as_float(atomicMin(reinterpret_cast<unsigned*>(addr), __float_as_uint(val)));
}
TL_DEVICE float atomic_min(float* addr, float val) {
  if (val >= 0.0f) return __int_as_float(atomicMin(reinterpret_cast<int*>(addr), __float_as_int(val)));
  return __uint_as_float(atomicMax(reinterpret_cast<unsigned*>(addr), __float_as_uint(val)));
}

template <typename T> TL_DEVICE T atomic_load(const T* addr) {
  return __hip_atomic_load(addr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T, typename V> TL_DEVICE void atomic_store(T* addr, V val) {
  __hip_atomic_store(addr, static_cast<T>(val), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace tl
