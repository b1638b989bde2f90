// tl/atomic.h — global / LDS atomics for gfx950.
//
// Counterpart of src/tl_templates/cuda/atomic.h (AtomicAdd / AtomicAddx2 / AtomicAddx4 / memory
// orders, :333-464); the reference's HIP path only has a scalar AtomicAdd in hip/common.h.
//
// gfx950 executes these at the memory side (L2 for global, the LDS unit for shared):
//   f32 add              global_atomic_add_f32 / ds_add_f32
//   f16 / bf16 pair add  global_atomic_pk_add_{f16,bf16} / ds_pk_add_{f16,bf16}
//   int add/max/min      global_atomic_{add,smax,smin,umax,umin}
// There is no scalar 16-bit float atomic: a single f16/bf16 element is a packed add on its
// aligned dword with -0.0 in the other half (-0.0 is the exact IEEE additive identity:
// x + -0.0 == x for every x, +0/-0 and NaN payloads included), one instruction, no CAS loop.
// f16 / bf16 max and min have no hardware op and are CAS loops on the containing dword.
//
// Memory orders: the template argument is a clang __ATOMIC_* constant (relaxed 0, consume 1,
// acquire 2, release 3, acq_rel 4, seq_cst 5 -- the reference's numbering in
// tilelang/language/atomic.py:11-18).  Scope is the agent (one GPU), as CUDA's device scope.
// Ops clang expresses directly (__hip_atomic_*) carry the order themselves; the packed builtins
// are relaxed, and release / acquire halves are fences around them (the AMDGPU memory model's
// own lowering: buffer_wbl2 before, buffer_inv after).
#pragma once

namespace tl {

typedef half_t half2_t __attribute__((ext_vector_type(2)));
typedef short short2_t __attribute__((ext_vector_type(2)));

namespace atomic_detail {

template <int MO> TL_DEVICE void fence_before() {
  if constexpr (MO == __ATOMIC_RELEASE || MO == __ATOMIC_ACQ_REL || MO == __ATOMIC_SEQ_CST)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}
template <int MO> TL_DEVICE void fence_after() {
  if constexpr (MO == __ATOMIC_ACQUIRE || MO == __ATOMIC_CONSUME || MO == __ATOMIC_ACQ_REL ||
                MO == __ATOMIC_SEQ_CST)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

template <typename T> constexpr bool is16f = __is_same(T, half_t) || __is_same(T, bfloat16_t);

// packed add of (lo, hi) into the dword at p (4-byte aligned); returns the previous pair
TL_DEVICE half2_t pk_add(half_t* p, half_t lo, half_t hi) {
  half2_t v = {lo, hi};
  return __builtin_amdgcn_flat_atomic_fadd_v2f16(reinterpret_cast<half2_t*>(p), v);
}
TL_DEVICE short2_t pk_add(bfloat16_t* p, bfloat16_t lo, bfloat16_t hi) {
  short2_t v = {__builtin_bit_cast(short, lo), __builtin_bit_cast(short, hi)};
  return __builtin_amdgcn_flat_atomic_fadd_v2bf16(reinterpret_cast<short2_t*>(p), v);
}
TL_DEVICE half_t lane_of(half2_t v, int i) { return i ? v.y : v.x; }
TL_DEVICE bfloat16_t lane_of(short2_t v, int i) { return __builtin_bit_cast(bfloat16_t, i ? v.y : v.x); }

// one 16-bit element: packed add on its aligned dword, -0.0 in the neighbour's half
template <typename T> TL_DEVICE T add16(T* addr, float val) {
  // pointer arithmetic (not an integer mask) keeps the global / LDS address space visible to
  // the compiler: global_atomic_pk_add / ds_pk_add instead of the flat form
  const int hi = (reinterpret_cast<uintptr_t>(addr) & 2) ? 1 : 0;
  T* base = addr - hi;
  const T v = static_cast<T>(val), nz = static_cast<T>(-0.0f);
  return lane_of(pk_add(base, hi ? nz : v, hi ? v : nz), hi);
}

// 16-bit max / min: CAS loop on the containing dword (no hardware op)
template <bool IsMax, typename T> TL_DEVICE T minmax16(T* addr, float val) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(addr);
  uint32_t* base = reinterpret_cast<uint32_t*>(a & ~uintptr_t(3));
  const int shift = (a & 2) ? 16 : 0;
  uint32_t old = __hip_atomic_load(base, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), assumed;
  do {
    assumed = old;
    const float cur = (float)__builtin_bit_cast(T, (uint16_t)(assumed >> shift));
    const bool take = IsMax ? (val > cur) : (val < cur);
    if (!take) break;
    const uint32_t nu = (assumed & ~(0xffffu << shift)) |
                        ((uint32_t)__builtin_bit_cast(uint16_t, static_cast<T>(val)) << shift);
    old = assumed;
    __hip_atomic_compare_exchange_strong(base, &old, nu, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
  } while (old != assumed);
  return __builtin_bit_cast(T, (uint16_t)(assumed >> shift));
}

// f32 max / min through the monotone int mapping of floats (sign-aware)
template <bool IsMax, int MO> TL_DEVICE float minmax32(float* addr, float val) {
  int* ip = reinterpret_cast<int*>(addr);
  unsigned* up = reinterpret_cast<unsigned*>(addr);
  if (val == 0.0f) val = 0.0f;  // -0.0 -> +0.0 (its int image INT_MIN would order below negatives)
  // val >= 0: floats order as signed ints against any stored value; val < 0: as unsigned ints
  // with the order reversed (larger magnitude = larger unsigned = smaller float)
  if (val >= 0.0f) {
    const int r = IsMax ? __hip_atomic_fetch_max(ip, __float_as_int(val), MO, __HIP_MEMORY_SCOPE_AGENT)
                        : __hip_atomic_fetch_min(ip, __float_as_int(val), MO, __HIP_MEMORY_SCOPE_AGENT);
    return __int_as_float(r);
  }
  const unsigned r = IsMax ? __hip_atomic_fetch_min(up, __float_as_uint(val), MO, __HIP_MEMORY_SCOPE_AGENT)
                           : __hip_atomic_fetch_max(up, __float_as_uint(val), MO, __HIP_MEMORY_SCOPE_AGENT);
  return __uint_as_float(r);
}

}  // namespace atomic_detail

// ---- scalar read-modify-write (returns the previous value) --------------------------------

template <int MO = __ATOMIC_RELAXED, typename T, typename V> TL_DEVICE T atomic_add(T* addr, V val) {
  if constexpr (atomic_detail::is16f<T>) {
    atomic_detail::fence_before<MO>();
    const T r = atomic_detail::add16(addr, (float)val);
    atomic_detail::fence_after<MO>();
    return r;
  } else {
    return __hip_atomic_fetch_add(addr, static_cast<T>(val), MO, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int MO = __ATOMIC_RELAXED, typename T, typename V> TL_DEVICE T atomic_max(T* addr, V val) {
  if constexpr (atomic_detail::is16f<T>) {
    atomic_detail::fence_before<MO>();
    const T r = atomic_detail::minmax16<true>(addr, (float)val);
    atomic_detail::fence_after<MO>();
    return r;
  } else if constexpr (__is_same(T, float)) {
    return atomic_detail::minmax32<true, MO>(addr, (float)val);
  } else {
    return __hip_atomic_fetch_max(addr, static_cast<T>(val), MO, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <int MO = __ATOMIC_RELAXED, typename T, typename V> TL_DEVICE T atomic_min(T* addr, V val) {
  if constexpr (atomic_detail::is16f<T>) {
    atomic_detail::fence_before<MO>();
    const T r = atomic_detail::minmax16<false>(addr, (float)val);
    atomic_detail::fence_after<MO>();
    return r;
  } else if constexpr (__is_same(T, float)) {
    return atomic_detail::minmax32<false, MO>(addr, (float)val);
  } else {
    return __hip_atomic_fetch_min(addr, static_cast<T>(val), MO, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- vector adds (AtomicAddx2 / x4): consecutive elements, first one naturally aligned -----
// f16 / bf16 pairs are one global_atomic_pk_add (ds_pk_add on LDS); f32 has no vector atomic
// on gfx950, so a pair / quad is 2 / 4 global_atomic_add_f32 (issued back to back).  The value
// returned is the previous value of the first element.

template <int MO = __ATOMIC_RELAXED, typename T, typename V0, typename V1>
TL_DEVICE T atomic_addx2(T* addr, V0 v0, V1 v1) {
  if constexpr (atomic_detail::is16f<T>) {
    atomic_detail::fence_before<MO>();
    const auto r = atomic_detail::pk_add(addr, static_cast<T>(v0), static_cast<T>(v1));
    atomic_detail::fence_after<MO>();
    return atomic_detail::lane_of(r, 0);
  } else {
    const T r = atomic_add<MO>(addr, v0);
    atomic_add<MO>(addr + 1, v1);
    return r;
  }
}

template <int MO = __ATOMIC_RELAXED, typename T, typename V0, typename V1, typename V2, typename V3>
TL_DEVICE T atomic_addx4(T* addr, V0 v0, V1 v1, V2 v2, V3 v3) {
  const T r = atomic_addx2<MO>(addr, v0, v1);
  atomic_addx2<MO>(addr + 2, v2, v3);
  return r;
}

// ---- loads / stores with an order ----------------------------------------------------------

template <int MO = __ATOMIC_SEQ_CST, typename T> TL_DEVICE T atomic_load(const T* addr) {
  if constexpr (sizeof(T) == 2) {
    const uint16_t r = __hip_atomic_load(reinterpret_cast<const uint16_t*>(addr), MO, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_bit_cast(T, r);
  } else {
    return __hip_atomic_load(addr, MO, __HIP_MEMORY_SCOPE_AGENT);
  }
}
template <int MO = __ATOMIC_SEQ_CST, typename T, typename V> TL_DEVICE void atomic_store(T* addr, V val) {
  if constexpr (sizeof(T) == 2) {
    __hip_atomic_store(reinterpret_cast<uint16_t*>(addr), __builtin_bit_cast(uint16_t, static_cast<T>(val)), MO,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_store(addr, static_cast<T>(val), MO, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace tl
