// tl/common.h — core types and helpers for gfx950 (CDNA4) kernels emitted by tilelang.
//
// Counterpart of the reference's src/tl_templates/hip/common.h, rewritten for gfx950:
// no ck_tile / rocwmma dependency, native _Float16 / __bf16 arithmetic, OCP fp8, wave64
// helpers, explicit LDS-DMA / waitcnt / barrier primitives used by the pipeline lowering.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define TL_DEVICE __device__ __forceinline__
#define TL_HOST_DEVICE __host__ __device__ __forceinline__

typedef _Float16 half_t;
typedef __bf16 bfloat16_t;

namespace tl {

// ---------------------------------------------------------------------------
// vector types
// ---------------------------------------------------------------------------
template <typename T, int N> struct vec_t {
  typedef T type __attribute__((ext_vector_type(N)));
};
template <typename T, int N> using vec = typename vec_t<T, N>::type;

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx2 __attribute__((ext_vector_type(2)));
typedef half_t halfx8 __attribute__((ext_vector_type(8)));
typedef half_t halfx4 __attribute__((ext_vector_type(4)));
typedef bfloat16_t bf16x8 __attribute__((ext_vector_type(8)));
typedef bfloat16_t bf16x4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef int intx4 __attribute__((ext_vector_type(4)));
typedef int intx16 __attribute__((ext_vector_type(16)));
typedef int intx8 __attribute__((ext_vector_type(8)));
typedef int intx2 __attribute__((ext_vector_type(2)));
typedef unsigned uintx4 __attribute__((ext_vector_type(4)));
typedef unsigned uintx2 __attribute__((ext_vector_type(2)));

// raw byte vectors used for vectorised copies (N bytes)
template <int BYTES> struct bytes_t;
template <> struct bytes_t<1> { typedef uint8_t type; };
template <> struct bytes_t<2> { typedef uint16_t type; };
template <> struct bytes_t<4> { typedef uint32_t type; };
template <> struct bytes_t<8> { typedef uintx2 type; };
template <> struct bytes_t<16> { typedef uintx4 type; };

template <int BYTES> TL_DEVICE void copy_bytes(void* dst, const void* src) {
  typedef typename bytes_t<BYTES>::type V;
  *reinterpret_cast<V*>(dst) = *reinterpret_cast<const V*>(src);
}

// pack N scalars into a vector and store them (dst must be N*sizeof(T) aligned)
template <typename T, int N> struct packed { T v[N]; };

template <typename T, int N> TL_DEVICE void store_vec(T* dst, const T (&vals)[N]) {
  constexpr int B = N * (int)sizeof(T);
  static_assert(B == 1 || B == 2 || B == 4 || B == 8 || B == 16, "vector store width");
  typedef typename bytes_t<B>::type V;
  V v;
  __builtin_memcpy(&v, vals, B);
  *reinterpret_cast<V*>(dst) = v;
}

// non-temporal variants (global_load / global_store ... nt): streamed-once data
template <typename T, int N> TL_DEVICE void store_vec_nt(T* dst, const T (&vals)[N]) {
  constexpr int B = N * (int)sizeof(T);
  static_assert(B == 1 || B == 2 || B == 4 || B == 8 || B == 16, "vector store width");
  typedef typename bytes_t<B>::type V;
  V v;
  __builtin_memcpy(&v, vals, B);
  __builtin_nontemporal_store(v, reinterpret_cast<V*>(dst));
}

template <typename T, int N> TL_DEVICE void load_vec_nt(T (&vals)[N], const T* src) {
  constexpr int B = N * (int)sizeof(T);
  typedef typename bytes_t<B>::type V;
  V v = __builtin_nontemporal_load(reinterpret_cast<const V*>(src));
  __builtin_memcpy(vals, &v, B);
}

template <typename T, int N> TL_DEVICE void load_vec(T (&vals)[N], const T* src) {
  constexpr int B = N * (int)sizeof(T);
  typedef typename bytes_t<B>::type V;
  V v = *reinterpret_cast<const V*>(src);
  __builtin_memcpy(vals, &v, B);
}

// ---------------------------------------------------------------------------
// thread / wave identity (wave64)
// ---------------------------------------------------------------------------
TL_DEVICE int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
// wave-vote helpers (a __ballot mask): set lanes, and set lanes below this one
TL_DEVICE int popc64(unsigned long long m) { return __builtin_popcountll(m); }
TL_DEVICE int mbcnt64(unsigned long long m) {
  return __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
}
TL_DEVICE int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// ---------------------------------------------------------------------------
// synchronisation
// ---------------------------------------------------------------------------
// Full barrier that also drains outstanding memory ops (what __syncthreads() does).
TL_DEVICE void sync_threads() { __syncthreads(); }

// Barrier that does NOT wait for outstanding vector-memory ops: LDS-DMA (global_load_lds)
// issued before it stays in flight (guide: "Pipelining across barriers").  LDS reads issued
// before it are retired (lgkmcnt(0)) so the barrier also orders LDS WAR hazards.
TL_DEVICE void barrier_raw() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Wave-level barrier (reference T.sync_warp): the 64 lanes of a wave issue in lockstep, so this
// only has to order memory (LDS / global) among the wave's lanes and stop the compiler from
// moving accesses across it.
TL_DEVICE void sync_warp() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Grid-wide barrier (reference T.sync_grid / sync_global).  Needs every workgroup of the grid
// resident at once: the launcher uses hipModuleLaunchCooperativeKernel for kernels that call it,
// which refuses grids larger than the device can hold.  Counter barrier with agent-scope
// release/acquire (MI355X guide, Guideline 16: per-XCD L2s are not coherent): lane 0 of every
// workgroup publishes with a release fence, arrives, and the last arriver resets the count and
// bumps the generation the others poll (relaxed loads + s_sleep).
// State is PER LAUNCH: `ws` = {count, generation, poisoned} in a zeroed workspace the launcher
// allocates for each launch on its stream (two concurrent launches of one kernel never share a
// barrier).  The wait is bounded by wall clock (s_memrealtime, 100 MHz): on timeout the block
// records GRID_SYNC (8) in the device error word `err` — raised by the host at its next check
// (tilelang/runtime/errors.py) — and poisons the barrier so every later barrier of this launch
// falls through at once (the kernel finishes instead of hanging the GPU).
#ifndef TL_GRID_SYNC_TIMEOUT_TICKS
#define TL_GRID_SYNC_TIMEOUT_TICKS 200000000ull  // 2 s
#endif
TL_DEVICE void sync_grid(long long ws_, long long err_) {
  unsigned* ws = reinterpret_cast<unsigned*>(ws_);
  int* err = reinterpret_cast<int*>(err_);
  __syncthreads();
  if (threadIdx.x == 0 && threadIdx.y == 0 && threadIdx.z == 0) {
    const unsigned nblocks = gridDim.x * gridDim.y * gridDim.z;
    const unsigned gen = __hip_atomic_load(&ws[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned arrived = __hip_atomic_fetch_add(&ws[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (arrived == nblocks) {
      __hip_atomic_store(&ws[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&ws[1], gen + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (__hip_atomic_load(&ws[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(&ws[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        if (__hip_atomic_load(&ws[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > TL_GRID_SYNC_TIMEOUT_TICKS) {
          __hip_atomic_fetch_or(err, 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(&ws[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}

// wave issue priority (0..3): raised around MFMA clusters so the co-resident wave's loads
// interleave with them (guide T5)
template <int N> TL_DEVICE void setprio() { __builtin_amdgcn_s_setprio(N); }

template <int N> TL_DEVICE void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int N> TL_DEVICE void wait_lgkmcnt() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}

TL_DEVICE void fence_workgroup() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }
TL_DEVICE void fence_agent() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent"); }
TL_DEVICE void fence_system() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, ""); }

// ---------------------------------------------------------------------------
// numeric helpers
// ---------------------------------------------------------------------------
template <typename T> TL_DEVICE T max_(T a, T b) { return a > b ? a : b; }
template <typename T> TL_DEVICE T min_(T a, T b) { return a < b ? a : b; }
TL_DEVICE float max_(float a, float b) { return __builtin_fmaxf(a, b); }
TL_DEVICE float min_(float a, float b) { return __builtin_fminf(a, b); }

template <typename T> TL_HOST_DEVICE T floordiv(T a, T b) {
  T q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}
template <typename T> TL_HOST_DEVICE T floormod(T a, T b) {
  T r = a % b;
  return (r != 0 && ((r < 0) != (b < 0))) ? r + b : r;
}

// float -> T conversion with round-to-nearest-even (hipcc emits v_cvt_pk_bf16_f32 for bf16)
template <typename To, typename From> TL_DEVICE To cvt(From x) { return static_cast<To>(x); }

TL_DEVICE float infinity() { return __builtin_huge_valf(); }

}  // namespace tl

#include "fp8.h"
#include "math.h"
