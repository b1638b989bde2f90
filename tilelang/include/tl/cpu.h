// tl/cpu.h — prelude for kernels compiled for the CPU plumbing target (host clang++).
//
// Counterpart of the reference's src/tl_templates/cpp/{common,gemm}.h (which vendors a 5.6k
// line half.hpp); host clang provides _Float16 and __bf16 natively.
#pragma once
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <cmath>
#include <type_traits>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

typedef _Float16 half_t;
typedef __bf16 bfloat16_t;

// OCP fp8 on the host: E exponent bits, M mantissa bits, FN = "finite" (no inf, NaN=S.1111.111).
// Round-to-nearest-even; overflow -> NaN (fn) / inf (e5m2), as torch's float8 casts.
template <int E, int M, bool FN> struct fp8_host_t {
  uint8_t v;
  static constexpr int kBias = (1 << (E - 1)) - 1;
  fp8_host_t() = default;
  fp8_host_t(float f) { v = encode(f); }
  fp8_host_t(double f) { v = encode((float)f); }
  fp8_host_t(int f) { v = encode((float)f); }
  operator float() const { return decode(v); }
  static float max_finite() {
    return FN ? std::ldexp(1.0f + (float)((1 << M) - 2) / (1 << M), (1 << E) - 1 - kBias)
              : std::ldexp(1.0f + (float)((1 << M) - 1) / (1 << M), (1 << E) - 2 - kBias);
  }
  static uint8_t encode(float f) {
    const uint8_t sign = std::signbit(f) ? 0x80 : 0;
    const uint8_t nan = FN ? 0x7F : (uint8_t)((((1 << E) - 1) << M) | 1);
    const uint8_t inf = FN ? nan : (uint8_t)(((1 << E) - 1) << M);
    if (std::isnan(f)) return sign | nan;
    float a = std::fabs(f);
    if (std::isinf(a)) return sign | inf;
    int e;
    (void)std::frexp(a, &e);  // a = m * 2^e, m in [0.5, 1)
    e -= 1;                   // a = 1.x * 2^e
    uint32_t code;
    if (a == 0.0f) return sign;
    if (e < 1 - kBias) {  // subnormal
      float q = std::nearbyint(std::ldexp(a, kBias - 1 + M));
      code = (uint32_t)q;  // may round up into the smallest normal (code == 1 << M)
    } else {
      float q = std::nearbyint((std::ldexp(a, -e) - 1.0f) * (1 << M));
      if (q >= (float)(1 << M)) {
        q = 0;
        ++e;
      }
      code = ((uint32_t)(e + kBias) << M) | (uint32_t)q;
    }
    const uint32_t max_code = FN ? ((1u << (E + M)) - 2) : (((1u << E) - 2) << M | ((1u << M) - 1));
    if (code > max_code) return sign | inf;
    return sign | (uint8_t)code;
  }
  static float decode(uint8_t c) {
    const float s = (c & 0x80) ? -1.0f : 1.0f;
    const int ex = (c >> M) & ((1 << E) - 1);
    const int mt = c & ((1 << M) - 1);
    if (FN && ex == (1 << E) - 1 && mt == (1 << M) - 1) return NAN;
    if (!FN && ex == (1 << E) - 1) return mt ? NAN : s * INFINITY;
    if (ex == 0) return s * std::ldexp((float)mt, 1 - kBias - M);
    return s * std::ldexp(1.0f + (float)mt / (1 << M), ex - kBias);
  }
};
typedef fp8_host_t<4, 3, true> fp8_e4_t;
typedef fp8_host_t<5, 2, false> fp8_e5_t;

namespace tl {

template <typename T> inline T max_(T a, T b) { return a > b ? a : b; }
template <typename T> inline T min_(T a, T b) { return a < b ? a : b; }
template <typename T> inline T floordiv(T a, T b) {
  T q = a / b;
  return (a % b != 0 && ((a < 0) != (b < 0))) ? q - 1 : q;
}
template <typename T> inline T floormod(T a, T b) {
  T r = a % b;
  return (r != 0 && ((r < 0) != (b < 0))) ? r + b : r;
}

#define TL_CPU_UNARY(NAME, EXPR)                                         \
  template <typename T> inline T NAME(T x) {                             \
    float v = (float)x;                                                  \
    return (T)(EXPR);                                                    \
  }
TL_CPU_UNARY(exp, std::exp(v))
TL_CPU_UNARY(exp2, std::exp2(v))
TL_CPU_UNARY(exp10, std::pow(10.0f, v))
TL_CPU_UNARY(log, std::log(v))
TL_CPU_UNARY(log2, std::log2(v))
TL_CPU_UNARY(log10, std::log10(v))
TL_CPU_UNARY(log1p, std::log1p(v))
TL_CPU_UNARY(expm1, std::expm1(v))
TL_CPU_UNARY(sqrt, std::sqrt(v))
TL_CPU_UNARY(rsqrt, 1.0f / std::sqrt(v))
TL_CPU_UNARY(rcp, 1.0f / v)
TL_CPU_UNARY(sin, std::sin(v))
TL_CPU_UNARY(cos, std::cos(v))
TL_CPU_UNARY(tan, std::tan(v))
TL_CPU_UNARY(asin, std::asin(v))
TL_CPU_UNARY(acos, std::acos(v))
TL_CPU_UNARY(atan, std::atan(v))
TL_CPU_UNARY(sinh, std::sinh(v))
TL_CPU_UNARY(cosh, std::cosh(v))
TL_CPU_UNARY(tanh, std::tanh(v))
TL_CPU_UNARY(erf, std::erf(v))
TL_CPU_UNARY(floor, std::floor(v))
TL_CPU_UNARY(ceil, std::ceil(v))
TL_CPU_UNARY(trunc, std::trunc(v))
TL_CPU_UNARY(round, std::round(v))
TL_CPU_UNARY(nearbyint, std::nearbyint(v))
TL_CPU_UNARY(sigmoid, 1.0f / (1.0f + std::exp(-v)))
TL_CPU_UNARY(fast_exp, std::exp(v))
TL_CPU_UNARY(fast_exp2, std::exp2(v))
TL_CPU_UNARY(fast_log, std::log(v))
TL_CPU_UNARY(fast_log2, std::log2(v))
TL_CPU_UNARY(fast_sin, std::sin(v))
TL_CPU_UNARY(fast_cos, std::cos(v))
#undef TL_CPU_UNARY
template <typename T> inline T abs(T x) { return x < (T)0 ? (T)(-x) : x; }
template <typename T, typename U> inline T pow(T x, U y) { return (T)std::pow((float)x, (float)y); }
template <typename T, typename U> inline T fmod(T x, U y) { return (T)std::fmod((float)x, (float)y); }
template <typename T> inline T fma(T a, T b, T c) { return (T)std::fma((float)a, (float)b, (float)c); }
template <typename T> inline bool isnan(T x) { return std::isnan((float)x); }
template <typename T> inline bool isinf(T x) { return std::isinf((float)x); }

template <typename T, int N> inline void store_vec(T* dst, const T (&vals)[N]) { memcpy(dst, vals, sizeof(T) * N); }
template <typename T, int N> inline void load_vec(T (&vals)[N], const T* src) { memcpy(vals, src, sizeof(T) * N); }
template <int B> inline void copy_bytes(void* dst, const void* src) { memcpy(dst, src, B); }

inline void sync_threads() {}
// blocks run one after another on the CPU target: memory fences are compiler barriers only
inline void fence_workgroup() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
inline void fence_agent() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
inline void fence_system() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
inline void sync_warp() {}
// T.sync_grid on the CPU target: kernels that use it run every block as a host thread
// (codegen/hip.py) meeting at this generation-counting barrier.
struct GridBarrier {
  explicit GridBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m_);
    const long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }
  int n_, count_ = 0;
  long gen_ = 0;
  std::mutex m_;
  std::condition_variable cv_;
};
inline GridBarrier*& cur_grid_barrier() {
  static thread_local GridBarrier* b = nullptr;
  return b;
}
inline void sync_grid() {
  if (cur_grid_barrier()) cur_grid_barrier()->wait();
}
inline void print_val(const char* msg, double v) { printf("%s: %g\n", msg, v); fflush(stdout); }
inline void print_val(const char* msg, float v) { print_val(msg, (double)v); }
inline void print_val(const char* msg, half_t v) { print_val(msg, (double)(float)v); }
inline void print_val(const char* msg, bfloat16_t v) { print_val(msg, (double)(float)v); }
inline void print_val(const char* msg, long long v) { printf("%s: %lld\n", msg, v); fflush(stdout); }
inline void print_val(const char* msg, long v) { print_val(msg, (long long)v); }
inline void print_val(const char* msg, int v) { print_val(msg, (long long)v); }
inline void print_val(const char* msg, unsigned v) { print_val(msg, (long long)v); }
inline void print_val(const char* msg, bool v) { print_val(msg, (long long)v); }
template <typename T> inline void print_buffer(const char* msg, const char* name, const T* buf, int n) {
  for (int i = 0; i < n; ++i) printf("%s %s[%d] = %g\n", msg, name, i, (double)(float)buf[i]);
  fflush(stdout);
}
inline void barrier_raw() {}
template <int N> inline void wait_vmcnt() {}

struct SumOp {};
struct MaxOp {};
struct MinOp {};
struct BitAndOp {};
struct BitOrOp {};
struct BitXorOp {};
template <typename Op, int M, typename T> inline T lane_allreduce(T v) { return v; }
// (no wave_reduce_* here: user-level wave reductions / shuffles need 64 lanes, which the
// one-thread-per-block CPU target does not have -- codegen refuses them for target "cpu")

// Atomics: blocks of a kernel that uses T.sync_grid run as concurrent host threads, so these are
// real read-modify-writes (CAS on the containing word), with the requested memory order.
namespace atomic_detail {
template <typename T> struct word {
  typedef typename std::conditional<sizeof(T) == 2, uint16_t,
          typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type type;
};
template <int MO, typename T, typename F> inline T rmw(T* p, F f) {
  typedef typename word<T>::type W;
  W* wp = reinterpret_cast<W*>(p);
  W old = __atomic_load_n(wp, __ATOMIC_RELAXED);
  for (;;) {
    T cur;
    memcpy(&cur, &old, sizeof(T));
    T nv = f(cur);
    W nw;
    memcpy(&nw, &nv, sizeof(T));
    if (__atomic_compare_exchange_n(wp, &old, nw, false, MO == __ATOMIC_RELAXED ? __ATOMIC_RELAXED : __ATOMIC_SEQ_CST,
                                    __ATOMIC_RELAXED))
      return cur;
  }
}
}  // namespace atomic_detail
template <int MO = __ATOMIC_RELAXED, typename T, typename V> inline T atomic_add(T* p, V v) {
  return atomic_detail::rmw<MO>(p, [&](T c) { return (T)((double)c + (double)v); });
}
template <int MO = __ATOMIC_RELAXED, typename T, typename V> inline T atomic_max(T* p, V v) {
  return atomic_detail::rmw<MO>(p, [&](T c) { return (T)v > c ? (T)v : c; });
}
template <int MO = __ATOMIC_RELAXED, typename T, typename V> inline T atomic_min(T* p, V v) {
  return atomic_detail::rmw<MO>(p, [&](T c) { return (T)v < c ? (T)v : c; });
}
template <int MO = __ATOMIC_RELAXED, typename T, typename V0, typename V1> inline T atomic_addx2(T* p, V0 a, V1 b) {
  T r = atomic_add<MO>(p, a);
  atomic_add<MO>(p + 1, b);
  return r;
}
template <int MO = __ATOMIC_RELAXED, typename T, typename V0, typename V1, typename V2, typename V3>
inline T atomic_addx4(T* p, V0 a, V1 b, V2 c, V3 d) {
  T r = atomic_addx2<MO>(p, a, b);
  atomic_addx2<MO>(p + 2, c, d);
  return r;
}
template <int MO = __ATOMIC_SEQ_CST, typename T> inline T atomic_load(const T* p) {
  typedef typename atomic_detail::word<T>::type W;
  W w = __atomic_load_n(reinterpret_cast<const W*>(p), MO == __ATOMIC_RELEASE ? __ATOMIC_SEQ_CST : MO);
  T r;
  memcpy(&r, &w, sizeof(T));
  return r;
}
template <int MO = __ATOMIC_SEQ_CST, typename T, typename V> inline void atomic_store(T* p, V v) {
  typedef typename atomic_detail::word<T>::type W;
  T t = (T)v;
  W w;
  memcpy(&w, &t, sizeof(T));
  const bool acq = MO == __ATOMIC_ACQUIRE || MO == __ATOMIC_CONSUME || MO == __ATOMIC_ACQ_REL;
  __atomic_store_n(reinterpret_cast<W*>(p), w, acq ? __ATOMIC_SEQ_CST : MO);
}

// C[M,N] += op(A) * op(B); C is the thread-local fp32 accumulator (row-major M x N).
template <typename T, int M, int N, int K, int TA, int TB, int A_COLS, int B_COLS, typename TC>
inline void cpu_gemm(const T* A, const T* B, TC* C) {
  // integer operands (int8 MFMA semantics) accumulate exactly in integers
  typedef typename std::conditional<std::is_integral<TC>::value, long long, float>::type acc_t;
  for (int i = 0; i < M; ++i)
    for (int k = 0; k < K; ++k) {
      const acc_t a = TA ? (acc_t)(float)A[k * A_COLS + i] : (acc_t)(float)A[i * A_COLS + k];
      for (int j = 0; j < N; ++j) {
        const acc_t b = TB ? (acc_t)(float)B[j * B_COLS + k] : (acc_t)(float)B[k * B_COLS + j];
        C[i * N + j] = (TC)((acc_t)C[i * N + j] + a * b);
      }
    }
}

// OCP MX element decode (FMT: 0 e4m3, 1 e5m2, 2 e2m3 / 3 e3m2 packed 4 per 3 bytes as a
// little-endian bit stream (element k at bits 6k..6k+5), 4 e2m1 packed two per byte, low nibble first)
template <int FMT> inline float mx_elem(const uint8_t* row, int k) {
  if constexpr (FMT == 0) {
    fp8_e4_t v;
    v.v = row[k];
    return (float)v;
  } else if constexpr (FMT == 1) {
    fp8_e5_t v;
    v.v = row[k];
    return (float)v;
  } else if constexpr (FMT == 2 || FMT == 3) {
    const int bit = 6 * k;
    // the second byte only when the field straddles (the last field of a row ends on a byte)
    const unsigned w = (unsigned)row[bit >> 3] | ((bit & 7) > 2 ? (unsigned)row[(bit >> 3) + 1] << 8 : 0u);
    const unsigned c = (w >> (bit & 7)) & 63u;
    constexpr int MB = FMT == 2 ? 3 : 2, BIAS = FMT == 2 ? 1 : 3;
    const int e = (int)((c & 31u) >> MB), m = (int)(c & ((1u << MB) - 1));
    const float mag = e == 0 ? std::ldexp((float)m, 1 - BIAS - MB) : std::ldexp((float)((1 << MB) + m), e - BIAS - MB);
    return (c & 32u) ? -mag : mag;
  } else {
    static const float lut[8] = {0.0f, 0.5f, 1.0f, 1.5f, 2.0f, 3.0f, 4.0f, 6.0f};
    const uint8_t nib = (row[k >> 1] >> (4 * (k & 1))) & 15;
    return (nib & 8 ? -1.0f : 1.0f) * lut[nib & 7];
  }
}

inline float e8m0(uint8_t s) { return s == 255 ? NAN : std::ldexp(1.0f, (int)s - 127); }

// tl/gemv.h mxfp4_gemv on the CPU target: the block's BLOCK_N rows, serially
template <int M, int BLOCK_N, int THREADS, int RG = BLOCK_N>
inline void mxfp4_gemv(const bfloat16_t* X, const uint8_t* Bq, const uint8_t* S, bfloat16_t* Y, int N, int K, int n0,
                       float*) {
  for (int n = n0; n < n0 + BLOCK_N && n < N; ++n)
    for (int m = 0; m < M; ++m) {
      float acc = 0.0f;
      for (int kb = 0; kb < K / 32; ++kb) {
        float part = 0.0f;
        for (int k = kb * 32; k < kb * 32 + 32; ++k)
          part += mx_elem<4>(Bq + (long long)n * (K / 2), k) * (float)X[(long long)m * K + k];
        acc += part * e8m0(S[(long long)n * (K / 32) + kb]);
      }
      Y[(long long)m * N + n] = (bfloat16_t)acc;
    }
}

// C[M][N] += sum_k (A[m][k] * 2^(SA[m][k/32]-127)) * (B[n][k] * 2^(SB[n][k/32]-127))
// PS = 1: pre-shuffled scale tiles (tl::mx_ps_index, T.gemm_scaled(scale_layout="preshuffled"))
template <int R>
inline int cpu_mx_ps_index(int row, int kb) {
  const int f = row >> 4, kk = kb >> 2, g = kb & 3;
  return ((((kk * (R / 64) + (f >> 2)) * 4 + g) * 16 + (row & 15)) * 4) + (f & 3);
}

template <int FA, int FB, int M, int N, int K, int A_COLS, int B_COLS, int SA_STRIDE, int SB_STRIDE, int PS = 0>
inline void cpu_gemm_mx(const void* A_, const void* B_, const void* SA_, const void* SB_, float* C) {
  const uint8_t* A = (const uint8_t*)A_;
  const uint8_t* B = (const uint8_t*)B_;
  const uint8_t* SA = (const uint8_t*)SA_;
  const uint8_t* SB = (const uint8_t*)SB_;
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < N; ++j) {
      float acc = 0.0f;
      for (int kb = 0; kb < K / 32; ++kb) {
        float part = 0.0f;
        for (int k = kb * 32; k < kb * 32 + 32; ++k)
          part += mx_elem<FA>(A + i * A_COLS, k) * mx_elem<FB>(B + j * B_COLS, k);
        const int ia = PS ? cpu_mx_ps_index<M>(i, kb) : i * SA_STRIDE + kb;
        const int ib = PS ? cpu_mx_ps_index<N>(j, kb) : j * SB_STRIDE + kb;
        acc += part * e8m0(SA[ia]) * e8m0(SB[ib]);
      }
      C[i * N + j] += acc;
    }
}

// 2:4 sparse A (T.gemm_sp): A holds the kept values [M][K/2] ([K/2][M] when TA), E the 2-bit
// positions, 16-bit word c of row i covering original K [16c, 16c+16) (value v at bits 2v).
template <typename T, int M, int N, int K, bool TA, bool TB, int A_COLS, int E_COLS, int B_COLS>
inline void cpu_gemm_sp(const T* A, const int16_t* E, const T* B, float* C) {
  for (int i = 0; i < M; ++i)
    for (int kc = 0; kc < K / 2; ++kc) {
      const float a = TA ? (float)A[kc * A_COLS + i] : (float)A[i * A_COLS + kc];
      const unsigned word = (unsigned)(uint16_t)E[i * E_COLS + kc / 8];
      const int pos = (int)((word >> (2 * (kc % 8))) & 3u);
      const int k = 4 * (kc / 2) + pos;
      for (int j = 0; j < N; ++j) {
        const float b = TB ? (float)B[j * B_COLS + k] : (float)B[k * B_COLS + j];
        C[i * N + j] += a * b;
      }
    }
}

}  // namespace tl
#include "mesh_cpu.h"
#include "ep_cpu.h"
