// tl/ep_cpu.h — the expert-parallel exchange protocol of tl/ep.h for the CPU plumbing target.
//
// Same symmetric-buffer layout (control words, EIDS, RECV[2], RET[2]), slot rule (a sender's
// running count per destination), parities and RFREE / TFREE reuse handshakes as the gfx950
// version; a rank is a process whose buffer is a /dev/shm mapping opened by every peer
// (parallel/mesh.py ProcessMesh.symmetric_buffer), so CPU process meshes of any size exercise the
// device protocol end to end (the bench's world-8 configuration included) without a GPU.  The
// CPU target runs a kernel's blocks one after another, so ops/ep.py launches these with ONE block:
// every function below is the whole grid's work.  Waits are bounded by wall clock and set the
// same error codes in `err` (1 slot not freed, 2 data not arrived, 16 routing overflow).
#pragma once
#include <chrono>
#include <sched.h>
#include <string.h>

#ifndef TL_EP_TIMEOUT_TICKS
#define TL_EP_TIMEOUT_TICKS 2000000000ull  // 20 s at 100 MHz (the device clock of tl/ep.h)
#endif

namespace tl {
namespace ep {

constexpr int MAXW = 32;
constexpr int CNT = 0, DFLAG = 2 * MAXW, RFLAG = 4 * MAXW, RFREE = 6 * MAXW, TFREE = 8 * MAXW;
constexpr long long CTRL_BYTES = 4096;

struct Layout {
  int W, cap;
  long long row_bytes;
  long long eids_off() const { return CTRL_BYTES; }
  long long recv_off() const { return (CTRL_BYTES + 2ll * W * cap * 4 + 4095) & ~4095ll; }
  long long ret_off() const { return recv_off() + 2ll * W * cap * row_bytes; }
};

inline unsigned* ctrl(char* base) { return reinterpret_cast<unsigned*>(base); }
inline void st_sys(unsigned* p, unsigned v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline unsigned ld_sys(unsigned* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline bool failed(int* err) { return __atomic_load_n(err, __ATOMIC_RELAXED) != 0; }

inline void spin(unsigned* p, unsigned v, bool at_least, int* err, int code) {
  const auto t0 = std::chrono::steady_clock::now();
  const double budget = (double)TL_EP_TIMEOUT_TICKS / 1e8;
  for (unsigned it = 0;; ++it) {
    const unsigned x = ld_sys(p);
    if (at_least ? ((int)(x - v) >= 0) : (x == v)) return;
    if (failed(err)) {
      __atomic_fetch_or(err, code, __ATOMIC_SEQ_CST);
      return;
    }
    if ((it & 255) == 255 &&
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > budget) {
      __atomic_fetch_or(err, code, __ATOMIC_SEQ_CST);
      return;
    }
    sched_yield();
  }
}

template <int W>
inline void dispatch(const void* x_, const int* ids, int* ret_index, long long ws_tab, int me, int epoch,
                     long long err_, int P, int topk, int n_loc, int cap, long long row_bytes) {
  static_assert(W <= MAXW, "EP group too large");
  const char* x = reinterpret_cast<const char*>(x_);
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const Layout L{W, cap, row_bytes};
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  if (e > 1u)  // my combine of step e-1 is done: peers may refill RET[(e-1)&1][me]
    for (int d = 0; d < W; ++d) st_sys(ctrl(ws[d]) + TFREE + ((e - 1u) & 1u) * MAXW + me, e - 1u);
  if (e > 2u)  // the destinations consumed what I sent them two steps ago into parity p
    for (int d = 0; d < W; ++d) spin(own + RFREE + p * MAXW + d, e - 2u, true, err, 1);
  int cnt[W];
  for (int d = 0; d < W; ++d) cnt[d] = 0;
  for (int j = 0; j < P; ++j) {
    const int d = ids[j] / n_loc;
    const int slot = (d >= 0 && d < W) ? cnt[d]++ : cap;
    if (d < 0 || d >= W || slot >= cap) {
      ret_index[j] = 0;
      __atomic_fetch_or(err, 16, __ATOMIC_SEQ_CST);
      continue;
    }
    ret_index[j] = d * cap + slot;
    memcpy(ws[d] + L.recv_off() + (((long long)p * W + me) * cap + slot) * row_bytes,
           x + (long long)(j / topk) * row_bytes, (size_t)row_bytes);
    reinterpret_cast<int*>(ws[d] + L.eids_off())[((long long)p * W + me) * cap + slot] = ids[j] - d * n_loc;
  }
  for (int d = 0; d < W; ++d) st_sys(ctrl(ws[d]) + CNT + p * MAXW + me, (unsigned)(cnt[d] < cap ? cnt[d] : cap));
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  for (int d = 0; d < W; ++d) st_sys(ctrl(ws[d]) + DFLAG + p * MAXW + me, e);
}

template <int W>
inline void recv_wait(int* ids_out, int* cnt_out, long long ws_tab, int me, int epoch, long long err_, int cap,
                      long long row_bytes) {
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const Layout L{W, cap, row_bytes};
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  for (int s = 0; s < W; ++s) spin(own + DFLAG + p * MAXW + s, e, false, err, 2);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  const int* eids = reinterpret_cast<const int*>(ws[me] + L.eids_off()) + (long long)p * W * cap;
  for (int s = 0; s < W; ++s) {
    const int c = (int)ld_sys(own + CNT + p * MAXW + s);
    cnt_out[s] = c;
    for (int k = 0; k < cap; ++k) ids_out[(long long)s * cap + k] = k < c ? eids[(long long)s * cap + k] : -1;
  }
}

template <int W>
inline void ret(const void* y_, const int* ydest, const int* cnt, long long ws_tab, int me, int epoch, long long err_,
                int cap, long long row_bytes) {
  const char* y = reinterpret_cast<const char*>(y_);
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const Layout L{W, cap, row_bytes};
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  // the expert FFN of step e has read RECV[p]: senders may refill it at e+2
  for (int s = 0; s < W; ++s) st_sys(ctrl(ws[s]) + RFREE + p * MAXW + me, e);
  if (e > 2u)
    for (int s = 0; s < W; ++s) spin(own + TFREE + p * MAXW + s, e - 2u, true, err, 1);
  for (int s = 0; s < W; ++s) {
    char* dst = ws[s] + L.ret_off() + ((long long)p * W + me) * cap * row_bytes;
    for (int i = 0; i < cnt[s]; ++i)
      memcpy(dst + (long long)i * row_bytes, y + (long long)ydest[s * cap + i] * row_bytes, (size_t)row_bytes);
  }
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  for (int s = 0; s < W; ++s) st_sys(ctrl(ws[s]) + RFLAG + p * MAXW + me, e);
}

template <int W>
inline void ret_wait(long long ws_tab, int me, int epoch, long long err_) {
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  for (int d = 0; d < W; ++d) spin(own + RFLAG + p * MAXW + d, e, false, err, 2);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
}

}  // namespace ep
}  // namespace tl
