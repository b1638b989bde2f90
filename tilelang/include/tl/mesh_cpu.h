// tl/mesh_cpu.h — the T.comm protocol of tl/mesh.h for the CPU plumbing target.
//
// Same workspace layout, tags and handshakes as the gfx950 version; a "core" is a host thread
// (virtual mesh) or a process whose workspace is a shared /dev/shm mapping (process mesh), so
// the device protocol is exercised end to end without a GPU.  One CPU "thread" runs a block,
// hence no workgroup barriers.
#pragma once
#include <chrono>
#include <sched.h>

#ifndef TL_MESH_TIMEOUT_SEC
#define TL_MESH_TIMEOUT_SEC 20.0
#endif

namespace tl {
namespace mesh {

struct Ctx {
  int rank, nrow, ncol;
  char* const* ws;
  unsigned epoch;
  unsigned* err;
  int nblocks, nops;
  long long slot_bytes;
};

inline Ctx make_ctx(int rank, int nrow, int ncol, long long ws, unsigned epoch, long long err, int nblocks, int nops,
                    long long slot_bytes) {
  Ctx c;
  c.rank = rank;
  c.nrow = nrow;
  c.ncol = ncol;
  c.ws = reinterpret_cast<char* const*>(ws);
  c.epoch = epoch;
  c.err = reinterpret_cast<unsigned*>(err);
  c.nblocks = nblocks;
  c.nops = nops;
  c.slot_bytes = slot_bytes;
  return c;
}

inline unsigned tag(const Ctx& c, unsigned cnt) { return (c.epoch << 12) | (cnt & 0xfffu); }
inline int group_size(const Ctx& c, int dir) { return dir == 0 ? c.ncol : (dir == 1 ? c.nrow : c.nrow * c.ncol); }
inline int group_index(const Ctx& c, int dir, int core) {
  return dir == 0 ? core % c.ncol : (dir == 1 ? core / c.ncol : core);
}
inline int group_member(const Ctx& c, int dir, int anchor, int k) {
  if (dir == 0) return (anchor / c.ncol) * c.ncol + k;
  if (dir == 1) return k * c.ncol + anchor % c.ncol;
  return k;
}
inline int group_member_rot(const Ctx& c, int dir, int anchor, int k) {
  int g = group_size(c, dir);
  return group_member(c, dir, anchor, (group_index(c, dir, anchor) + k) % g);
}
inline bool in_group(const Ctx& c, int dir, int anchor, int core) {
  if (dir == 0) return core / c.ncol == anchor / c.ncol;
  if (dir == 1) return core % c.ncol == anchor % c.ncol;
  return true;
}
inline long long flags_bytes(const Ctx& c) {
  return (((long long)c.nblocks * c.nops * c.nrow * c.ncol * 4) + 255) & ~255ll;
}
inline unsigned* flag_at(const Ctx& c, int owner, int blk, int op, int src) {
  return reinterpret_cast<unsigned*>(c.ws[owner]) + ((long long)blk * c.nops + op) * (c.nrow * c.ncol) + src;
}
inline unsigned* ready_at(const Ctx& c, int owner, int blk, int op, int dst) {
  unsigned* base = reinterpret_cast<unsigned*>(c.ws[owner] + flags_bytes(c));
  return base + ((long long)blk * c.nops + op) * (c.nrow * c.ncol) + dst;
}
inline char* slot(const Ctx& c, int owner, int blk, int op, int src) {
  return c.ws[owner] + 2 * flags_bytes(c) +
         (((long long)blk * c.nops + op) * (c.nrow * c.ncol) + src) * c.slot_bytes;
}
inline void store_flag(unsigned* p, unsigned v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline void spin(const Ctx& c, unsigned* p, unsigned v, bool at_least, unsigned code) {
  auto t0 = std::chrono::steady_clock::now();
  for (unsigned it = 0;; ++it) {
    unsigned x = __atomic_load_n(p, __ATOMIC_ACQUIRE);
    if (at_least ? ((int)(x - v) >= 0) : (x == v)) return;
    if ((it & 255) == 255) {
      double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (dt > TL_MESH_TIMEOUT_SEC) {
        __atomic_fetch_or(c.err, code, __ATOMIC_SEQ_CST);
        return;
      }
    }
    sched_yield();
  }
}
inline void post_ready(const Ctx& c, int blk, int op, int src, unsigned t) {
  store_flag(ready_at(c, src, blk, op, c.rank), t);
}
inline void wait_ready(const Ctx& c, int blk, int op, int dst, unsigned t) {
  spin(c, ready_at(c, c.rank, blk, op, dst), t, false, 1u);
}
inline void publish(const Ctx& c, int blk, int op, int dst, unsigned t) {
  __atomic_thread_fence(__ATOMIC_RELEASE);
  store_flag(flag_at(c, dst, blk, op, c.rank), t);
}
inline void wait_data(const Ctx& c, int blk, int op, int src, unsigned t) {
  spin(c, flag_at(c, c.rank, blk, op, src), t, false, 2u);
}
inline void barrier_arrive() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }
inline void barrier_post(const Ctx& c, int blk, int op, int peer, unsigned t) {
  store_flag(flag_at(c, peer, blk, op, c.rank), t);
}
inline void barrier_wait(const Ctx& c, int blk, int op, int peer, unsigned t) {
  spin(c, flag_at(c, c.rank, blk, op, peer), t, true, 4u);
}
inline void fence() { __atomic_thread_fence(__ATOMIC_SEQ_CST); }

}  // namespace mesh
}  // namespace tl
