// tl/mesh.h — device-initiated inter-GPU tile communication for T.comm on MI355X.
//
// The reference fork lowers T.comm.* to an opaque `tl.broadcast_` intrinsic that has no code
// generator (src/op/comm.cc:27-48).  Here a mesh "core" is one GPU of the node.  Every rank
// owns a symmetric workspace (fine-grained device memory — hipDeviceMallocFinegrained, coherent
// at system scope across GPUs — exported with hipIpcGetMemHandle and opened by every peer), so a
// workgroup stores its tile straight into a peer's HBM over xGMI — every GPU pair has its own
// link, so transfers are direct (no 2-D mesh routing).
//
// Workspace of one rank (F = align256(nblocks * nops * nranks * 4)):
//   [0, F)        u32 flag [blk][op][src]   data from `src` is in my slot (or barrier arrival)
//   [F, 2F)       u32 ready[blk][op][dst]   `dst` consumed my previous tile, I may overwrite
//   [2F, ...)     slots    [blk][op][src][slot_bytes]
// A transfer src -> dst of one op instance, tag = (epoch << 12) | instance_count:
//   dst: ready@src[blk][op][dst] = tag
//   src: wait ready == tag; all threads store the tile into slot@dst[blk][op][src];
//        drain stores; workgroup barrier; system-scope release; flag@dst[blk][op][src] = tag
//   dst: wait flag == tag; system-scope acquire; workgroup barrier; read the slot.
// Waits are bounded by a wall-clock budget (s_memrealtime, 100 MHz): on timeout the rank
// records an error bit that the host checks, and continues — a broken peer never hangs the GPU.
#pragma once

#ifndef TL_MESH_TIMEOUT_TICKS
#define TL_MESH_TIMEOUT_TICKS 2000000000ull  // 20 s at 100 MHz
#endif

namespace tl {
namespace mesh {

struct Ctx {
  int rank, nrow, ncol;
  char* const* ws;  // [nranks] workspace base pointers (own + IPC-mapped peers)
  unsigned epoch;
  unsigned* err;
  int nblocks, nops;
  long long slot_bytes;
};

TL_DEVICE Ctx make_ctx(int rank, int nrow, int ncol, long long ws, unsigned epoch, long long err, int nblocks,
                       int nops, long long slot_bytes) {
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

TL_DEVICE unsigned tag(const Ctx& c, unsigned cnt) { return (c.epoch << 12) | (cnt & 0xfffu); }

// ---- groups: 0 = row ("h"), 1 = column ("v"), 2 = whole mesh -------------------------------
TL_DEVICE int group_size(const Ctx& c, int dir) { return dir == 0 ? c.ncol : (dir == 1 ? c.nrow : c.nrow * c.ncol); }
TL_DEVICE int group_index(const Ctx& c, int dir, int core) {
  return dir == 0 ? core % c.ncol : (dir == 1 ? core / c.ncol : core);
}
TL_DEVICE int group_member(const Ctx& c, int dir, int anchor, int k) {
  if (dir == 0) return (anchor / c.ncol) * c.ncol + k;
  if (dir == 1) return k * c.ncol + anchor % c.ncol;
  return k;
}
TL_DEVICE int group_member_rot(const Ctx& c, int dir, int anchor, int k) {
  int g = group_size(c, dir);
  return group_member(c, dir, anchor, (group_index(c, dir, anchor) + k) % g);
}
TL_DEVICE bool in_group(const Ctx& c, int dir, int anchor, int core) {
  if (dir == 0) return core / c.ncol == anchor / c.ncol;
  if (dir == 1) return core % c.ncol == anchor % c.ncol;
  return true;
}

// ---- workspace addressing --------------------------------------------------------------------
TL_DEVICE long long flags_bytes(const Ctx& c) {
  return (((long long)c.nblocks * c.nops * c.nrow * c.ncol * 4) + 255) & ~255ll;
}
TL_DEVICE unsigned* flag_at(const Ctx& c, int owner, int blk, int op, int src) {
  return reinterpret_cast<unsigned*>(c.ws[owner]) + ((long long)blk * c.nops + op) * (c.nrow * c.ncol) + src;
}
TL_DEVICE unsigned* ready_at(const Ctx& c, int owner, int blk, int op, int dst) {
  unsigned* base = reinterpret_cast<unsigned*>(c.ws[owner] + flags_bytes(c));
  return base + ((long long)blk * c.nops + op) * (c.nrow * c.ncol) + dst;
}
TL_DEVICE char* slot(const Ctx& c, int owner, int blk, int op, int src) {
  return c.ws[owner] + 2 * flags_bytes(c) +
         (((long long)blk * c.nops + op) * (c.nrow * c.ncol) + src) * c.slot_bytes;
}

// ---- primitives -----------------------------------------------------------------------------
TL_DEVICE void store_flag(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
TL_DEVICE unsigned load_flag(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// one lane spins until *p == v (exact) or (int)(*p - v) >= 0 (at_least); bounded by wall clock.
// A set error word (an earlier wait of this rank timed out and was not raised yet) ends every
// later wait at once, so a dead peer costs one budget, not one per wait.
TL_DEVICE void spin(const Ctx& c, unsigned* p, unsigned v, bool at_least, unsigned code) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    unsigned x = load_flag(p);
    if (at_least ? ((int)(x - v) >= 0) : (x == v)) return;
    if (__hip_atomic_load(c.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
        __builtin_amdgcn_s_memrealtime() - t0 > TL_MESH_TIMEOUT_TICKS) {
      atomicOr(c.err, code);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

TL_DEVICE void release_system() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back L2, wait for stores
}
TL_DEVICE void acquire_system() {
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system scope: invalidate L1/L2 for fresh reads
}

// receiver side: tell `src` that my slot for it may be (over)written
TL_DEVICE void post_ready(const Ctx& c, int blk, int op, int src, unsigned t) {
  if (threadIdx.x == 0) store_flag(ready_at(c, src, blk, op, c.rank), t);
}
// sender side: wait until `dst` consumed the previous tile
TL_DEVICE void wait_ready(const Ctx& c, int blk, int op, int dst, unsigned t) {
  if (threadIdx.x == 0) spin(c, ready_at(c, c.rank, blk, op, dst), t, false, 1u);
  __syncthreads();
}
// sender side: every thread stored its part of the tile into slot@dst — publish it
TL_DEVICE void publish(const Ctx& c, int blk, int op, int dst, unsigned t) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    release_system();
    store_flag(flag_at(c, dst, blk, op, c.rank), t);
  }
}
// receiver side: wait for the tile from `src`
TL_DEVICE void wait_data(const Ctx& c, int blk, int op, int src, unsigned t) {
  if (threadIdx.x == 0) {
    spin(c, flag_at(c, c.rank, blk, op, src), t, false, 2u);
    acquire_system();
  }
  __syncthreads();
}
// barrier among cores: announce my arrival to `peer`, then wait for everyone's
TL_DEVICE void barrier_arrive() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) release_system();
}
TL_DEVICE void barrier_post(const Ctx& c, int blk, int op, int peer, unsigned t) {
  if (threadIdx.x == 0) store_flag(flag_at(c, peer, blk, op, c.rank), t);
}
TL_DEVICE void barrier_wait(const Ctx& c, int blk, int op, int peer, unsigned t) {
  if (threadIdx.x == 0) {
    spin(c, flag_at(c, c.rank, blk, op, peer), t, true, 4u);
    acquire_system();
  }
  __syncthreads();
}
TL_DEVICE void fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, ""); }

}  // namespace mesh
}  // namespace tl
