// tl/ep.h — expert-parallel token exchange over xGMI, driven entirely by the GPU.
//
// The reference's DeepSeek-V3.2 demo reaches its experts with host collectives
// (examples/deepseek_v32/inference/model.py:787-850: local experts + dist.all_reduce).  A
// host all-to-all-v needs the split sizes on the host — one device->host sync per MoE layer.
// Here every rank owns a symmetric buffer (fine-grained device memory, see "Memory model"
// below; exported with HIP IPC and opened by every peer) and the
// routed rows are stored straight into the destination GPU's buffer at a slot the SENDER
// computes (its own running count per destination), so no rank ever needs another rank's
// counts before moving data, and nothing waits on the host:
//
//   dispatch(e)   pair j of token t -> rank d = expert / n_loc, slot = rank of j among my pairs
//                 for d; row x[t] -> RECV[p][me][slot]@d, local expert id -> EIDS[p][me][slot]@d;
//                 last block: CNT[p][me]@d = count, DFLAG[p][me]@d = e        (p = e & 1)
//   recv_wait(e)  DFLAG[p][s] == e for all s; ids[s*cap + i] = EIDS[p][s][i] (i < CNT) else -1
//   (the expert FFN reads RECV[p] as a [W*cap, H] row table, skipping id -1)
//   ret(e)        row y of received pair (s, i) -> RET[p][me][i]@s; last block: RFLAG[p][me]@s = e
//   ret_wait(e)   RFLAG[p][d] == e for all d; pair j's result is RET[p] row d*cap + slot
//
// Buffer reuse: parity p alternates per step; before overwriting a peer's RECV[p] / RET[p] the
// writer waits for that peer's "consumed" word (RFREE / TFREE, stored into the writer's buffer
// by the consumer at its next kernel, which stream order places after the consuming kernel).
// All waits are bounded by wall clock (s_memrealtime, 100 MHz) and record a mesh error code in
// `err` (raised by the host: tilelang/runtime/errors.py) instead of hanging the GPU; once `err` is
// set every later wait returns at once (a dead peer costs one budget in total).  Codes: 1 slot
// not freed, 2 data not arrived, 16 routing overflow (a row that would not fit its slot region).
// Memory model: the workspace (control words AND payload) is FINE-GRAINED device memory
// (hipDeviceMallocFinegrained, runtime ws_alloc flags=2, the default): HIP/HSA define
// system-scope coherence for fine-grained memory, so a peer's stores that precede its
// system-scope release (and the flag store after it) are visible to this GPU after its
// system-scope acquire that follows reading the flag — no reliance on L2 write-back of
// coarse-grained memory.  Payload = plain 16-byte stores over xGMI, then every storing wave's
// vmcnt(0) + workgroup barrier + system-scope release fence before the arrival counter; the
// last arriving block publishes with another release + system-scope flag store; readers poll
// relaxed system-scope loads and acquire (system scope) before touching the payload.
#pragma once

#ifndef TL_EP_TIMEOUT_TICKS
#define TL_EP_TIMEOUT_TICKS 2000000000ull  // 20 s at 100 MHz
#endif

namespace tl {
namespace ep {

// control words (u32 offsets into the buffer); W <= 32
constexpr int MAXW = 32;
constexpr int CNT = 0, DFLAG = 2 * MAXW, RFLAG = 4 * MAXW, RFREE = 6 * MAXW, TFREE = 8 * MAXW, CTR = 10 * MAXW;
constexpr long long CTRL_BYTES = 4096;

struct Layout {
  int W, cap;
  long long row_bytes;
  TL_DEVICE long long eids_off() const { return CTRL_BYTES; }
  TL_DEVICE long long recv_off() const { return (CTRL_BYTES + 2ll * W * cap * 4 + 4095) & ~4095ll; }
  TL_DEVICE long long ret_off() const { return recv_off() + 2ll * W * cap * row_bytes; }
};

TL_DEVICE unsigned* ctrl(char* base) { return reinterpret_cast<unsigned*>(base); }
TL_DEVICE void st_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
TL_DEVICE unsigned ld_sys(unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); }

// one lane: wait until *p == v (exact) or (int)(*p - v) >= 0; bounded; error code on timeout.
// Once this rank's error word is set (by any wait of this or an earlier kernel that has not been
// raised yet) every later wait gives up at once: a dead peer costs ONE budget, not one per wait.
TL_DEVICE bool failed(int* err) { return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0; }
TL_DEVICE void spin(unsigned* p, unsigned v, bool at_least, int* err, int code) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (true) {
    const unsigned x = ld_sys(p);
    if (at_least ? ((int)(x - v) >= 0) : (x == v)) return;
    if (failed(err) || __builtin_amdgcn_s_memrealtime() - t0 > TL_EP_TIMEOUT_TICKS) {
      __hip_atomic_fetch_or(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// copy one row (row_bytes, multiple of 16) with the 64 lanes of a wave: up to 8 x 16 B loads
// per lane in flight before their (remote) stores
TL_DEVICE void copy_row(char* __restrict__ dst, const char* __restrict__ src, long long row_bytes, int lane) {
  typedef int __attribute__((ext_vector_type(4))) i4;
  constexpr int U = 8;
  for (long long o0 = 0; o0 < row_bytes; o0 += U * 64 * 16) {
    i4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + ((long long)u * 64 + lane) * 16;
      if (o < row_bytes) v[u] = *reinterpret_cast<const i4*>(src + o);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long o = o0 + ((long long)u * 64 + lane) * 16;
      if (o < row_bytes) *reinterpret_cast<i4*>(dst + o) = v[u];
    }
  }
}

// every block: all waves' stores are complete and released at system scope; returns true in
// the block that arrived last (the counter is reset for the next use of this parity)
TL_DEVICE bool arrive_last(unsigned* ctr) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: write back, wait for stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned n = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    last = (n == gridDim.x);
    if (last) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
  }
  __syncthreads();
  return last != 0;
}

// x [T][H] rows of `row_bytes`; ids [P] global expert ids (P = T*topk, pair j reads row j/topk);
// ret_index [P] out: where pair j's result will be in RET[p] ([W*cap] rows)
template <int W>
TL_DEVICE void dispatch(const void* x_, const int* ids, int* ret_index, long long ws_tab, int me, int epoch,
                        long long err_, int P, int topk, int n_loc, int cap, long long row_bytes) {
  static_assert(W <= MAXW, "EP group too large");
  const char* x = reinterpret_cast<const char*>(x_);
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const Layout L{W, cap, row_bytes};
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  __shared__ int cnt_s[W];
  // slot of every pair: its rank among my pairs for the same destination (stable, computed
  // redundantly by every block: P is small, and this avoids a second kernel)
  if (threadIdx.x < W) cnt_s[threadIdx.x] = 0;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0 && e > 1u) {
    // my combine of step e-1 has finished (stream order): peers may refill RET[(e-1)&1][me]
    for (int d = 0; d < W; ++d) st_sys(ctrl(ws[d]) + TFREE + ((e - 1u) & 1u) * MAXW + me, e - 1u);
  }
  if (threadIdx.x == 0) {
    // the destinations consumed what I sent them two steps ago into parity p
    for (int d = 0; d < W; ++d)
      if (e > 2u) spin(own + RFREE + p * MAXW + d, e - 2u, true, err, 1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // each wave walks the pairs in order keeping per-destination counts in registers of lane d
  // (a prefix over all pairs: O(P) per wave, P = tokens*topk is a few thousand)
  int run = 0;  // lane d: pairs for destination d seen so far
  for (int j0 = 0; j0 < P; j0 += 64) {
    const int j = j0 + lane;
    const int d = j < P ? ids[j] / n_loc : -1;
    // lanes with the same destination, lower lane index: exclusive rank inside this chunk
    int rank_in_chunk = 0, chunk_cnt_mine = 0;
#pragma unroll
    for (int dd = 0; dd < W; ++dd) {
      const unsigned long long m = __ballot(d == dd);
      if (d == dd) rank_in_chunk = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == dd) chunk_cnt_mine = __popcll(m);
    }
    const int base = __shfl(run, d < 0 ? 0 : d, 64);
    run += chunk_cnt_mine;
    const int slot = base + rank_in_chunk;
    // an overflowing pair (flagged below, rows dropped) reads row 0: in range, and raised
    if (j < P && wave == 0 && blockIdx.x == 0) ret_index[j] = (d >= 0 && d < W && slot < cap) ? d * cap + slot : 0;
    // rows are dealt round-robin over every wave of the grid; a wave moves a row with all lanes
    const int gw = blockIdx.x * nw + wave, nwaves = gridDim.x * nw;
    for (int l = (gw - j0 % nwaves + nwaves) % nwaves; l < 64 && j0 + l < P; l += nwaves) {
      const int dl = __shfl(d, l, 64), sl = __shfl(slot, l, 64);
      const int jl = j0 + l;
      if (dl < 0 || dl >= W || sl >= cap) {
        // a routing id out of range, or more pairs for one destination than its RECV region
        // holds (cap assumes distinct experts per token): record it, never store past the slot
        if (lane == 0) __hip_atomic_fetch_or(err, 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        continue;
      }
      char* dst = ws[dl] + L.recv_off() + (((long long)p * W + me) * cap + sl) * row_bytes;
      copy_row(dst, x + (long long)(jl / topk) * row_bytes, row_bytes, lane);
      if (lane == 0) {
        int* eids = reinterpret_cast<int*>(ws[dl] + L.eids_off());
        eids[((long long)p * W + me) * cap + sl] = ids[jl] - dl * n_loc;
      }
    }
  }
  if (wave == 0 && lane < W) cnt_s[lane] = run;
  if (arrive_last(own + CTR + p)) {
    if (threadIdx.x < W) {
      const int d = threadIdx.x;
      st_sys(ctrl(ws[d]) + CNT + p * MAXW + me, (unsigned)cnt_s[d]);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int d = 0; d < W; ++d) st_sys(ctrl(ws[d]) + DFLAG + p * MAXW + me, e);
    }
  }
}

// wait for every sender's rows of step e; ids_out [W*cap]: local expert id or -1 (empty slot)
template <int W>
TL_DEVICE void recv_wait(int* ids_out, int* cnt_out, long long ws_tab, int me, int epoch, long long err_, int cap,
                         long long row_bytes) {
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const Layout L{W, cap, row_bytes};
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  __shared__ int cnt_s[W];
  if (threadIdx.x == 0) {
    for (int s = 0; s < W; ++s) spin(own + DFLAG + p * MAXW + s, e, false, err, 2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  if (threadIdx.x < W) {
    cnt_s[threadIdx.x] = (int)ld_sys(own + CNT + p * MAXW + threadIdx.x);
    if (blockIdx.x == 0) cnt_out[threadIdx.x] = cnt_s[threadIdx.x];
  }
  __syncthreads();
  const int* eids = reinterpret_cast<const int*>(ws[me] + L.eids_off()) + (long long)p * W * cap;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (long long)W * cap;
       i += (long long)gridDim.x * blockDim.x) {
    const int s = (int)(i / cap), k = (int)(i % cap);
    ids_out[i] = k < cnt_s[s] ? eids[i] : -1;
  }
}

// send the expert results back: row y[ydest[s*cap + i]] -> RET[p][me][i]@s for i < cnt[s]
template <int W>
TL_DEVICE void ret(const void* y_, const int* ydest, const int* cnt, long long ws_tab, int me, int epoch,
                   long long err_, int cap, long long row_bytes) {
  const char* y = reinterpret_cast<const char*>(y_);
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const Layout L{W, cap, row_bytes};
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the expert FFN of step e has read RECV[p] (stream order): senders may refill it at e+2
    for (int s = 0; s < W; ++s) st_sys(ctrl(ws[s]) + RFREE + p * MAXW + me, e);
  }
  if (threadIdx.x == 0) {
    for (int s = 0; s < W; ++s)
      if (e > 2u) spin(own + TFREE + p * MAXW + s, e - 2u, true, err, 1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int gw = blockIdx.x * nw + wave, nwaves = gridDim.x * nw;
  for (int s = 0; s < W; ++s) {
    const int n = cnt[s];
    char* dst = ws[s] + L.ret_off() + ((long long)p * W + me) * cap * row_bytes;
    for (int i = gw; i < n; i += nwaves)
      copy_row(dst + (long long)i * row_bytes, y + (long long)ydest[s * cap + i] * row_bytes, row_bytes, lane);
  }
  if (arrive_last(own + CTR + 2 + p)) {
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int s = 0; s < W; ++s) st_sys(ctrl(ws[s]) + RFLAG + p * MAXW + me, e);
    }
  }
}

// wait until every destination returned my rows of step e
template <int W>
TL_DEVICE void ret_wait(long long ws_tab, int me, int epoch, long long err_) {
  char* const* ws = reinterpret_cast<char* const*>(ws_tab);
  int* err = reinterpret_cast<int*>(err_);
  const unsigned e = (unsigned)epoch, p = e & 1u;
  unsigned* own = ctrl(ws[me]);
  if (threadIdx.x == 0) {
    for (int d = 0; d < W; ++d) spin(own + RFLAG + p * MAXW + d, e, false, err, 2);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  __syncthreads();
}

}  // namespace ep
}  // namespace tl
