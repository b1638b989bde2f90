"""MoE expert-FFN kernels (tilelang DSL) and the device-side token dispatch around them.

Layout (MI355X-first): tokens routed to expert ``e`` occupy a row block of a *padded* row
space whose start is a multiple of ``block_M``; a ``tile_expert`` table gives the expert of
every ``block_M`` row tile (``-1`` = empty tile, the block exits at once) and ``row_src`` the
source row of every padded row (``-1`` = padding).  Shapes are therefore static (``max_rows``
is the worst case), one compiled kernel serves every routing, nothing syncs with the host and
the launches are hipGraph-capturable.

One layer = 6 launches, all tilelang kernels except the router logits GEMM:
  router_topk   softmax-free top-k over the logits (renormalised weights cancel the softmax
                denominator), one thread per token
  moe_align     one workgroup: per-expert histogram (LDS atomics), padded prefix offsets,
                slot of every assignment, ``row_src`` / ``tile_expert`` tables
  gemm1         ``[g | u] = x[row_src] @ W1[e]^T`` — the A rows are gathered straight from
                the token matrix into LDS by per-lane LDS-DMA (``T.gather_rows``); no
                dispatch copy of the activations is ever materialised
  silu_mul      ``act = silu(g) * u``
  gemm2         ``y = act @ W2[e]^T`` (optionally summed across the mesh in-kernel)
  combine       ``out[t] = sum_k w[t, k] * y[dest[t, k]]`` in fp32, one pass, no atomics

Reference: ``examples/grouped_gemm/example_grouped_gemm_fwd.py`` (group search per tile) and
``examples/fusedmoe/example_fusedmoe_tilelang.py`` (routed SwiGLU experts).
"""
from __future__ import annotations

import functools
from typing import Optional, Tuple

import torch

import tilelang
import tilelang.language as T
from tilelang.layout import PaddedLayout


def _target(device) -> str:
    return "cpu" if torch.device(device).type == "cpu" else "hip"


def _tdt(dtype: torch.dtype) -> str:
    return {torch.float16: "float16", torch.bfloat16: "bfloat16", torch.float32: "float32"}[dtype]


def _bucket(n: int, lo: int = 256) -> int:
    """Power-of-two bucket >= n: data-dependent row counts reuse a handful of compiled kernels."""
    nb = lo
    while nb < n:
        nb *= 2
    return nb


@functools.lru_cache(maxsize=None)
def router_topk_kernel(n_tok: int, E: int, topk: int, target: str, threads: int = 256, parts: int = 0,
                       E_stride: int = 0, round_dtype: Optional[str] = None):
    """``ids[t] = topk(logits[t])``, ``w[t] = softmax(logits[t])[ids] / sum`` — the renormalised
    top-k weights equal ``exp(l_k - m) / sum_k' exp(l_k' - m)`` (the softmax denominator cancels).
    ``parts`` > 0: ``L`` is ``[parts, n_tok, E_stride]`` fp32 partial logits (a K-split router GEMM),
    summed here; ``round_dtype``: the summed logit is rounded to that dtype first (as a library
    GEMM's output would be)."""
    Es = E_stride or E
    L_shape = (parts, n_tok, Es) if parts else (n_tok, E)

    @T.prim_func
    def moe_router_topk(L: T.Tensor(L_shape, "float32"), ids: T.Tensor((n_tok, topk), "int32"),
             w: T.Tensor((n_tok, topk), "float32")):
        with T.Kernel(T.ceildiv(n_tok, threads), threads=threads) as bx:
            for i in T.Parallel(threads):
                v = T.alloc_local((E,), "float32")
                sel = T.alloc_local((topk,), "int32")
                p = T.alloc_local((topk,), "float32")
                best = T.alloc_var("float32")
                bi = T.alloc_var("int32")
                tot = T.alloc_var("float32")
                if bx * threads + i < n_tok:
                    for e in T.serial(E):
                        if parts:
                            v[e] = L[0, bx * threads + i, e]
                            for q in T.serial(parts - 1):
                                v[e] = v[e] + L[q + 1, bx * threads + i, e]
                        else:
                            v[e] = L[bx * threads + i, e]
                        if round_dtype is not None:
                            v[e] = T.Cast("float32", T.Cast(round_dtype, v[e]))
                    for k in T.serial(topk):
                        best = -T.infinity("float32")
                        bi = 0
                        for e in T.serial(E):
                            if v[e] > best:
                                best = v[e]
                                bi = e
                        sel[k] = bi
                        p[k] = best
                        v[bi] = -T.infinity("float32")
                    tot = 0.0
                    best = p[0]
                    for k in T.serial(topk):
                        p[k] = T.exp(p[k] - best)
                        tot = tot + p[k]
                    for k in T.serial(topk):
                        ids[bx * threads + i, k] = sel[k]
                        w[bx * threads + i, k] = p[k] / tot

    return tilelang.compile(moe_router_topk, out_idx=None, target=target)


@functools.lru_cache(maxsize=None)
def router_fused_kernel(n_tok: int, H: int, E: int, topk: int, dtype: str, target: str, block_T: int = 16,
                        block_K: int = 256, num_stages: int = 3):
    """Router in one kernel: logits = x Wg^T on the matrix cores (experts padded to the 16-wide MFMA
    N dimension, padded rows of Wg are zero and masked), rounded to the activation dtype like a
    library GEMM's output, then the top-k of each row and its renormalised softmax weights
    (``router_topk_kernel``'s rule) from LDS.  Replaces vendor GEMM + fp32 cast + top-k kernel
    (three launches, ~25 us at 2048 x 4096 x 8 on MI355X) with one pass over x.
    kernel(x [n_tok, H], Wg [Ep, H] (Ep = E rounded up to 16), ids, w)."""
    Ep = max(16, -(-E // 16) * 16)
    assert H % block_K == 0

    @T.prim_func
    def moe_router_fused(X: T.Tensor((n_tok, H), dtype), Wg: T.Tensor((Ep, H), dtype),
                         ids: T.Tensor((n_tok, topk), "int32"), w: T.Tensor((n_tok, topk), "float32")):
        with T.Kernel(T.ceildiv(n_tok, block_T), threads=64) as bx:
            X_s = T.alloc_shared((block_T, block_K), dtype)
            W_s = T.alloc_shared((Ep, block_K), dtype)
            L = T.alloc_fragment((block_T, Ep), "float32")
            L_s = T.alloc_shared((block_T, Ep), "float32")
            T.clear(L)
            for k in T.Pipelined(H // block_K, num_stages=num_stages):
                T.copy(X[bx * block_T, k * block_K], X_s)
                T.copy(Wg[0, k * block_K], W_s)
                T.gemm(X_s, W_s, L, transpose_B=True)
            for i, e in T.Parallel(block_T, Ep):
                L_s[i, e] = T.Cast("float32", T.Cast(dtype, L[i, e]))
            for i in T.Parallel(64):
                v = T.alloc_local((Ep,), "float32")
                sel = T.alloc_local((topk,), "int32")
                p = T.alloc_local((topk,), "float32")
                best = T.alloc_var("float32")
                bi = T.alloc_var("int32")
                tot = T.alloc_var("float32")
                if (i < block_T) & (bx * block_T + i < n_tok):
                    for e in T.serial(E):
                        v[e] = L_s[i, e]
                    for kk in T.serial(topk):
                        best = -T.infinity("float32")
                        bi = 0
                        for e in T.serial(E):
                            if v[e] > best:
                                best = v[e]
                                bi = e
                        sel[kk] = bi
                        p[kk] = best
                        v[bi] = -T.infinity("float32")
                    tot = 0.0
                    best = p[0]
                    for kk in T.serial(topk):
                        p[kk] = T.exp(p[kk] - best)
                        tot = tot + p[kk]
                    for kk in T.serial(topk):
                        ids[bx * block_T + i, kk] = sel[kk]
                        w[bx * block_T + i, kk] = p[kk] / tot

    return tilelang.compile(moe_router_fused, out_idx=None, target=target)


@functools.lru_cache(maxsize=None)
def router_logits_sk_kernel(n_tok: int, H: int, E: int, dtype: str, target: str, splits: int = 4, block_T: int = 16,
                            block_K: int = 256, num_stages: int = 3):
    """Router logits as a K-split MFMA GEMM: workgroup (token block, split) writes the fp32 partial
    ``x[:, split] Wg[:, split]^T`` of its 16 tokens to ``P[split]`` (plain stores; the top-k kernel
    sums the ``splits`` partials).  The fused router streams each token block's whole ``H`` through
    ONE wave (n_tok / 16 waves on the chip: 128 for the bench layer, latency-bound); this puts
    ``splits`` times as many waves -- and bytes in flight -- on the same pass over x."""
    Ep = max(16, -(-E // 16) * 16)
    Hs = H // splits
    assert H % splits == 0 and Hs % block_K == 0

    @T.prim_func
    def moe_router_logits_sk(X: T.Tensor((n_tok, H), dtype), Wg: T.Tensor((Ep, H), dtype),
                             P: T.Tensor((splits, n_tok, Ep), "float32")):
        with T.Kernel(T.ceildiv(n_tok, block_T), splits, threads=64) as (bx, sk):
            X_s = T.alloc_shared((block_T, block_K), dtype)
            W_s = T.alloc_shared((Ep, block_K), dtype)
            L = T.alloc_fragment((block_T, Ep), "float32")
            T.clear(L)
            for k in T.Pipelined(Hs // block_K, num_stages=num_stages):
                T.copy(X[bx * block_T, sk * Hs + k * block_K], X_s)
                T.copy(Wg[0, sk * Hs + k * block_K], W_s)
                T.gemm(X_s, W_s, L, transpose_B=True)
            T.copy(L, P[sk, bx * block_T, 0])

    return tilelang.compile(moe_router_logits_sk, out_idx=None, target=target)


@functools.lru_cache(maxsize=None)
def router_wide_kernel(n_tok: int, H: int, E: int, topk: int, dtype: str, target: str, block_T: int = 8, kc: int = 4,
                       block_K: int = 128, num_stages: int = 4, threads: int = 512):
    """Router with the K dimension spread over ``kc`` chunks that run side by side in ONE tile
    GEMM (the fused router streams a token block's whole ``H`` through a single wave: 128
    latency-bound waves on the chip for the bench layer, ~9 us).  With x viewed as
    ``[n_tok * kc, H / kc]`` (row ``t * kc + c`` = chunk c of token t) and the padded gate as
    ``[Ep * kc, H / kc]`` (row ``e * kc + c``), P = x' Wg'^T holds every (token chunk, expert
    chunk) product and the logit is the sum of its ``kc`` matching-chunk entries
    ``P[t*kc + c, e*kc + c]`` -- kc times the (tiny) MFMA work, but ``block_T * kc`` rows of x in
    flight per workgroup on 8 waves and ``n_tok / block_T`` workgroups.  Logits are rounded to the
    activation dtype and the top-k / softmax rule is ``router_topk_kernel``'s.  Defaults from
    scripts/router_wide_probe.py (bench layer 2048 x 4096 x 8, cold): 9.8 us vs 12.0 us fused, ids
    identical (profiles/r5/router_wide2.log).
    kernel(x [n_tok * kc, H / kc], Wg [Ep * kc, H / kc], ids, w)."""
    Ep = max(16, -(-E // 16) * 16)
    Hc = H // kc
    R, Rw = block_T * kc, Ep * kc
    assert H % kc == 0 and Hc % block_K == 0 and n_tok % block_T == 0 and R % 16 == 0

    @T.prim_func
    def moe_router_wide(X: T.Tensor((n_tok * kc, Hc), dtype), Wg: T.Tensor((Rw, Hc), dtype),
                        ids: T.Tensor((n_tok, topk), "int32"), w: T.Tensor((n_tok, topk), "float32")):
        with T.Kernel(n_tok // block_T, threads=threads) as bx:
            X_s = T.alloc_shared((R, block_K), dtype)
            W_s = T.alloc_shared((Rw, block_K), dtype)
            P = T.alloc_fragment((R, Rw), "float32")
            P_s = T.alloc_shared((R, Rw), "float32")
            L_s = T.alloc_shared((block_T, Ep), "float32")
            T.clear(P)
            for k in T.Pipelined(Hc // block_K, num_stages=num_stages):
                T.copy(X[bx * R, k * block_K], X_s)
                T.copy(Wg[0, k * block_K], W_s)
                T.gemm(X_s, W_s, P, transpose_B=True)
            T.copy(P, P_s)
            for i, e in T.Parallel(block_T, Ep):
                acc = T.alloc_var("float32")
                acc = 0.0
                for c in T.serial(kc):
                    acc = acc + P_s[i * kc + c, e * kc + c]
                L_s[i, e] = T.Cast("float32", T.Cast(dtype, acc))
            for i in T.Parallel(64):
                v = T.alloc_local((Ep,), "float32")
                sel = T.alloc_local((topk,), "int32")
                p = T.alloc_local((topk,), "float32")
                best = T.alloc_var("float32")
                bi = T.alloc_var("int32")
                tot = T.alloc_var("float32")
                if i < block_T:
                    for e in T.serial(E):
                        v[e] = L_s[i, e]
                    for kk in T.serial(topk):
                        best = -T.infinity("float32")
                        bi = 0
                        for e in T.serial(E):
                            if v[e] > best:
                                best = v[e]
                                bi = e
                        sel[kk] = bi
                        p[kk] = best
                        v[bi] = -T.infinity("float32")
                    tot = 0.0
                    best = p[0]
                    for kk in T.serial(topk):
                        p[kk] = T.exp(p[kk] - best)
                        tot = tot + p[kk]
                    for kk in T.serial(topk):
                        ids[bx * block_T + i, kk] = sel[kk]
                        w[bx * block_T + i, kk] = p[kk] / tot

    return tilelang.compile(moe_router_wide, out_idx=None, target=target)


ROUTER_SPLITS = int(__import__("os").environ.get("TL_MOE_ROUTER_SPLITS", "0"))  # 0: the fused one-pass router
# the wide router (router_wide_kernel) for the shapes it takes; TL_MOE_ROUTER_WIDE=0: the fused one
ROUTER_WIDE = __import__("os").environ.get("TL_MOE_ROUTER_WIDE", "1") != "0"


_GATE_PAD = {}


def _padded_gate(gate_w: torch.Tensor) -> torch.Tensor:
    """Wg padded with zero rows to a multiple of 16 experts (cached per weight tensor)."""
    key = (gate_w.data_ptr(), tuple(gate_w.shape), gate_w.dtype, gate_w._version)
    g = _GATE_PAD.get(key)
    if g is None:
        E, H = gate_w.shape
        Ep = max(16, -(-E // 16) * 16)
        g = torch.zeros(Ep, H, dtype=gate_w.dtype, device=gate_w.device)
        g[:E] = gate_w
        if len(_GATE_PAD) > 64:
            _GATE_PAD.clear()
        _GATE_PAD[key] = g
    return g


def max_padded_rows(n_assign: int, E: int, block_M: int) -> int:
    """Worst-case rows of the padded layout for ``n_assign`` (row, expert) pairs."""
    rows = n_assign + E * (block_M - 1)
    return (rows + block_M - 1) // block_M * block_M


@functools.lru_cache(maxsize=None)
def align_kernel(n: int, E: int, block_M: int, max_rows: int, div: int, target: str, stable: bool = False,
                 threads: int = 1024, full_first: bool = True, even: bool = False, vote: Optional[bool] = None):
    """Dispatch plan of ``n`` assignments (``expert_ids[n]``; assignment ``j`` reads source row
    ``j // div``; a negative id is an empty slot: not placed, ``dest[j] = -1``): ``dest[j]`` (its
    padded row), ``row_src[max_rows]``, ``tile_expert``, ``counts[E]``,
    ``tile_rows`` (valid rows of every row tile: they are a prefix of the tile).

    One workgroup.  ``stable=False``: rows of one expert are placed in LDS-atomic order (each
    row's result is independent of its position, so the layer output does not depend on it).
    ``stable=True``: assignment order is kept inside every expert (per-thread runs + a scan of
    the per-thread counts; on gfx950 ``vote``: per-wave ballot counts + a scan over the waves) —
    identical placement on every rank, which the tensor-parallel in-kernel reduction needs.

    ``full_first``: every expert's FULL row tiles come first (expert order), then one partial tile
    per expert with a remainder.  The tail-balanced expert GEMM runs the leading units as whole
    tiles and splits only the trailing ones: with the partial tiles (usually a few valid rows)
    last, the whole-tile rounds are all full tiles and the split tail is the nearly-empty work
    (before, an expert's partial tile sat between full ones and full tiles landed in the tail).

    ``even``: an expert's ``cnt`` rows are spread evenly over its ``ceil(cnt / block_M)`` row tiles
    (the first ``cnt % n`` tiles hold one row more), not filled tile by tile.  With ``block_M`` a
    row-tile *slot* of ``main + ext`` rows (``expert_gemm_sk_kernel(ext_M=)``) an expert of 529
    rows becomes two tiles of 265 / 264 rows -- two units of a one-round grid -- instead of two
    full tiles plus a 17-row tile that costs a whole extra round."""
    if even:
        full_first = False
    if vote is None:
        # measured (scripts/align_probe.py, profiles/r5/align_probe3.log): the vote form keeps
        # assignment order at 12.4 us vs 27.8 us for the per-thread-run stable form; the unordered
        # LDS-atomic form stays the default (11.3 vs 12.3 us)
        vote = target == "hip" and stable
    n_tiles = max_rows // block_M
    if stable and not vote:
        threads = 256
    c = -(-n // threads)
    nw = threads // 64

    def _units(c):  # row tiles of an expert with c rows
        return (c + block_M - 1) // block_M

    def _even_row(sl, c):
        """Padded offset of the expert's sl-th row under the even split: tile j holds q + (j < r)
        rows, q = c // n, r = c % n, n = _units(c)."""
        nu = T.max(_units(c), 1)
        q = c // nu
        big = (q + 1) * (c % nu)
        j = T.if_then_else(sl < big, sl // (q + 1), c % nu + (sl - big) // T.max(q, 1))
        off = T.if_then_else(sl < big, sl % (q + 1), (sl - big) % T.max(q, 1))
        return j * block_M + off

    @T.prim_func
    def moe_align(expert_ids: T.Tensor((n,), "int32"), dest: T.Tensor((n,), "int32"),
             row_src: T.Tensor((max_rows,), "int32"), tile_expert: T.Tensor((n_tiles,), "int32"),
             counts: T.Tensor((E,), "int32"), tile_rows: T.Tensor((n_tiles,), "int32")):
        # written with T.Parallel (one iteration per thread on the GPU, a serial loop on the
        # CPU target), never with raw thread ids, so the same program runs on both
        with T.Kernel(1, threads=threads):
            cnt = T.alloc_shared((E,), "int32")
            start = T.alloc_shared((E + 1,), "int32")
            fill = T.alloc_shared((E,), "int32")
            acc = T.alloc_var("int32")
            if vote:
                # wave votes (gfx950): wave w owns the c*64 consecutive assignments from w*c*64, its
                # lanes cover 64 at a time; per expert the wave counts its lanes with a ballot, an
                # exclusive scan over the waves gives each wave its offset, and a lane's slot is
                # offset + the wave's running count + the set lanes below it -- assignment order
                # inside every expert (stable) and no LDS atomics
                wc = T.alloc_shared((nw, E), "int32")
                for t in T.Parallel(threads):
                    tot = T.alloc_local((E,), "int32")
                    for e in T.serial(E):
                        tot[e] = 0
                    for it in T.serial(c):
                        j = (t // 64) * (c * 64) + it * 64 + t % 64
                        idv = T.alloc_var("int32")
                        idv = T.if_then_else(j < n, expert_ids[T.min(j, n - 1)], -1)
                        for e in T.serial(E):
                            tot[e] = tot[e] + T.call_extern("int32", "tl::popc64", T.ballot(idv == e))
                    if t % 64 == 0:
                        for e in T.serial(E):
                            wc[t // 64, e] = tot[e]
                for e in T.Parallel(E):
                    acc = 0
                    for w_ in T.serial(nw):
                        cq = T.alloc_var("int32")
                        cq = wc[w_, e]
                        wc[w_, e] = acc
                        acc = acc + cq
                    cnt[e] = acc
            elif stable:
                tc = T.alloc_shared((threads, E), "int32")
                run = T.alloc_shared((threads, E), "int32")
                for t in T.Parallel(threads):
                    for e in T.serial(E):
                        tc[t, e] = 0
                    for i in T.serial(c):
                        if t * c + i < n and expert_ids[t * c + i] >= 0:
                            tc[t, expert_ids[t * c + i]] = tc[t, expert_ids[t * c + i]] + 1
                T.cumsum(tc, run, dim=0)
                for e in T.Parallel(E):
                    cnt[e] = run[threads - 1, e]
            else:
                for e in T.Parallel(E):
                    cnt[e] = 0
                    fill[e] = 0
                for j in T.Parallel(n):
                    if expert_ids[j] >= 0:
                        T.atomic_add(cnt[expert_ids[j]], 1)
            for r in T.Parallel(max_rows):
                row_src[r] = -1
            if full_first:
                pstart = T.alloc_shared((E,), "int32")
                for z in T.Parallel(1):
                    acc = 0
                    for e in T.serial(E):  # full tiles of every expert
                        start[e] = acc
                        acc = acc + cnt[e] // block_M * block_M
                    # then one partial tile per expert with a remainder, fullest first: the
                    # tail-balanced GEMM splits the LAST units, which are then the lightest
                    npart = T.alloc_var("int32")
                    npart = 0
                    for e in T.serial(E):
                        rk = T.alloc_var("int32")
                        rk = 0
                        for e2 in T.serial(E):
                            if cnt[e2] % block_M > cnt[e] % block_M or (
                                    cnt[e2] % block_M == cnt[e] % block_M and e2 < e):
                                rk = rk + 1
                        pstart[e] = acc + rk * block_M
                        if cnt[e] % block_M > 0:
                            npart = npart + 1
                    start[E] = acc + npart * block_M + z
            else:
                for z in T.Parallel(1):
                    acc = 0
                    for e in T.serial(E):
                        start[e] = acc
                        acc = acc + (cnt[e] + block_M - 1) // block_M * block_M
                    start[E] = acc + z
            for e in T.Parallel(E):
                counts[e] = cnt[e]
            for tt in T.Parallel(n_tiles):
                te = T.alloc_var("int32")
                tr = T.alloc_var("int32")
                te = -1
                tr = 0
                for e in T.serial(E):
                    if full_first:
                        if tt * block_M >= start[e] and tt * block_M < start[e] + cnt[e] // block_M * block_M:
                            te = e
                            tr = block_M
                        if cnt[e] % block_M > 0 and tt * block_M == pstart[e]:
                            te = e
                            tr = cnt[e] % block_M
                    elif even:
                        if tt * block_M >= start[e] and tt * block_M < start[e] + _units(cnt[e]) * block_M:
                            te = e
                            tr = cnt[e] // _units(cnt[e]) + T.if_then_else(
                                (tt * block_M - start[e]) // block_M < cnt[e] % _units(cnt[e]), 1, 0)
                    else:
                        if tt * block_M >= start[e] and tt * block_M < start[e] + cnt[e]:
                            te = e
                            tr = T.min(start[e] + cnt[e] - tt * block_M, block_M)
                tile_expert[tt] = te
                tile_rows[tt] = tr
            if vote:
                for t in T.Parallel(threads):
                    run_ = T.alloc_local((E,), "int32")
                    for e in T.serial(E):
                        run_[e] = wc[t // 64, e]
                    for it in T.serial(c):
                        j = (t // 64) * (c * 64) + it * 64 + t % 64
                        idv = T.alloc_var("int32")
                        sl = T.alloc_var("int32")
                        idv = T.if_then_else(j < n, expert_ids[T.min(j, n - 1)], -1)
                        sl = 0
                        for e in T.serial(E):
                            m = T.ballot(idv == e)
                            if idv == e:
                                sl = run_[e] + T.call_extern("int32", "tl::mbcnt64", m)
                            run_[e] = run_[e] + T.call_extern("int32", "tl::popc64", m)
                        if j < n and idv >= 0:
                            e_ = T.min(idv, E - 1)
                            d = start[e_] + sl
                            if full_first:  # slot sl of expert e -> its full or partial tile
                                d = T.if_then_else(sl < cnt[e_] // block_M * block_M, start[e_] + sl,
                                                   pstart[e_] + sl - cnt[e_] // block_M * block_M)
                            if even:
                                d = start[e_] + _even_row(sl, cnt[e_])
                            dest[j] = d
                            row_src[d] = j // div
                        if j < n and idv < 0:
                            dest[j] = -1
            elif stable:
                for t in T.Parallel(threads):
                    for e in T.serial(E):
                        run[t, e] = start[e] + run[t, e] - tc[t, e]
                    for i in T.serial(c):
                        if t * c + i < n and expert_ids[t * c + i] >= 0:
                            e_ = expert_ids[t * c + i]
                            d = run[t, e_]
                            run[t, e_] = d + 1
                            if full_first:  # slot d - start[e] of expert e -> its full or partial tile
                                sl = d - start[e_]
                                d = T.if_then_else(sl < cnt[e_] // block_M * block_M, d,
                                                   pstart[e_] + sl - cnt[e_] // block_M * block_M)
                            if even:
                                d = start[e_] + _even_row(d - start[e_], cnt[e_])
                            dest[t * c + i] = d
                            row_src[d] = (t * c + i) // div
                        if t * c + i < n and expert_ids[t * c + i] < 0:
                            dest[t * c + i] = -1
            else:
                for j in T.Parallel(n):
                    if expert_ids[j] >= 0:
                        e_ = expert_ids[j]
                        slot = T.atomic_add(fill[e_], 1, return_prev=True)
                        if full_first:
                            d = T.if_then_else(slot < cnt[e_] // block_M * block_M, start[e_] + slot,
                                               pstart[e_] + slot - cnt[e_] // block_M * block_M)
                            dest[j] = d
                            row_src[d] = j // div
                        elif even:
                            d = start[e_] + _even_row(slot, cnt[e_])
                            dest[j] = d
                            row_src[d] = j // div
                        else:
                            dest[j] = start[e_] + slot
                            row_src[start[e_] + slot] = j // div
                    if expert_ids[j] < 0:
                        dest[j] = -1

    return tilelang.compile(moe_align, out_idx=None, target=target)



@functools.lru_cache(maxsize=None)
def expert_gemm_kernel(max_rows: int, K: int, N: int, E: int, dtype: str, target: str, block_M: int = 128,
                       block_N: int = 128, block_K: int = 64, num_stages: int = 2, threads: int = 256,
                       reduce_mesh: Optional[str] = None, mesh_shape: Optional[Tuple[int, int]] = None,
                       n_src: Optional[int] = None, swiglu: bool = False, persistent_blocks: int = 256,
                       skip_padding: bool = True):
    """``C[r, :] = A[src(r), :] @ W[tile_expert[r // block_M]].T`` for every non-empty row tile.

    ``n_src`` given: A is the ``[n_src, K]`` source-row matrix and row ``r`` of the padded row
    space reads ``A[row_src[r]]`` (``-1`` = padding = zeros), gathered straight into LDS.
    ``reduce_mesh`` ("all"/"h"/"v"): tensor-parallel partial products are summed across the
    mesh inside the kernel (``T.comm.all_reduce_tile`` on the fp32 accumulator tile) by a persistent
    grid of ``persistent_blocks`` workgroups (one per CU) walking the tiles.
    ``swiglu``: W's rows are interleaved in groups of 4 (gate 2p, gate 2p+1, up 2p, up 2p+1, see
    ``swiglu_interleave``) and the epilogue writes ``C[r, p] = silu(gate) * up`` ([max_rows, N/2]):
    the 4 columns of such a group sit in the registers of ONE lane (MFMA C layout), so the
    activation needs no data movement and no separate kernel.
    ``skip_padding``: waves whose rows of a row tile are all padding skip their MFMAs
    (``T.gemm(valid_m=tile_rows[tile])``) — an expert's last tile is usually mostly padding."""
    n_tiles = max_rows // block_M
    n_by = (N + block_N - 1) // block_N
    n_work = n_tiles * n_by
    n_prog = min(n_work, persistent_blocks)
    accum = "float32"
    a_rows = n_src if n_src is not None else max_rows
    n_out = N // 2 if swiglu else N
    assert not (swiglu and reduce_mesh), "the SwiGLU epilogue belongs to the first expert GEMM"

    if reduce_mesh is None:

        @T.prim_func
        def moe_expert_gemm(A: T.Tensor((a_rows, K), dtype), W: T.Tensor((E, N, K), dtype),
                            tile_expert: T.Tensor((n_tiles,), "int32"), row_src: T.Tensor((max_rows,), "int32"),
                            tile_rows: T.Tensor((n_tiles,), "int32"), C: T.Tensor((max_rows, n_out), dtype)):
            with T.Kernel(n_tiles, T.ceildiv(N, block_N), threads=threads) as (bx, by):
                A_s = T.alloc_shared((block_M, block_K), dtype)
                W_s = T.alloc_shared((block_N, block_K), dtype)
                C_l = T.alloc_fragment((block_M, block_N), accum)
                e = tile_expert[bx]
                if e >= 0:
                    T.clear(C_l)
                    for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                        if n_src is not None:
                            T.gather_rows(A[:, k * block_K:(k + 1) * block_K],
                                          row_src[bx * block_M:(bx + 1) * block_M], A_s, row_dim=0)
                        else:
                            T.copy(A[bx * block_M, k * block_K], A_s)
                        # clamped expert id: provably in bounds, so the W tile is an LDS-DMA producer
                        T.copy(W[T.min(T.max(e, 0), E - 1), by * block_N, k * block_K], W_s)
                        # an expert's last row tile is partly padding: its empty waves skip the MFMAs
                        T.gemm(A_s, W_s, C_l, transpose_B=True, valid_m=tile_rows[bx] if skip_padding else None)
                    if swiglu:
                        for i, j in T.Parallel(block_M, block_N):
                            if j % 4 < 2:
                                C[bx * block_M + i, by * (block_N // 2) + (j // 4) * 2 + j % 4] = T.Cast(
                                    dtype, C_l[i, j] / (1.0 + T.exp(-C_l[i, j])) * C_l[i, j + 2])
                    else:
                        T.copy(C_l, C[bx * block_M, by * block_N])

        return tilelang.compile(moe_expert_gemm, out_idx=None, target=target,
                                pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True} if swiglu else None)

    @T.prim_func
    def moe_expert_gemm_tp(A: T.Tensor((a_rows, K), dtype), W: T.Tensor((E, N, K), dtype),
                           tile_expert: T.Tensor((n_tiles,), "int32"), row_src: T.Tensor((max_rows,), "int32"),
                           tile_rows: T.Tensor((n_tiles,), "int32"), C: T.Tensor((max_rows, n_out), dtype)):
        # persistent grid: the cross-GPU all-reduce needs every block of every rank resident at
        # once (tl_runtime refuses larger grids), and the mesh workspace scales with the grid
        with T.Kernel(n_prog, threads=threads) as pid:
            A_s = T.alloc_shared((block_M, block_K), dtype)
            W_s = T.alloc_shared((block_N, block_K), dtype)
            C_l = T.alloc_fragment((block_M, block_N), accum)
            C_r = T.alloc_fragment((block_M, block_N), accum)
            for it in T.serial(T.ceildiv(n_work, n_prog)):
                t = pid + it * n_prog
                # every rank holds the same tile table (replicated tokens), so all ranks take
                # the same branches and meet at the same mesh op instances
                if t < n_work:
                    bx = t // n_by
                    by = t % n_by
                    e = tile_expert[bx]
                    if e >= 0:
                        T.clear(C_l)
                        for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                            if n_src is not None:
                                T.gather_rows(A[:, k * block_K:(k + 1) * block_K],
                                              row_src[bx * block_M:(bx + 1) * block_M], A_s, row_dim=0)
                            else:
                                T.copy(A[bx * block_M, k * block_K], A_s)
                            T.copy(W[T.min(T.max(e, 0), E - 1), by * block_N, k * block_K], W_s)
                            T.gemm(A_s, W_s, C_l, transpose_B=True, valid_m=tile_rows[bx] if skip_padding else None)
                        T.comm.all_reduce_tile(C_l, C_r, "sum", reduce_mesh)
                        T.copy(C_r, C[bx * block_M, by * block_N])

    return tilelang.compile(moe_expert_gemm_tp, out_idx=None, target=target)


@functools.lru_cache(maxsize=None)
def expert_gemm_sk_kernel(max_rows: int, K: int, N: int, E: int, dtype: str, target: str, block_M: int = 256,
                          block_N: int = 256, block_K: int = 64, num_stages: int = 2, threads: int = 512,
                          n_src: Optional[int] = None, swiglu: bool = False, n_cu: int = 256, tail_split: int = 4,
                          phased: bool = False, skip_padding: bool = True, partial_first: bool = False,
                          tail_ksplit: int = 0, tail_stages: Optional[int] = None, ext_M: int = 0,
                          quad: bool = True, staged_epi: bool = True):
    """Tail-balanced variant of ``expert_gemm_kernel`` (same arguments and output).

    ``staged_epi``: the tile's C (or its SwiGLU activation) goes through row-padded LDS and leaves
    as row-contiguous 16-byte stores (the 32 extension rows keep direct stores).  The staging tile
    shares bytes with the operand ring: the persistent tile loops are ``lds_iteration_local``
    (transform/lds_plan.py), so the planner separates the two tenants inside every iteration.
    Dense stand-in of GEMM2 (4608x4096x2048 bf16): 743 -> 811 TF; bench layer, random routing:
    GEMM1 118 -> 115.5 us, GEMM2 69.5 -> 65.7 us (``profiles/r5/moe_epi/``).

    ``quad``: the whole-tile main loop (256x256x64, 512 threads, row gather + ``ext_M`` = 32
    extension included) runs the 8-phase quadrant schedule ``tl::gemm_quad_nt_x`` (tl.gemm_quad);
    False keeps the generic 2-stage pipeline.

    ``ext_M`` > 0: a row tile is a slot of ``block_M + ext_M`` rows (the dispatch layout's
    ``block_M`` is that slot, ``align_kernel(even=True)``): the first ``block_M`` rows run as the
    usual tile, rows ``block_M..`` as an ``ext_M x block_N`` extension GEMM on the SAME W tile in
    the same K loop (its own small gather; waves split it by columns so every wave skips the same
    empty fragments).  A 529-row expert is then two units of 265 / 264 rows, 12.5 % more MFMA
    work on one of them, instead of a 17-row third unit that needs its own pass over W.

    ``tail_ksplit`` = S > 0: the trailing units run as S K-chunks each (full tile width) instead of
    narrow tiles.  Measured SLOWER on the bench layer (GEMM1 173 -> 255 / 357 / 572 us for S = 2 /
    4 / 8, profiles/r3/s3/moe/expert_gemm_probe.log): the partial tiles of the tail are often
    nearly full (an expert with 500 rows has one full tile and a 244-row partial), so the fp32
    partials are large and their traffic grows with S.  Kept as an option, off by default.  Every chunk writes its fp32
    partial (valid rows only) to a workspace slot, publishes it (release fence + counter); the
    last of the S chunks to arrive adds the others' partials and runs the epilogue, then resets
    the counter -- one kernel, no host sync, no separate reduction pass.  Extra arguments:
    ``WS [n_cu, S, block_M, block_N] fp32`` and ``Cnt [n_cu] int32`` (zero before the first call).

    ``partial_first``: with the full-tiles-first dispatch layout, rotate the unit order so the
    (nearly-empty) partial tiles run in the whole-tile rounds and full tiles form the split tail:
    the workgroups that drew a partial tile finish early and start on the tail at once.

    The (row tile x N tile) units are a data-dependent count U (the routing decides how many
    row tiles are real), and a plain grid runs ceil(U / n_cu) rounds of whole tiles: U = 320 on
    256 CUs -- the bench's 8-expert layer -- is two rounds for 1.25 rounds of work.  Here a
    persistent grid of ``n_cu`` workgroups runs the floor(U / n_cu) * n_cu leading units as whole
    ``block_M x block_N`` tiles, and the R = U mod n_cu trailing units as ``tail_split`` times
    narrower ``block_M x block_N / tail_split`` tiles over the full K (R * tail_split workgroups:
    one short round instead of a long one).  No K split, so no partial sums, workspace or second
    kernel; the SwiGLU epilogue's 4-column groups stay inside a narrow tile.  Every workgroup
    derives U and R from ``tile_expert`` (the real tiles are a prefix): nothing waits on the host."""
    slot = block_M + ext_M
    assert not (ext_M and tail_ksplit), "ext_M runs with the narrow-tile tail"
    staged_epi = staged_epi and not tail_ksplit  # the K-split tail's loops are not iteration-local
    n_tiles = max_rows // slot
    n_by = (N + block_N - 1) // block_N
    nk = (K + block_K - 1) // block_K
    bn_t = block_N // tail_split
    # the narrow tail tiles are latency-bound (a partial tile's K loop carries little MFMA work):
    # a deeper LDS ring there (the whole-tile ring is dead by then; the LDS planner shares bytes)
    # (+3 stages: GEMM1 172 -> 156 us, GEMM2 100 -> 92 us on the bench layer, profiles/r3/s3/moe/)
    narrow_stage_bytes = (block_M + bn_t) * block_K * (2 if dtype in ("bfloat16", "float16") else 4)
    if tail_stages is None:
        t_stages = max(num_stages, 3) if 3 * narrow_stage_bytes <= 144 * 1024 else num_stages
    else:
        t_stages = tail_stages
    assert tail_ksplit or bn_t % 64 == 0 or bn_t == 32, "tail tiles must stay MFMA / SwiGLU-group aligned"
    accum = "float32"
    a_rows = n_src if n_src is not None else max_rows
    n_out = N // 2 if swiglu else N

    @T.macro
    def tile(A, W, row_src, tile_rows, C, A_s, W_s, C_l, bx_raw, e_raw, col0, bn, stages, A_x=None, C_x=None):
        # tile / expert ids come from device tables: clamp them so the operand copies are provably
        # in bounds (LDS-DMA instead of guarded register staging) and read them once per tile
        bx = T.min(bx_raw, n_tiles - 1)  # expressions, so the bounds prover sees the clamps
        e = T.min(T.max(e_raw, 0), E - 1)
        nrows = T.alloc_var("int32")
        nrows = tile_rows[bx]
        r0 = bx * slot
        T.clear(C_l)
        if ext_M:
            T.clear(C_x)
        for k in T.Pipelined(nk, num_stages=stages):
            if n_src is not None:
                T.gather_rows(A[:, k * block_K:(k + 1) * block_K], row_src[r0:r0 + block_M], A_s, row_dim=0)
                if ext_M:
                    T.gather_rows(A[:, k * block_K:(k + 1) * block_K], row_src[r0 + block_M:r0 + slot], A_x,
                                  row_dim=0)
            else:
                T.copy(A[r0, k * block_K], A_s)
                if ext_M:
                    T.copy(A[r0 + block_M, k * block_K], A_x)
            T.copy(W[e, col0, k * block_K], W_s)
            T.gemm(A_s, W_s, C_l, transpose_B=True, valid_m=nrows if skip_padding else None)
            if ext_M:
                # column-split waves (when the tile is wide enough) all skip the same empty fragments
                T.gemm(A_x, W_s, C_x, transpose_B=True, valid_m=nrows - block_M,
                       policy=T.GemmWarpPolicy.FullCol if bn // 16 >= threads // 64 else T.GemmWarpPolicy.Square)
        if swiglu and staged_epi:
            # activation pairs into a row-padded LDS tile, then row-contiguous 16-byte stores
            A_o = T.alloc_shared((block_M, bn // 2), dtype)
            T.annotate_layout({A_o: PaddedLayout((block_M, bn // 2), 8)})
            for i, j in T.Parallel(block_M, bn):
                if j % 4 < 2:
                    A_o[i, (j // 4) * 2 + j % 4] = T.Cast(dtype, C_l[i, j] / (1.0 + T.exp(-C_l[i, j])) * C_l[i, j + 2])
            T.copy(A_o, C[r0, col0 // 2])
            if ext_M:
                for i, j in T.Parallel(ext_M, bn):
                    if j % 4 < 2:
                        C[r0 + block_M + i, col0 // 2 + (j // 4) * 2 + j % 4] = T.Cast(
                            dtype, C_x[i, j] / (1.0 + T.exp(-C_x[i, j])) * C_x[i, j + 2])
        elif swiglu:
            for i, j in T.Parallel(block_M, bn):
                if j % 4 < 2:
                    C[r0 + i, col0 // 2 + (j // 4) * 2 + j % 4] = T.Cast(
                        dtype, C_l[i, j] / (1.0 + T.exp(-C_l[i, j])) * C_l[i, j + 2])
            if ext_M:
                for i, j in T.Parallel(ext_M, bn):
                    if j % 4 < 2:
                        C[r0 + block_M + i, col0 // 2 + (j // 4) * 2 + j % 4] = T.Cast(
                            dtype, C_x[i, j] / (1.0 + T.exp(-C_x[i, j])) * C_x[i, j + 2])
        elif staged_epi:
            C_s = T.alloc_shared((block_M, bn), dtype)
            T.annotate_layout({C_s: PaddedLayout((block_M, bn), 8)})
            T.copy(C_l, C_s)
            T.copy(C_s, C[r0, col0])
            if ext_M:
                T.copy(C_x, C[r0 + block_M, col0])
        else:
            T.copy(C_l, C[r0, col0])
            if ext_M:
                T.copy(C_x, C[r0 + block_M, col0])

    S_ = max(1, tail_ksplit)
    nks = nk // S_
    assert tail_ksplit == 0 or nk % S_ == 0, "tail_ksplit must divide the K steps"

    @T.macro
    def kchunk(A, W, row_src, A_s, W_s, C_l, bx, e, col0, nrows, kbase):
        T.clear(C_l)
        for k in T.Pipelined(nks, num_stages=num_stages):
            if n_src is not None:
                T.gather_rows(A[:, (kbase + k) * block_K:(kbase + k + 1) * block_K],
                              row_src[bx * block_M:(bx + 1) * block_M], A_s, row_dim=0)
            else:
                T.copy(A[bx * block_M, (kbase + k) * block_K], A_s)
            T.copy(W[e, col0, (kbase + k) * block_K], W_s)
            T.gemm(A_s, W_s, C_l, transpose_B=True, valid_m=nrows if skip_padding else None)

    @T.macro
    def epilogue(C, C_l, bx, col0, bn):
        if swiglu:
            for i, j in T.Parallel(block_M, bn):
                if j % 4 < 2:
                    C[bx * block_M + i, col0 // 2 + (j // 4) * 2 + j % 4] = T.Cast(
                        dtype, C_l[i, j] / (1.0 + T.exp(-C_l[i, j])) * C_l[i, j + 2])
        else:
            T.copy(C_l, C[bx * block_M, col0])

    @T.macro
    def body(A, W, tile_expert, row_src, tile_rows, C, WS, Cnt, pid):
        A_s = T.alloc_shared((block_M, block_K), dtype)
        W_s = T.alloc_shared((block_N, block_K), dtype)
        C_l = T.alloc_fragment((block_M, block_N), accum)
        nt = T.alloc_var("int32")
        nfull = T.alloc_var("int32")
        nt = 0
        nfull = 0
        for t in T.serial(n_tiles):
            if tile_expert[t] >= 0:
                nt = t + 1
                if tile_rows[t] == block_M:
                    nfull = t + 1
        units = nt * n_by
        full = units - units % n_cu
        shift = (nt - nfull) * n_by if partial_first else 0
        for it in T.serial(full // n_cu):  # whole tiles
            u = (pid + it * n_cu + shift) % units
            tile(A, W, row_src, tile_rows, C, A_s, W_s, C_l, u // n_by, tile_expert[u // n_by],
                 (u % n_by) * block_N, block_N, num_stages)
        prev = T.alloc_shared((1, ), "int32")
        for it in T.serial(T.ceildiv((units - full) * S_, n_cu)):  # K-chunks of the tail units
            q = pid + it * n_cu
            if q < (units - full) * S_:
                slot = T.max(T.min(q // S_, n_cu - 1), 0)
                kc = q % S_
                u = (full + q // S_ + shift) % units
                bx = T.min(u // n_by, n_tiles - 1)
                e = T.min(T.max(tile_expert[bx], 0), E - 1)
                col0 = (u % n_by) * block_N
                nrows = T.alloc_var("int32")
                nrows = tile_rows[bx]
                kchunk(A, W, row_src, A_s, W_s, C_l, bx, e, col0, nrows, kc * nks)
                for i, j in T.Parallel(block_M, block_N):  # publish the partial (valid rows)
                    if i < nrows:
                        WS[slot, kc, i, j] = C_l[i, j]
                T.memory_fence()
                T.sync_threads()
                if T.get_thread_binding() == 0:
                    prev[0] = T.atomic_add(Cnt[slot], 1, return_prev=True)
                T.sync_threads()
                if prev[0] == S_ - 1:  # last chunk: sum the others' partials, run the epilogue
                    T.memory_fence()
                    for kc2 in T.serial(S_):
                        if kc2 != kc:
                            for i, j in T.Parallel(block_M, block_N):
                                if i < nrows:
                                    C_l[i, j] += WS[slot, kc2, i, j]
                    epilogue(C, C_l, bx, col0, block_N)
                    if T.get_thread_binding() == 0:
                        Cnt[slot] = 0
                T.sync_threads()

    if tail_ksplit:

        @T.prim_func
        def moe_expert_gemm_tbk(A: T.Tensor((a_rows, K), dtype), W: T.Tensor((E, N, K), dtype),
                                tile_expert: T.Tensor((n_tiles,), "int32"), row_src: T.Tensor((max_rows,), "int32"),
                                tile_rows: T.Tensor((n_tiles,), "int32"), C: T.Tensor((max_rows, n_out), dtype),
                                WS: T.Tensor((n_cu, S_, block_M, block_N), accum), Cnt: T.Tensor((n_cu,), "int32")):
            with T.Kernel(n_cu, threads=threads) as pid:
                body(A, W, tile_expert, row_src, tile_rows, C, WS, Cnt, pid)

        cfg = {"tl.gemm_phased": bool(phased)}
        if swiglu:
            cfg[tilelang.PassConfigKey.TL_ENABLE_FAST_MATH] = True
        return tilelang.compile(moe_expert_gemm_tbk, out_idx=None, target=target, pass_configs=cfg)

    @T.prim_func
    def moe_expert_gemm_tb(A: T.Tensor((a_rows, K), dtype), W: T.Tensor((E, N, K), dtype),
                           tile_expert: T.Tensor((n_tiles,), "int32"), row_src: T.Tensor((max_rows,), "int32"),
                           tile_rows: T.Tensor((n_tiles,), "int32"), C: T.Tensor((max_rows, n_out), dtype)):
        with T.Kernel(n_cu, threads=threads) as pid:
            A_s = T.alloc_shared((block_M, block_K), dtype)
            W_s = T.alloc_shared((block_N, block_K), dtype)
            C_l = T.alloc_fragment((block_M, block_N), accum)
            Wt_s = T.alloc_shared((bn_t, block_K), dtype)
            Ct_l = T.alloc_fragment((block_M, bn_t), accum)
            # the tail loop has operand tiles of its own: every LDS buffer then lives inside one
            # iteration-local loop, so the staging tiles can take the rings' bytes
            At_s = T.alloc_shared((block_M, block_K), dtype) if staged_epi else A_s
            A_x = C_x = Ct_x = At_x = None
            if ext_M:
                A_x = T.alloc_shared((ext_M, block_K), dtype)
                At_x = T.alloc_shared((ext_M, block_K), dtype) if staged_epi else A_x
                C_x = T.alloc_fragment((ext_M, block_N), accum)
                Ct_x = T.alloc_fragment((ext_M, bn_t), accum)
            nt = T.alloc_var("int32")
            nfull = T.alloc_var("int32")
            nt = 0
            nfull = 0
            for t in T.serial(n_tiles):
                if tile_expert[t] >= 0:
                    nt = t + 1
                    if tile_rows[t] >= block_M:
                        nfull = t + 1
            units = nt * n_by
            full = units - units % n_cu
            # unit u -> tile (u + shift) % units: partial tiles first when asked
            shift = (nt - nfull) * n_by if partial_first else 0
            # no LDS value crosses a tile: the operand ring and the C staging tile share bytes
            loc = {"lds_iteration_local": True}
            for it in T.serial(full // n_cu, annotations=loc):  # whole tiles
                u = (pid + it * n_cu + shift) % units
                tile(A, W, row_src, tile_rows, C, A_s, W_s, C_l, u // n_by, tile_expert[u // n_by],
                     (u % n_by) * block_N, block_N, num_stages, A_x, C_x)
            for it in T.serial(T.ceildiv((units - full) * tail_split, n_cu), annotations=loc):  # narrow tail tiles
                q = pid + it * n_cu
                if q < (units - full) * tail_split:
                    u = (full + q // tail_split + shift) % units
                    tile(A, W, row_src, tile_rows, C, At_s, Wt_s, Ct_l, u // n_by, tile_expert[u // n_by],
                         (u % n_by) * block_N + (q % tail_split) * bn_t, bn_t, t_stages, At_x, Ct_x)

    # K-half phased main loop (row gathers included) measured slower here: 382-403 vs 300-356 us per
    # layer (profiles/r2/session2/moe_phased_tail_sweep.log), so off by default
    cfg = {"tl.gemm_phased": bool(phased), "tl.gemm_quad": bool(quad)}
    if swiglu:
        cfg[tilelang.PassConfigKey.TL_ENABLE_FAST_MATH] = True
    return tilelang.compile(moe_expert_gemm_tb, out_idx=None, target=target, pass_configs=cfg)


def swiglu_interleave(w1: torch.Tensor) -> torch.Tensor:
    """``[E, 2F, H]`` (gate rows then up rows) -> the row order of the fused SwiGLU GEMM:
    groups of 4 rows (gate 2p, gate 2p+1, up 2p, up 2p+1)."""
    E, F2, H = w1.shape
    F = F2 // 2
    g = w1[:, :F].reshape(E, F // 2, 2, H)
    u = w1[:, F:].reshape(E, F // 2, 2, H)
    return torch.cat([g, u], 2).reshape(E, F2, H).contiguous()


def _mesh_shape():
    from ..parallel.mesh import get_device_mesh_config
    return get_device_mesh_config()


@functools.lru_cache(maxsize=None)
def silu_mul_kernel(rows: int, F: int, dtype: str, target: str, block_R: int = 32, threads: int = 256):
    """``out[r, j] = silu(H[r, j]) * H[r, F + j]`` (gate | up halves of the first expert GEMM)."""
    block_F = min(F, 256)
    assert F % block_F == 0 and rows % block_R == 0

    @T.prim_func
    def moe_silu_mul(H: T.Tensor((rows, 2 * F), dtype), O: T.Tensor((rows, F), dtype)):
        with T.Kernel(rows // block_R, F // block_F, threads=threads) as (bx, by):
            for i, j in T.Parallel(block_R, block_F):
                g = T.Cast("float32", H[bx * block_R + i, by * block_F + j])
                u = T.Cast("float32", H[bx * block_R + i, F + by * block_F + j])
                O[bx * block_R + i, by * block_F + j] = T.Cast(dtype, g / (1.0 + T.exp(-g)) * u)

    return tilelang.compile(moe_silu_mul, out_idx=None, target=target,
                            pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})


@functools.lru_cache(maxsize=None)
def combine_kernel(n_tok: int, H: int, topk: int, max_rows: int, dtype: str, target: str, block_H: int = 1024,
                   threads: int = 128):
    """``out[t, :] = sum_k w[t, k] * Y[dest[t * topk + k], :]`` (fp32 sum, one pass, no atomics)."""
    block_H = min(block_H, H)
    assert H % block_H == 0

    @T.prim_func
    def moe_combine(Y: T.Tensor((max_rows, H), dtype), dest: T.Tensor((n_tok * topk,), "int32"),
             w: T.Tensor((n_tok, topk), "float32"), out: T.Tensor((n_tok, H), dtype)):
        with T.Kernel(n_tok, H // block_H, threads=threads) as (bx, by):
            acc = T.alloc_fragment((block_H,), "float32")
            T.clear(acc)
            # unrolled over k: every row's index load and its row loads issue before the first
            # accumulate (one memory round trip per phase instead of one per routed row)
            for k in T.unroll(topk):
                r = dest[bx * topk + k]
                wk = w[bx, k]
                for h in T.Parallel(block_H):
                    acc[h] += wk * T.Cast("float32", Y[r, by * block_H + h])
            for h in T.Parallel(block_H):
                out[bx, by * block_H + h] = T.Cast(dtype, acc[h])

    return tilelang.compile(moe_combine, out_idx=None, target=target)


def route(x: torch.Tensor, gate_w: torch.Tensor, topk: int):
    """Router -> top-k ids [T, k] int32 + renormalised weights [T, k].  16-bit activations with
    H % 256 == 0 take the fused MFMA GEMM + top-k kernel; otherwise logits come from
    ``ops.gemm.linear`` (the exact-f32 MFMA GEMM for fp32 routers, K zero-padded for odd widths)
    and ``router_topk_kernel``."""
    n_tok, H = x.shape
    E = gate_w.shape[0]
    if x.dtype in (torch.float16, torch.bfloat16) and H % 256 == 0 and gate_w.dtype == x.dtype and E <= 64:
        ids = torch.empty(n_tok, topk, dtype=torch.int32, device=x.device)
        w = torch.empty(n_tok, topk, dtype=torch.float32, device=x.device)
        sp = ROUTER_SPLITS
        if sp > 1 and H % (sp * 256) == 0 and n_tok % 16 == 0:
            Ep = max(16, -(-E // 16) * 16)
            part = torch.empty(sp, n_tok, Ep, dtype=torch.float32, device=x.device)
            router_logits_sk_kernel(n_tok, H, E, _tdt(x.dtype), _target(x.device), sp)(x.contiguous(),
                                                                                       _padded_gate(gate_w), part)
            router_topk_kernel(n_tok, E, topk, _target(x.device), parts=sp, E_stride=Ep,
                               round_dtype=_tdt(x.dtype))(part, ids, w)
            return ids, w
        kc = 4
        if ROUTER_WIDE and _target(x.device) == "hip" and n_tok % 8 == 0 and H % (kc * 128) == 0 and E <= 16:
            g = _padded_gate(gate_w)
            router_wide_kernel(n_tok, H, E, topk, _tdt(x.dtype), "hip", kc=kc)(
                x.contiguous().view(n_tok * kc, H // kc), g.view(g.shape[0] * kc, H // kc), ids, w)
            return ids, w
        router_fused_kernel(n_tok, H, E, topk, _tdt(x.dtype), _target(x.device))(x.contiguous(), _padded_gate(gate_w),
                                                                                  ids, w)
        return ids, w
    from .gemm import linear
    logits = linear(x, gate_w.to(x.dtype)).float()  # MFMA (exact-f32 form for fp32 routers)
    n_tok, E = logits.shape
    ids = torch.empty(n_tok, topk, dtype=torch.int32, device=x.device)
    w = torch.empty(n_tok, topk, dtype=torch.float32, device=x.device)
    router_topk_kernel(n_tok, E, topk, _target(x.device))(logits, ids, w)
    return ids, w


def dispatch_plan(expert_ids: torch.Tensor, E: int, block_M: int, max_rows: int, div: int = 1,
                  stable: bool = False, even: bool = False):
    """Device-side padded placement: ``(dest[n], row_src[max_rows], tile_expert, counts[E], tile_rows)``.
    ``even``: rows spread evenly over each expert's row tiles (``align_kernel(even=True)``)."""
    dev = expert_ids.device
    n = expert_ids.numel()
    ids = expert_ids.reshape(-1).to(torch.int32).contiguous()
    dest = torch.empty(n, dtype=torch.int32, device=dev)
    row_src = torch.empty(max_rows, dtype=torch.int32, device=dev)
    te = torch.empty(max_rows // block_M, dtype=torch.int32, device=dev)
    counts = torch.empty(E, dtype=torch.int32, device=dev)
    tile_rows = torch.empty(max_rows // block_M, dtype=torch.int32, device=dev)
    align_kernel(n, E, block_M, max_rows, div, _target(dev), stable, even=even)(ids, dest, row_src, te, counts,
                                                                                tile_rows)
    return dest, row_src, te, counts, tile_rows


def pack_by_expert(expert_ids: torch.Tensor, E: int, block_M: int, max_rows: int):
    """``(dest[n], tile_expert[max_rows // block_M], counts[E])`` (see ``dispatch_plan``)."""
    dest, _, te, counts, _ = dispatch_plan(expert_ids, E, block_M, max_rows, stable=True)
    return dest.long(), te, counts.long()


_TAIL_WS = {}


def _tail_workspace(dev, n_cu, S, block_M, block_N):
    """fp32 partial-sum slots + arrival counters of the K-split tail (expert_gemm_sk_kernel);
    the counters are reset by the last arriver, so one zeroed allocation serves every call."""
    key = (str(dev), n_cu, S, block_M, block_N)
    if key not in _TAIL_WS:
        _TAIL_WS[key] = (torch.empty(n_cu, S, block_M, block_N, dtype=torch.float32, device=dev),
                         torch.zeros(n_cu, dtype=torch.int32, device=dev))
    return _TAIL_WS[key]


def expert_ffn_padded(src_rows: torch.Tensor, expert_ids: torch.Tensor, div: int, w1: torch.Tensor,
                      w2: torch.Tensor, block_M: int = 128, reduce_mesh: Optional[str] = None,
                      cfg: Optional[dict] = None, w1_interleaved: bool = False):
    """SwiGLU experts for the assignments ``expert_ids[n]`` (assignment j reads ``src_rows[j // div]``).
    Returns ``(Y [max_rows, H], dest [n])``: assignment j's result is row ``dest[j]`` of Y.
    ``w1_interleaved``: ``w1`` is in ``swiglu_interleave`` row order (fused activation)."""
    cfg = dict(cfg or {})
    E, F2, H = w1.shape
    F = F2 // 2
    n = expert_ids.numel()
    dev = src_rows.device
    tgt = _tdt(src_rows.dtype)
    target = _target(dev)
    sk = cfg.pop("stream_k", None)
    n_cu = cfg.pop("n_cu", 256)
    if sk is None:
        sk = target == "hip"
    sk = sk and reduce_mesh is None and w1_interleaved
    ext = cfg.pop("ext_M", 0) if sk else 0
    cfg.pop("ext_M", None)
    slot = block_M + ext
    max_rows = max_padded_rows(_bucket(n), E, slot)
    n_src = _bucket(src_rows.shape[0])
    if src_rows.shape[0] != n_src:
        src_rows = torch.cat([src_rows, src_rows.new_zeros(n_src - src_rows.shape[0], src_rows.shape[1])])
    dest, row_src, te, _, trows = dispatch_plan(expert_ids, E, slot, max_rows, div, stable=reduce_mesh is not None,
                                                even=ext > 0)
    act = torch.empty(max_rows, F, dtype=src_rows.dtype, device=dev)
    if sk:
        # tail-balanced grid: whole tiles for the leading rounds, narrow tiles for the trailing partial round
        skc = {k: v for k, v in cfg.items() if k in ("block_N", "block_K", "num_stages", "threads", "tail_split",
                                                      "phased", "skip_padding", "tail_ksplit", "tail_stages", "quad")}
        # partial_first for the down projection: measured neutral (profiles/r3/s3/moe/), off
        pf2 = cfg.get("partial_first2", False)
        ws = ()
        if skc.get("tail_ksplit"):
            ws = _tail_workspace(dev, n_cu, skc["tail_ksplit"], block_M, skc.get("block_N", 256))
        k1 = expert_gemm_sk_kernel(max_rows, H, F2, E, tgt, target, block_M, n_src=n_src, swiglu=True, n_cu=n_cu,
                                   ext_M=ext, **skc)
        k1(src_rows.contiguous(), w1, te, row_src, trows, act, *ws)
        k2 = expert_gemm_sk_kernel(max_rows, F, H, E, tgt, target, block_M, n_cu=n_cu, partial_first=pf2,
                                   ext_M=ext, **skc)
        y = torch.empty(max_rows, H, dtype=src_rows.dtype, device=dev)
        k2(act, w2, te, row_src, trows, y, *ws)
        return y, dest
    for key in ("tail_split", "phased", "partial_first2", "tail_ksplit", "tail_stages", "quad"):  # tail-balanced only
        cfg.pop(key, None)
    if w1_interleaved:
        # gate/up rows interleaved: the activation is the first GEMM's epilogue
        k1 = expert_gemm_kernel(max_rows, H, F2, E, tgt, target, block_M, n_src=n_src, swiglu=True, **cfg)
        k1(src_rows.contiguous(), w1, te, row_src, trows, act)
    else:
        k1 = expert_gemm_kernel(max_rows, H, F2, E, tgt, target, block_M, n_src=n_src, **cfg)
        h = torch.empty(max_rows, F2, dtype=src_rows.dtype, device=dev)
        k1(src_rows.contiguous(), w1, te, row_src, trows, h)
        silu_mul_kernel(max_rows, F, tgt, target)(h, act)
    k2 = expert_gemm_kernel(max_rows, F, H, E, tgt, target, block_M, reduce_mesh=reduce_mesh,
                            mesh_shape=_mesh_shape() if reduce_mesh else None, **cfg)
    y = torch.empty(max_rows, H, dtype=src_rows.dtype, device=dev)
    k2(act, w2, te, row_src, trows, y)
    return y, dest


def expert_ffn(x_rows: torch.Tensor, expert_ids: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor,
               block_M: int = 128, reduce_mesh: Optional[str] = None, cfg: Optional[dict] = None) -> torch.Tensor:
    """SwiGLU experts on already-dispatched rows: ``y_i = W2[e_i] (silu(g) * u)``, with
    ``[g | u] = W1[e_i] x_i``.  ``w1``: ``[E, 2F, H]``, ``w2``: ``[E, H, F]``."""
    y, dest = expert_ffn_padded(x_rows, expert_ids, 1, w1, w2, block_M, reduce_mesh, cfg)
    return y[dest.long()]


def combine(y: torch.Tensor, dest: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``out[t] = sum_k w[t, k] * y[dest[t * topk + k]]``."""
    n_tok, topk = w.shape
    H = y.shape[1]
    bh = 1024 if H % 1024 == 0 else H
    out = torch.empty(n_tok, H, dtype=y.dtype, device=y.device)
    combine_kernel(n_tok, H, topk, y.shape[0], _tdt(y.dtype), _target(y.device), block_H=bh)(
        y, dest.to(torch.int32).contiguous(), w.float().contiguous(), out)
    return out
