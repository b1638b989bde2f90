"""Native Sparse Attention selected-block attention, backward
(reference: examples/deepseek_nsa/example_tilelang_nsa_bwd.py).  Forward: example_nsa_fwd.py.

Per (token t, kv head h) the G query heads attend to the selected key blocks; with the forward's
log-sum-exp L (log2 domain) and delta = rowsum(O * dO):

    P  = exp2(s * scale - L),   dP = dO V^T,   dS = P * (dP - delta)
    dQ = sm_scale dS K,   dK = sm_scale dS^T Q,   dV = P^T dO

Kernels (MI355X):
  nsa_fwd_lse     the forward, also writing L [B, SQ, HQ] (fp32)
  nsa_bwd_prep    delta
  nsa_block_mask  Mask[b, h, j, t] = 1 when token t selected key block j (inverse of BlockIndices)
  token_lists     the same inverse as compacted, padded token lists per (batch, kv head, block)
  nsa_bwd_dq      one workgroup per (token, kv head) walks its selected blocks (like the forward):
                  dQ is produced whole, no atomics
  nsa_bwd_dkv     one workgroup per (key block, kv head, batch) keeps K_j, V_j and the dK/dV
                  accumulators resident and walks ONLY the tokens that selected the block (its
                  token list), ``64 / G`` tokens per tile (G * tokens = 64 MFMA rows): Q / dO rows
                  arrive by LDS-DMA row gathers in a pipelined loop.  dK/dV are produced whole.
"""
import argparse

import tilelang
import tilelang.language as T

from example_nsa_fwd import FAST_MATH, LOG2E


@tilelang.jit(out_idx=[-2, -1], pass_configs=FAST_MATH)
def nsa_fwd_lse(batch, heads, seq_len, seq_len_kv, dim, is_causal=True, scale=None, block_size=64, groups=16,
                selected_blocks=16, num_stages=2, block_T=32, dtype="bfloat16"):
    sm = (1.0 / dim)**0.5 if scale is None else scale
    scale = sm * LOG2E
    head_kv = heads // groups
    G, BS, S, D = groups, block_size, selected_blocks, dim
    BT = min(block_T, BS)
    NT = BS // BT
    assert G % 16 == 0
    threads = 64 * (G // 16)
    past = seq_len_kv - seq_len
    accum_dtype = "float"

    @T.prim_func
    def main(Q: T.Tensor([batch, seq_len, heads, D], dtype), K: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             V: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             BlockIndices: T.Tensor([batch, seq_len, head_kv, S], "int32"),
             Output: T.Tensor([batch, seq_len, heads, D], dtype), LSE: T.Tensor([batch, seq_len, heads], "float32")):
        with T.Kernel(seq_len, batch * head_kv, threads=threads) as (bx, bz):
            Q_shared = T.alloc_shared([G, D], dtype)
            K_shared = T.alloc_shared([BT, D], dtype)
            V_shared = T.alloc_shared([BT, D], dtype)
            acc_s = T.alloc_fragment([G, BT], accum_dtype)
            acc_s_cast = T.alloc_fragment([G, BT], dtype)
            acc_o = T.alloc_fragment([G, D], accum_dtype)
            o_cast = T.alloc_fragment([G, D], dtype)
            m = T.alloc_fragment([G], accum_dtype)
            m_prev = T.alloc_fragment([G], accum_dtype)
            alpha = T.alloc_fragment([G], accum_dtype)
            l_sum = T.alloc_fragment([G], accum_dtype)
            r_sum = T.alloc_fragment([G], accum_dtype)
            b = bz // head_kv
            h = bz % head_kv
            pos = bx + past
            T.copy(Q[b, bx, h * G:(h + 1) * G, :], Q_shared)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            for i in T.Pipelined(S * NT, num_stages=num_stages):
                blk = BlockIndices[b, bx, h, i // NT]
                i_s = T.min(T.max(blk, 0), seq_len_kv // BS - 1) * BS + (i % NT) * BT
                T.copy(K[b, i_s:i_s + BT, h, :], K_shared)
                T.copy(V[b, i_s:i_s + BT, h, :], V_shared)
                for g, j in T.Parallel(G, BT):
                    ok = (blk >= 0) & (blk * BS <= pos)
                    if is_causal:
                        ok = ok & (i_s + j <= pos)
                    acc_s[g, j] = T.if_then_else(ok, 0, -T.infinity(accum_dtype))
                T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(m, m_prev)
                T.reduce_max(acc_s, m, dim=1, clear=False)
                for g in T.Parallel(G):
                    alpha[g] = T.exp2((m_prev[g] - m[g]) * scale)
                for g, j in T.Parallel(G, BT):
                    acc_s[g, j] = T.exp2(acc_s[g, j] * scale - m[g] * scale)
                T.reduce_sum(acc_s, r_sum, dim=1)
                for g in T.Parallel(G):
                    l_sum[g] = l_sum[g] * alpha[g] + r_sum[g]
                for g, d in T.Parallel(G, D):
                    acc_o[g, d] *= alpha[g]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for g, d in T.Parallel(G, D):
                o_cast[g, d] = acc_o[g, d] / T.max(l_sum[g], 1e-30)
            T.copy(o_cast, Output[b, bx, h * G:(h + 1) * G, :])
            for g in T.Parallel(G):
                # rows with no visible key: +inf, so the backward's P is exactly 0 there
                LSE[b, bx, h * G + g] = T.if_then_else(l_sum[g] > 0, m[g] * scale + T.log2(l_sum[g]),
                                                       T.infinity("float32"))

    return main


@tilelang.jit(out_idx=[2])
def nsa_bwd_prep(batch, seq_len, heads, dim, dtype="bfloat16", block_R=64, threads=256):
    """Delta = rowsum(O * dO) over the B*SQ*HQ rows of the flattened [rows, dim] views (one HBM
    pass; ``block_R`` rows per workgroup keep the fp32 products at 32 registers per lane)."""
    rows = batch * seq_len * heads

    @T.prim_func
    def main(O: T.Tensor([rows, dim], dtype), dO: T.Tensor([rows, dim], dtype), Delta: T.Tensor([rows], "float32")):
        with T.Kernel(T.ceildiv(rows, block_R), threads=threads) as bx:
            o = T.alloc_fragment([block_R, dim], dtype)
            do = T.alloc_fragment([block_R, dim], dtype)
            acc = T.alloc_fragment([block_R, dim], "float32")
            dsum = T.alloc_fragment([block_R], "float32")
            T.copy(O[bx * block_R:(bx + 1) * block_R, :], o)
            T.copy(dO[bx * block_R:(bx + 1) * block_R, :], do)
            for r, d in T.Parallel(block_R, dim):
                acc[r, d] = T.cast(o[r, d], "float32") * T.cast(do[r, d], "float32")
            T.reduce_sum(acc, dsum, dim=1)
            T.copy(dsum, Delta[bx * block_R:(bx + 1) * block_R])

    return main


@tilelang.jit(out_idx=[1])
def nsa_block_mask(batch, seq_len, head_kv, selected_blocks, num_blocks):

    @T.prim_func
    def main(BlockIndices: T.Tensor([batch, seq_len, head_kv, selected_blocks], "int32"),
             Mask: T.Tensor([batch, head_kv, num_blocks, seq_len], "int8")):
        with T.Kernel(T.ceildiv(seq_len, 64), batch * head_kv, threads=64) as (bx, bz):
            b, h = bz // head_kv, bz % head_kv
            for t in T.Parallel(64):
                tt = bx * 64 + t
                if tt < seq_len:
                    for j in T.serial(num_blocks):
                        Mask[b, h, j, tt] = 0
                    for i in T.serial(selected_blocks):
                        blk = BlockIndices[b, tt, h, i]
                        if blk >= 0 and blk < num_blocks:
                            Mask[b, h, blk, tt] = 1

    return main


@tilelang.jit(out_idx=[-1], pass_configs=FAST_MATH)
def nsa_bwd_dq(batch, heads, seq_len, seq_len_kv, dim, is_causal=True, scale=None, block_size=64, groups=16,
               selected_blocks=16, block_T=64, dtype="bfloat16", threads=None):
    """One workgroup per (token, kv head).  The G x BT score tile and the G x D dQ tile are split
    over ``threads // 64`` waves along their columns (default 4 waves for G=16), so a token's
    16 x 1024 x 128 chain of small GEMMs runs on four SIMDs instead of one."""
    sm = (1.0 / dim)**0.5 if scale is None else scale
    scale = sm * LOG2E
    head_kv = heads // groups
    G, BS, S, D = groups, block_size, selected_blocks, dim
    BT = min(block_T, BS)
    NT = BS // BT
    if threads is None:
        threads = 64 * max(1, min(4, BT // 16))
    pol = T.GemmWarpPolicy.FullRow if threads == 64 * (G // 16) else T.GemmWarpPolicy.FullCol
    past = seq_len_kv - seq_len
    accum_dtype = "float"

    @T.prim_func
    def main(Q: T.Tensor([batch, seq_len, heads, D], dtype), K: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             V: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             BlockIndices: T.Tensor([batch, seq_len, head_kv, S], "int32"),
             dO: T.Tensor([batch, seq_len, heads, D], dtype), LSE: T.Tensor([batch, seq_len, heads], "float32"),
             Delta: T.Tensor([batch, seq_len, heads], "float32"), dQ: T.Tensor([batch, seq_len, heads, D], dtype)):
        with T.Kernel(seq_len, batch * head_kv, threads=threads) as (bx, bz):
            q_s = T.alloc_shared([G, D], dtype)
            do_s = T.alloc_shared([G, D], dtype)
            k_s = T.alloc_shared([BT, D], dtype)
            v_s = T.alloc_shared([BT, D], dtype)
            ds_s = T.alloc_shared([G, BT], dtype)
            lse_s = T.alloc_shared([G], "float32")
            dl_s = T.alloc_shared([G], "float32")
            s = T.alloc_fragment([G, BT], accum_dtype)
            dp = T.alloc_fragment([G, BT], accum_dtype)
            dq = T.alloc_fragment([G, D], accum_dtype)
            b = bz // head_kv
            h = bz % head_kv
            pos = bx + past
            T.copy(Q[b, bx, h * G:(h + 1) * G, :], q_s)
            T.copy(dO[b, bx, h * G:(h + 1) * G, :], do_s)
            T.copy(LSE[b, bx, h * G:(h + 1) * G], lse_s)
            T.copy(Delta[b, bx, h * G:(h + 1) * G], dl_s)
            T.clear(dq)
            for i in T.Pipelined(S * NT, num_stages=2):
                blk = BlockIndices[b, bx, h, i // NT]
                i_s = T.min(T.max(blk, 0), seq_len_kv // BS - 1) * BS + (i % NT) * BT
                T.copy(K[b, i_s:i_s + BT, h, :], k_s)
                T.copy(V[b, i_s:i_s + BT, h, :], v_s)
                T.clear(s)
                T.gemm(q_s, k_s, s, transpose_B=True, policy=pol)
                T.clear(dp)
                T.gemm(do_s, v_s, dp, transpose_B=True, policy=pol)
                for g, j in T.Parallel(G, BT):
                    ok = (blk >= 0) & (blk * BS <= pos)
                    if is_causal:
                        ok = ok & (i_s + j <= pos)
                    # the mask selects the exponent (exp2(-inf) = 0): no per-element branch around the exp
                    p = T.exp2(T.if_then_else(ok, s[g, j] * scale - lse_s[g], -T.infinity("float32")))
                    ds_s[g, j] = p * (dp[g, j] - dl_s[g]) * sm
                T.gemm(ds_s, k_s, dq, policy=pol)
            T.copy(dq, dQ[b, bx, h * G:(h + 1) * G, :])

    return main


def _list_bounds(batch, seq_len, head_kv, selected_blocks, num_blocks, tokens_per_tile, chunk_tiles):
    """Static upper bounds of the token-list buffers (so the kernels never recompile as the
    selection changes): pairs incl. per-list padding, tiles, and work items (chunks)."""
    n_lists = batch * head_kv * num_blocks
    pairs = batch * seq_len * head_kv * selected_blocks
    p_max = pairs + n_lists * (tokens_per_tile - 1)
    t_max = p_max // tokens_per_tile
    i_max = -(-t_max // chunk_tiles) + n_lists
    return p_max, i_max


@tilelang.jit(pass_configs=FAST_MATH)  # dK / dV: caller-zeroed fp32 accumulators (atomics)
def nsa_bwd_dkv(batch, heads, seq_len, seq_len_kv, dim, selected_blocks, is_causal=True, scale=None, block_size=64,
                groups=16, tokens_per_tile=4, chunk_tiles=32, threads=256, num_stages=2, dtype="bfloat16"):
    """dK/dV over the compacted (block -> selecting tokens) lists built by ``token_lists``.

    Work item = (key block j of one kv head and batch, a chunk of <= ``chunk_tiles`` tiles of its
    token list): early key blocks are selected by far more tokens than late ones (causal
    selection), so whole lists per workgroup left the grid waiting on block 0's list; chunks keep
    every item about the same size.  An item keeps K_j / V_j in LDS, walks only tokens that
    selected j, ``tokens_per_tile`` at a time (R = tokens * G query-head rows): Q / dO rows are
    gathered by LDS-DMA (``T.gather_rows`` over the flattened [B*SQ*HQ, D] views; pad entries are
    -1 -> zero rows), LSE / Delta come pre-gathered, and the partial dK / dV are added into fp32
    accumulators with atomics (one 64 x 128 tile per item)."""
    sm = (1.0 / dim)**0.5 if scale is None else scale
    scale = sm * LOG2E
    head_kv = heads // groups
    G, BS, D, TT = groups, block_size, dim, tokens_per_tile
    R = TT * G
    NB = seq_len_kv // BS
    past = seq_len_kv - seq_len
    rows = batch * seq_len * heads
    p_max, i_max = _list_bounds(batch, seq_len, head_kv, selected_blocks, NB, TT, chunk_tiles)
    accum_dtype = "float"

    @T.prim_func
    def main(Q: T.Tensor([rows, D], dtype), K: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             V: T.Tensor([batch, seq_len_kv, head_kv, D], dtype), dO: T.Tensor([rows, D], dtype),
             RowIdx: T.Tensor([p_max * G], "int32"), TokP: T.Tensor([p_max], "int32"),
             LseP: T.Tensor([p_max * G], "float32"), DeltaP: T.Tensor([p_max * G], "float32"),
             ItemList: T.Tensor([i_max], "int32"), ItemPair0: T.Tensor([i_max], "int32"),
             ItemTiles: T.Tensor([i_max], "int32"),
             dK: T.Tensor([batch, seq_len_kv, head_kv, D], accum_dtype),
             dV: T.Tensor([batch, seq_len_kv, head_kv, D], accum_dtype)):
        with T.Kernel(i_max, threads=threads) as item:
            k_s = T.alloc_shared([BS, D], dtype)
            v_s = T.alloc_shared([BS, D], dtype)
            q_s = T.alloc_shared([R, D], dtype)
            do_s = T.alloc_shared([R, D], dtype)
            p_s = T.alloc_shared([R, BS], dtype)
            ds_s = T.alloc_shared([R, BS], dtype)
            lse_s = T.alloc_shared([R], "float32")
            dl_s = T.alloc_shared([R], "float32")
            tok_s = T.alloc_shared([TT], "int32")
            s = T.alloc_fragment([R, BS], accum_dtype)
            dp = T.alloc_fragment([R, BS], accum_dtype)
            dk = T.alloc_fragment([BS, D], accum_dtype)
            dv = T.alloc_fragment([BS, D], accum_dtype)
            lst = ItemList[item]
            if lst >= 0:
                # list id -> (batch, kv head, block), clamped for the bounds prover
                j = T.max(T.min(lst % NB, NB - 1), 0)
                h = T.max(T.min((lst // NB) % head_kv, head_kv - 1), 0)
                b = T.max(T.min(lst // (NB * head_kv), batch - 1), 0)
                p0 = ItemPair0[item]
                T.copy(K[b, j * BS:(j + 1) * BS, h, :], k_s)
                T.copy(V[b, j * BS:(j + 1) * BS, h, :], v_s)
                T.clear(dk)
                T.clear(dv)
                for it in T.Pipelined(ItemTiles[item], num_stages=num_stages):
                    base = p0 + it * TT
                    T.gather_rows(Q[:, :], RowIdx[base * G:base * G + R], q_s, row_dim=0)
                    T.gather_rows(dO[:, :], RowIdx[base * G:base * G + R], do_s, row_dim=0)
                    T.copy(LseP[base * G:base * G + R], lse_s)
                    T.copy(DeltaP[base * G:base * G + R], dl_s)
                    T.copy(TokP[base:base + TT], tok_s)
                    T.clear(s)
                    T.gemm(q_s, k_s, s, transpose_B=True)
                    T.clear(dp)
                    T.gemm(do_s, v_s, dp, transpose_B=True)
                    for r, c in T.Parallel(R, BS):
                        ok = tok_s[r // G] >= 0
                        if is_causal:
                            ok = ok & (j * BS + c <= tok_s[r // G] + past)
                        p = T.exp2(T.if_then_else(ok, s[r, c] * scale - lse_s[r], -T.infinity("float32")))
                        p_s[r, c] = p
                        ds_s[r, c] = p * (dp[r, c] - dl_s[r]) * sm
                    T.gemm(p_s, do_s, dv, transpose_A=True)
                    T.gemm(ds_s, q_s, dk, transpose_A=True)
                T.atomic_add(dK[b, j * BS:(j + 1) * BS, h, :], dk)
                T.atomic_add(dV[b, j * BS:(j + 1) * BS, h, :], dv)

    return main


def token_lists(block_indices, lse, delta, num_blocks, heads, tokens_per_tile=4, chunk_tiles=32):
    """Invert BlockIndices [B, SQ, H, S] into per-(batch, kv head, block) lists of the tokens that
    selected the block (on the device: torch sort + scatters, no host sync), each list padded to a
    multiple of ``tokens_per_tile`` with -1 entries, and cut into work items of <= ``chunk_tiles``
    tiles.  Buffers have the static sizes of ``_list_bounds``.  Returns (RowIdx, TokP, LseP, DeltaP,
    ItemList, ItemPair0, ItemTiles): the flattened Q row of every (pair, query head in the group),
    the token of every pair, the LSE / Delta of every row, and per work item its list id (-1:
    unused), first pair and tile count."""
    import torch
    B, SQ, H, S = block_indices.shape
    G = heads // H
    TT, CH = tokens_per_tile, chunk_tiles
    dev = block_indices.device
    nl = B * H * num_blocks
    p_max, i_max = _list_bounds(B, SQ, H, S, num_blocks, TT, CH)
    blk = block_indices.long()
    bb = torch.arange(B, device=dev).view(B, 1, 1, 1).expand_as(blk)
    tt = torch.arange(SQ, device=dev).view(1, SQ, 1, 1).expand_as(blk)
    hh = torch.arange(H, device=dev).view(1, 1, H, 1).expand_as(blk)
    ok = (blk >= 0) & (blk < num_blocks)
    # invalid pairs sort to the end under key nl (dropped by the bincount range below)
    key = torch.where(ok, (bb * H + hh) * num_blocks + blk, torch.full_like(blk, nl)).reshape(-1)
    tok = tt.reshape(-1)
    order = torch.argsort(key * SQ + tok)
    key, tok = key[order], tok[order]
    cnt = torch.bincount(key, minlength=nl + 1)[:nl]
    tiles = (cnt + TT - 1) // TT
    off = torch.zeros(nl + 1, dtype=torch.long, device=dev)
    off[1:] = torch.cumsum(tiles * TT, 0)
    start = torch.zeros(nl + 1, dtype=torch.long, device=dev)
    start[1:] = torch.cumsum(cnt, 0)
    valid = key < nl
    kv_ = torch.where(valid, key, torch.zeros_like(key))
    rank = torch.arange(key.numel(), device=dev) - start[kv_]
    dest = torch.where(valid, off[kv_] + rank, torch.full_like(key, p_max))  # p_max: a dump slot
    tokp = torch.full((p_max + 1, ), -1, dtype=torch.int32, device=dev)
    tokp[dest] = torch.where(valid, tok, torch.full_like(tok, -1)).int()
    b_of = kv_ // (H * num_blocks)
    h_of = (kv_ // num_blocks) % H
    g = torch.arange(G, device=dev)
    rows = ((b_of * SQ + tok) * (H * G) + h_of * G).view(-1, 1) + g.view(1, -1)  # [pairs, G]
    rowidx = torch.full((p_max + 1, G), -1, dtype=torch.int32, device=dev)
    rowidx[dest] = torch.where(valid.view(-1, 1), rows, torch.full_like(rows, -1)).int()
    lsep = torch.zeros((p_max + 1, G), dtype=torch.float32, device=dev)
    dlp = torch.zeros((p_max + 1, G), dtype=torch.float32, device=dev)
    lsep[dest] = lse.reshape(-1)[rows]
    dlp[dest] = delta.reshape(-1)[rows]
    # work items: list l contributes ceil(tiles_l / CH) chunks
    nchunk = (tiles + CH - 1) // CH
    ilist = torch.repeat_interleave(torch.arange(nl, device=dev), nchunk)
    cstart = torch.zeros(nl + 1, dtype=torch.long, device=dev)
    cstart[1:] = torch.cumsum(nchunk, 0)
    ci = torch.arange(ilist.numel(), device=dev) - cstart[ilist]
    item_list = torch.full((i_max, ), -1, dtype=torch.int32, device=dev)
    item_p0 = torch.zeros((i_max, ), dtype=torch.int32, device=dev)
    item_nt = torch.zeros((i_max, ), dtype=torch.int32, device=dev)
    n_items = ilist.numel()  # <= i_max by construction
    item_list[:n_items] = ilist.int()
    item_p0[:n_items] = (off[ilist] + ci * CH * TT).int()
    item_nt[:n_items] = torch.minimum(tiles[ilist] - ci * CH, torch.full_like(ci, CH)).int()
    return (rowidx[:p_max].reshape(-1), tokp[:p_max], lsep[:p_max].reshape(-1), dlp[:p_max].reshape(-1), item_list,
            item_p0, item_nt)


def nsa_backward(q, k, v, block_indices, o, lse, do, block_size=64, is_causal=True):
    """(dq, dk, dv) of the NSA selected-block attention."""
    import torch
    B, SQ, HQ, D = q.shape
    SKV, H = k.shape[1], k.shape[2]
    S = block_indices.shape[-1]
    G = HQ // H
    delta = nsa_bwd_prep(B, SQ, HQ, D, _dt(q))(o.reshape(-1, D), do.reshape(-1, D)).view(B, SQ, HQ)
    dq = nsa_bwd_dq(B, HQ, SQ, SKV, D, is_causal, None, block_size, G, S, dtype=_dt(q), **DQ_CFG)(
        q, k, v, block_indices, do, lse, delta)
    TT, CH = max(1, 64 // G), 32
    lists = token_lists(block_indices, lse, delta, SKV // block_size, HQ, TT, CH)
    dk32 = torch.zeros(k.shape, dtype=torch.float32, device=k.device)
    dv32 = torch.zeros(v.shape, dtype=torch.float32, device=v.device)
    nsa_bwd_dkv(B, HQ, SQ, SKV, D, S, is_causal, None, block_size, G, TT, CH, dtype=_dt(q))(
        q.reshape(-1, D), k, v, do.reshape(-1, D), *lists, dk32, dv32)
    return dq, dk32.to(k.dtype), dv32.to(v.dtype)


DQ_CFG = {}  # nsa_bwd_dq tile overrides (block_T, threads) for A/B runs


def _dt(t):
    return str(t.dtype).replace("torch.", "")


class NativeSparseAttention:
    """``NativeSparseAttention.apply(q, k, v, block_indices, block_size)`` -> o, differentiable."""

    @staticmethod
    def apply(q, k, v, block_indices, block_size=64, is_causal=True):
        import torch

        class _Fn(torch.autograd.Function):

            @staticmethod
            def forward(ctx, q, k, v):
                B, SQ, HQ, D = q.shape
                fwd = nsa_fwd_lse(B, HQ, SQ, k.shape[1], D, is_causal, None, block_size, HQ // k.shape[2],
                                  block_indices.shape[-1], dtype=_dt(q))
                o, lse = fwd(q, k, v, block_indices)
                ctx.save_for_backward(q, k, v, o, lse)
                return o

            @staticmethod
            def backward(ctx, do):
                q, k, v, o, lse = ctx.saved_tensors
                return nsa_backward(q, k, v, block_indices, o, lse, do.contiguous().to(q.dtype), block_size,
                                    is_causal)

        return _Fn.apply(q, k, v)


def ref_attention(q, k, v, block_indices, block_size, scale=None, is_causal=True):
    """Differentiable fp32 reference (dense masked softmax over the selected tokens)."""
    import torch
    B, SQ, HQ, D = q.shape
    SKV, H = k.shape[1], k.shape[2]
    G = HQ // H
    scale = D**-0.5 if scale is None else scale
    past = SKV - SQ
    bi = block_indices.long().cpu()
    allowed = torch.zeros(B, SQ, H, SKV, dtype=torch.bool)
    tok = torch.arange(SKV)
    for s in range(bi.shape[-1]):
        blk = bi[..., s]
        inblk = (tok // block_size)[None, None, None, :] == blk[..., None]
        allowed |= inblk & (blk[..., None] >= 0)
    pos = (torch.arange(SQ) + past)[None, :, None, None]
    allowed &= (tok[None, None, None, :] // block_size) * block_size <= pos
    if is_causal:
        allowed &= tok[None, None, None, :] <= pos
    qf = q.float().cpu().view(B, SQ, H, G, D)
    kf, vf = k.float().cpu(), v.float().cpu()
    s = torch.einsum("bthgd,bshd->bthgs", qf, kf) * scale
    s = s.masked_fill(~allowed[:, :, :, None, :], float("-inf"))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    o = torch.einsum("bthgs,bshd->bthgd", p, vf)
    return o.reshape(B, SQ, HQ, D)


def main(B=2, SQ=4096, SKV=4096, HQ=64, H=4, D=128, S=16, block_size=64):
    import torch
    q = torch.randn(B, SQ, HQ, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, SKV, H, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, SKV, H, D, device="cuda", dtype=torch.bfloat16)
    g = torch.Generator(device="cuda").manual_seed(0)
    nb = SKV // block_size
    vis = (torch.arange(SQ, device="cuda")[:, None] + SKV - SQ) // block_size >= torch.arange(nb, device="cuda")
    r = torch.where(vis[None, :, None, :], torch.rand(B, SQ, H, nb, device="cuda", generator=g), -1.0)
    top = r.topk(min(S, nb), -1)
    bi = torch.where(top.values >= 0, top.indices, -1).int().sort(-1)[0].contiguous()
    fwd = nsa_fwd_lse(B, HQ, SQ, SKV, D, True, None, block_size, HQ // H, S)
    o, lse = fwd(q, k, v, bi)
    do = torch.randn_like(o)
    from tilelang.profiler import do_bench
    nsa_backward(q, k, v, bi, o, lse, do, block_size)
    lat = do_bench(lambda: nsa_backward(q, k, v, bi, o, lse, do, block_size))
    flops = 2.5 * 4 * B * SQ * HQ * D * S * block_size
    print(f"NSA bwd B{B} SQ{SQ} HQ{HQ} H{H} D{D} S{S}x{block_size}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=2)
    p.add_argument("--seq", type=int, default=4096)
    a = p.parse_args()
    main(B=a.batch, SQ=a.seq, SKV=a.seq)
