"""Mamba-2 SSD chunk scan forward (reference: examples/linear_attention/example_mamba_chunk_scan.py,
benchmark/mamba2/benchmark_mamba_chunk_scan.py; reference headline 126-136 TFLOPS on H800 for
b8 h80 chunk 256 headdim 64 dstate 128).

out[c, l] = exp(dA_l) * C_l . prev_state_c                                   (inter-chunk)
          + sum_{s<=l} cb[l, s] * exp(dA_l - dA_s) * dt_s * x_s              (intra-chunk)
          + D * x_l
Block = (head, (m-tile, n-tile), batch*chunk).  The decay-weighted, causally masked CB tile is
built in registers in the MFMA A-operand layout and fed straight to the x-tile MFMA (no LDS
round trip); the per-column dA/dt slices ride the same LDS-DMA pipeline as the CB and x tiles
(no register loads from HBM inside the loop); the decays use exp2 with log2(e) folded in.
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(out_idx=[7], pass_configs=FAST_MATH)
def chunk_scan_fwd(batch, seqlen, chunk_size, ngroups, nheads, headdim, dstate, block_M=128, block_N=64,
                   block_K=64, num_stages=2, threads=256, dtype="float16", xcd_group=False, lean=False,
                   factored=False, xscale=False, ds_blk=None, mask_split=True, heavy_first=False):
    """``factored``: the decay ``exp(a_i - b_j)`` (a = row, b = key cumulative dA) of every
    (row, key) element as ``exp(a_i - c) * exp(c - b_j)`` with ``c`` the key window's last (smallest)
    ``b``: one exp per row and one per key per K step instead of one per element (the kernel is
    VALU-bound and the exponential issues at a quarter of the VALU rate).  Needs ``dA_cumsum``
    non-increasing inside a chunk (Mamba-2: ``A < 0``, ``dt > 0``): then ``exp(c - b_j) <= 1`` never
    overflows, and where ``exp(a_i - c)`` underflows the exact product is below fp32 range too.
    Rows inside the key window have ``a_i - c`` up to the window's span: a K step whose span is
    not far below fp32's range (2^96) takes the per-element exp instead (uniform branch).
``lean``: the intra-chunk loop split into the tiles wholly below the causal diagonal (no
    mask: no index compare / select per element) and the diagonal tiles, with the row decays in
    log2 units precomputed once -- the kernel is VALU-bound (PMC: 20x more VALU than MFMA
    instructions), this trims the per-element decay arithmetic.
    ``xscale``: the key tiles wholly below the row tile (every key precedes every row) take the
    decay off the per-element path: with ``c`` the cumulative dA of the last key before the row tile,
    ``exp(a_i - b_j) = exp(a_i - c) * exp(c - b_j)`` and both factors are <= 1 (dA_cumsum is
    non-increasing), so the key factor (times dt_j) scales the x tile's rows in LDS (block_K x
    headdim elements instead of block_M x block_K), cb feeds the MFMA straight from LDS, and the
    row factor multiplies that partial sum once at the end.  A key factor that underflows belongs to
    a product that is smaller still.  The diagonal tiles keep the per-element exponent (there the
    factors can leave the fp16 range).  Measured (profiles/r6/mamba_xscale_ab.log): 205 TF against
    231 for the plain 128x64x64 tile -- the workgroup's 2-4 key tiles make the split into two short
    pipelined loops (as in ``lean``) cost more than the per-element exponentials it saves.
    ``ds_blk``: the inter-chunk GEMM C x prev_state^T streamed over dstate in ds_blk-wide slices
    (serial, one LDS slice of each) instead of staging the whole [block_M + block_N, dstate] pair:
    the workgroup's LDS peak falls to the main loop's ring, so more workgroups fit on a CU.
    ``mask_split``: one pipelined loop (not ``lean``'s two) in which only the key tiles that cross
    the causal diagonal take the index compare + select; the tiles wholly below it skip them behind a
    workgroup-uniform branch (default; 215.8 -> 218.9 TF at 4K, same process,
    profiles/r6/mamba_mask_split_ab.log).  ``heavy_first``: row tiles in reverse order on the grid
    axis, so the tiles with the most key tiles (the last rows of a chunk) are dispatched first
    (214.3 TF: off).
    ``xcd_group``: every workgroup of one (batch, chunk) -- all heads and row tiles, which share
    that chunk's ``cb`` and ``C`` tiles (one group) -- is placed on the same XCD (workgroups go
    round-robin over the 8 XCDs by dispatch id), so the shared tiles are fetched into one XCD's L2
    once instead of into all eight."""
    accum_dtype = "float"
    nchunks = seqlen // chunk_size
    assert seqlen % chunk_size == 0 and chunk_size % block_M == 0 and chunk_size % block_K == 0
    n_n = headdim // block_N
    hpg = nheads // ngroups
    n_tiles = (chunk_size // block_M) * n_n
    per_group = nheads * n_tiles  # workgroups of one (batch, chunk)
    xcd_group = xcd_group and (batch * nchunks) % 8 == 0 and ngroups == 1

    @T.macro
    def load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k):
        T.copy(cb[b, c, g, m_idx * block_M:(m_idx + 1) * block_M, k * block_K:(k + 1) * block_K], cb_shared)
        T.copy(x[b, c * chunk_size + k * block_K:c * chunk_size + (k + 1) * block_K, bz,
                 n_idx * block_N:(n_idx + 1) * block_N], x_shared)
        T.copy(dA_cumsum[b, bz, c, k * block_K:(k + 1) * block_K], dA_k)
        T.copy(dt[b, bz, c, k * block_K:(k + 1) * block_K], dt_k)

    @T.prim_func
    def main(cb: T.Tensor((batch, nchunks, ngroups, chunk_size, chunk_size), dtype),
             x: T.Tensor((batch, seqlen, nheads, headdim), dtype),
             dt: T.Tensor((batch, nheads, nchunks, chunk_size), dtype),
             dA_cumsum: T.Tensor((batch, nheads, nchunks, chunk_size), dtype),
             C: T.Tensor((batch, seqlen, ngroups, dstate), dtype),
             prev_states: T.Tensor((batch, nchunks, nheads, headdim, dstate), dtype),
             D: T.Tensor((nheads, ), dtype),
             Output: T.Tensor((batch, seqlen, nheads, headdim), dtype)):
        with T.Kernel(nheads, n_tiles, batch * nchunks, threads=threads) as (bz_, bx_, by_):
            if xcd_group:
                pid = bz_ + nheads * (bx_ + n_tiles * by_)  # dispatch order; XCD = pid % 8
                jj = pid // 8
                by = (jj // per_group) * 8 + pid % 8
                bz = jj % per_group % nheads
                bx = jj % per_group // nheads
            else:
                bz, bx, by = bz_, bx_, by_
            acc_o = T.alloc_fragment((block_M, block_N), accum_dtype)
            cb_shared = T.alloc_shared((block_M, block_K), dtype)
            cb_local = T.alloc_fragment((block_M, block_K), dtype)
            x_shared = T.alloc_shared((block_K, block_N), dtype)
            dsb = ds_blk or dstate
            C_shared = T.alloc_shared((block_M, dsb), dtype)
            st_shared = T.alloc_shared((block_N, dsb), dtype)
            dA_m = T.alloc_fragment((block_M, ), accum_dtype)
            scale_m = T.alloc_fragment((block_M, ), accum_dtype)
            dA_k = T.alloc_shared((block_K, ), dtype)
            dt_k = T.alloc_shared((block_K, ), dtype)
            x_res = T.alloc_fragment((block_M, block_N), dtype)
            o_cast = T.alloc_fragment((block_M, block_N), dtype)
            b = by % batch
            c = by // batch
            m_idx = (chunk_size // block_M - 1 - bx // n_n) if heavy_first else bx // n_n
            n_idx = bx % n_n
            g = bz // hpg
            row0 = c * chunk_size + m_idx * block_M

            T.copy(dA_cumsum[b, bz, c, m_idx * block_M:(m_idx + 1) * block_M], dA_m)
            for i in T.Parallel(block_M):
                scale_m[i] = T.exp2(dA_m[i] * LOG2E)
            T.clear(acc_o)
            if dsb == dstate:
                T.copy(C[b, row0:row0 + block_M, g, :], C_shared)
                T.copy(prev_states[b, c, bz, n_idx * block_N:(n_idx + 1) * block_N, :], st_shared)
                T.gemm(C_shared, st_shared, acc_o, transpose_B=True)
            else:
                for s in T.serial(dstate // dsb):
                    T.copy(C[b, row0:row0 + block_M, g, s * dsb:(s + 1) * dsb], C_shared)
                    T.copy(prev_states[b, c, bz, n_idx * block_N:(n_idx + 1) * block_N, s * dsb:(s + 1) * dsb],
                           st_shared)
                    T.gemm(C_shared, st_shared, acc_o, transpose_B=True)
            for i, j in T.Parallel(block_M, block_N):
                acc_o[i, j] *= scale_m[i]
            n_tot = T.ceildiv((m_idx + 1) * block_M, block_K)
            if lean:
                am = T.alloc_fragment((block_M, ), accum_dtype)
                for i in T.Parallel(block_M):
                    am[i] = dA_m[i] * LOG2E
                n_full = (m_idx * block_M) // block_K  # tiles whose every key precedes every row
                for k in T.Pipelined(n_full, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    for i, j in T.Parallel(block_M, block_K):
                        cb_local[i, j] = T.Cast(accum_dtype, cb_shared[i, j]) * T.exp2(
                            am[i] - T.Cast(accum_dtype, dA_k[j]) * LOG2E) * T.Cast(accum_dtype, dt_k[j])
                    T.gemm(cb_local, x_shared, acc_o)
                for k in T.Pipelined(n_full, n_tot, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    for i, j in T.Parallel(block_M, block_K):
                        cb_local[i, j] = T.Cast(accum_dtype, cb_shared[i, j]) * T.exp2(
                            T.if_then_else(m_idx * block_M + i >= k * block_K + j,
                                           am[i] - T.Cast(accum_dtype, dA_k[j]) * LOG2E,
                                           -T.infinity(accum_dtype))) * T.Cast(accum_dtype, dt_k[j])
                    T.gemm(cb_local, x_shared, acc_o)
            elif xscale:
                am = T.alloc_fragment((block_M, ), accum_dtype)
                xs_shared = T.alloc_shared((block_K, block_N), dtype)
                acc_f = T.alloc_fragment((block_M, block_N), accum_dtype)
                cref = T.alloc_var(accum_dtype)
                for i in T.Parallel(block_M):
                    am[i] = dA_m[i] * LOG2E
                n_full = (m_idx * block_M) // block_K  # tiles whose every key precedes every row
                cref = T.Cast(accum_dtype, dA_cumsum[b, bz, c, T.max(m_idx * block_M - 1, 0)]) * LOG2E
                T.clear(acc_f)
                for k in T.Pipelined(n_full, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    for j, n in T.Parallel(block_K, block_N):  # one key row per thread's vector
                        xs_shared[j, n] = T.Cast(dtype, T.Cast(accum_dtype, x_shared[j, n]) * (T.exp2(
                            cref - T.Cast(accum_dtype, dA_k[j]) * LOG2E) * T.Cast(accum_dtype, dt_k[j])))
                    T.gemm(cb_shared, xs_shared, acc_f)
                for i, j in T.Parallel(block_M, block_N):
                    acc_o[i, j] += acc_f[i, j] * T.exp2(am[i] - cref)
                for k in T.Pipelined(n_full, n_tot, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    for i, j in T.Parallel(block_M, block_K):
                        cb_local[i, j] = T.Cast(accum_dtype, cb_shared[i, j]) * T.exp2(
                            T.if_then_else(m_idx * block_M + i >= k * block_K + j,
                                           am[i] - T.Cast(accum_dtype, dA_k[j]) * LOG2E,
                                           -T.infinity(accum_dtype))) * T.Cast(accum_dtype, dt_k[j])
                    T.gemm(cb_local, x_shared, acc_o)
            elif factored:
                am = T.alloc_fragment((block_M, ), accum_dtype)
                rf = T.alloc_fragment((block_M, ), accum_dtype)
                gk = T.alloc_shared((block_K, ), accum_dtype)
                for i in T.Parallel(block_M):
                    am[i] = dA_m[i] * LOG2E
                for k in T.Pipelined(n_tot, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    # rows inside the key window see exp(a_i - c) up to exp(window span): factor only
                    # when the span is far from fp32's range (block-uniform test; Mamba-2 steps are small)
                    if (T.Cast(accum_dtype, dA_k[0]) - T.Cast(accum_dtype, dA_k[block_K - 1])) * LOG2E < 96.0:
                        for j in T.Parallel(block_K):  # key factors exp(c - b_j) dt_j, c = b of the last key
                            gk[j] = T.exp2((T.Cast(accum_dtype, dA_k[block_K - 1]) - T.Cast(accum_dtype, dA_k[j])) *
                                           LOG2E) * T.Cast(accum_dtype, dt_k[j])
                        for i in T.Parallel(block_M):
                            rf[i] = T.exp2(am[i] - T.Cast(accum_dtype, dA_k[block_K - 1]) * LOG2E)
                        for i, j in T.Parallel(block_M, block_K):
                            cb_local[i, j] = T.if_then_else(m_idx * block_M + i >= k * block_K + j,
                                                            T.Cast(accum_dtype, cb_shared[i, j]) * (rf[i] * gk[j]), 0)
                    else:
                        for i, j in T.Parallel(block_M, block_K):
                            cb_local[i, j] = T.Cast(accum_dtype, cb_shared[i, j]) * T.exp2(
                                T.if_then_else(m_idx * block_M + i >= k * block_K + j,
                                               am[i] - T.Cast(accum_dtype, dA_k[j]) * LOG2E,
                                               -T.infinity(accum_dtype))) * T.Cast(accum_dtype, dt_k[j])
                    T.gemm(cb_local, x_shared, acc_o)
            elif mask_split:
                for k in T.Pipelined(n_tot, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    if k * block_K + block_K - 1 <= m_idx * block_M:  # every key precedes every row
                        for i, j in T.Parallel(block_M, block_K):
                            cb_local[i, j] = cb_shared[i, j] * T.exp2(
                                dA_m[i] * LOG2E - T.Cast(accum_dtype, dA_k[j]) * LOG2E) * T.Cast(accum_dtype, dt_k[j])
                    else:
                        for i, j in T.Parallel(block_M, block_K):
                            cb_local[i, j] = cb_shared[i, j] * T.exp2(
                                T.if_then_else(m_idx * block_M + i >= k * block_K + j,
                                               dA_m[i] * LOG2E - T.Cast(accum_dtype, dA_k[j]) * LOG2E,
                                               -T.infinity(accum_dtype))) * T.Cast(accum_dtype, dt_k[j])
                    T.gemm(cb_local, x_shared, acc_o)
            else:
                for k in T.Pipelined(n_tot, num_stages=num_stages):
                    load_k(cb, x, dA_cumsum, dt, cb_shared, x_shared, dA_k, dt_k, b, c, g, bz, m_idx, n_idx, k)
                    for i, j in T.Parallel(block_M, block_K):
                        # the causal mask selects the exponent (exp2(-inf) = 0), not the product: a
                        # select around the exp became a per-element exec-mask branch (5 SALU each)
                        cb_local[i, j] = cb_shared[i, j] * T.exp2(
                            T.if_then_else(m_idx * block_M + i >= k * block_K + j,
                                           dA_m[i] * LOG2E - T.Cast(accum_dtype, dA_k[j]) * LOG2E,
                                           -T.infinity(accum_dtype))) * T.Cast(accum_dtype, dt_k[j])
                    T.gemm(cb_local, x_shared, acc_o)
            T.copy(x[b, row0:row0 + block_M, bz, n_idx * block_N:(n_idx + 1) * block_N], x_res)
            for i, j in T.Parallel(block_M, block_N):
                o_cast[i, j] = acc_o[i, j] + x_res[i, j] * D[bz]
            T.copy(o_cast, Output[b, row0:row0 + block_M, bz, n_idx * block_N:(n_idx + 1) * block_N])

    return main


@tilelang.jit(out_idx=[7], pass_configs=FAST_MATH)
def chunk_scan_fwd_fused(batch, seqlen, chunk_size, ngroups, nheads, headdim, dstate, block_K=64, num_stages=2,
                         threads=512, dtype="float16"):
    """One workgroup per (batch, chunk, head): the whole chunk's rows at once, so the per-chunk
    vectors (dA in log2 units, dt) are loaded once into LDS as f32, the inter-chunk term is one
    [chunk x dstate] x [dstate x headdim] MFMA GEMM, and the intra-chunk product streams ``cb``
    and ``x`` in ``block_K``-wide slices through a pipelined LDS ring (LDS-DMA).  The slice loop
    covers every row (masked entries are zeros), trading some wasted MFMA work on the upper
    triangle for full-width GEMMs and no per-row-tile prologue."""
    accum_dtype = "float"
    nchunks = seqlen // chunk_size
    assert seqlen % chunk_size == 0 and chunk_size % block_K == 0
    hpg = nheads // ngroups

    @T.prim_func
    def main(cb: T.Tensor((batch, nchunks, ngroups, chunk_size, chunk_size), dtype),
             x: T.Tensor((batch, seqlen, nheads, headdim), dtype),
             dt: T.Tensor((batch, nheads, nchunks, chunk_size), dtype),
             dA_cumsum: T.Tensor((batch, nheads, nchunks, chunk_size), dtype),
             C: T.Tensor((batch, seqlen, ngroups, dstate), dtype),
             prev_states: T.Tensor((batch, nchunks, nheads, headdim, dstate), dtype),
             D: T.Tensor((nheads, ), dtype),
             Output: T.Tensor((batch, seqlen, nheads, headdim), dtype)):
        with T.Kernel(nheads, batch * nchunks, threads=threads) as (bz, by):
            acc_o = T.alloc_fragment((chunk_size, headdim), accum_dtype)
            a_s = T.alloc_shared((chunk_size, ), accum_dtype)
            w_s = T.alloc_shared((chunk_size, ), accum_dtype)
            C_shared = T.alloc_shared((chunk_size, dstate), dtype)
            st_shared = T.alloc_shared((headdim, dstate), dtype)
            cb_shared = T.alloc_shared((chunk_size, block_K), dtype)
            cb_local = T.alloc_fragment((chunk_size, block_K), dtype)
            x_shared = T.alloc_shared((block_K, headdim), dtype)
            x_res = T.alloc_fragment((chunk_size, headdim), dtype)
            o_cast = T.alloc_fragment((chunk_size, headdim), dtype)
            b = by % batch
            c = by // batch
            g = bz // hpg
            row0 = c * chunk_size
            T.copy(C[b, row0:row0 + chunk_size, g, :], C_shared)
            T.copy(prev_states[b, c, bz, :, :], st_shared)
            for i in T.Parallel(chunk_size):
                a_s[i] = T.Cast(accum_dtype, dA_cumsum[b, bz, c, i]) * LOG2E
                w_s[i] = T.Cast(accum_dtype, dt[b, bz, c, i])
            T.clear(acc_o)
            T.gemm(C_shared, st_shared, acc_o, transpose_B=True)
            for i, j in T.Parallel(chunk_size, headdim):
                acc_o[i, j] *= T.exp2(a_s[i])
            for k in T.Pipelined(chunk_size // block_K, num_stages=num_stages):
                T.copy(cb[b, c, g, :, k * block_K:(k + 1) * block_K], cb_shared)
                T.copy(x[b, row0 + k * block_K:row0 + (k + 1) * block_K, bz, :], x_shared)
                for i, j in T.Parallel(chunk_size, block_K):
                    cb_local[i, j] = T.if_then_else(
                        i >= k * block_K + j,
                        cb_shared[i, j] * T.exp2(a_s[i] - a_s[k * block_K + j]) * w_s[k * block_K + j], 0)
                T.gemm(cb_local, x_shared, acc_o)
            T.copy(x[b, row0:row0 + chunk_size, bz, :], x_res)
            for i, j in T.Parallel(chunk_size, headdim):
                o_cast[i, j] = acc_o[i, j] + x_res[i, j] * D[bz]
            T.copy(o_cast, Output[b, row0:row0 + chunk_size, bz, :])

    return main


def ref_program(cb, x, dt, dA_cumsum, C, prev_states, D):
    import torch
    from einops import rearrange, repeat
    _, _, ngroups, _, _ = cb.shape
    batch, seqlen, nheads, headdim = x.shape
    _, _, nchunks, chunk_size = dt.shape
    cb, x, dt, dA_cumsum, C, prev_states, D = [t.float() for t in (cb, x, dt, dA_cumsum, C, prev_states, D)]
    C = repeat(C, "b l g d -> b l (g h) d", h=nheads // ngroups)
    cb = repeat(cb, "b c g l s -> b c (g h) l s", h=nheads // ngroups)
    decay = torch.exp(dA_cumsum[:, :, :, :, None] - dA_cumsum[:, :, :, None, :])
    scores = cb * rearrange(decay, "b h c l s -> b c h l s")
    mask = torch.tril(torch.ones(chunk_size, chunk_size, device=x.device, dtype=torch.bool))
    scores = scores.masked_fill(~mask, 0)
    out = torch.einsum("bchls,bhcs,bcshp->bclhp", scores, dt, rearrange(x, "b (c s) h p -> b c s h p", c=nchunks))
    decay_out = torch.exp(rearrange(dA_cumsum, "b h c l -> b c l h 1"))
    out_prev = torch.einsum("bclhn,bchpn->bclhp", rearrange(C, "b (c l) h n -> b c l h n", c=nchunks),
                            prev_states) * decay_out
    out = rearrange(out + out_prev, "b c l h p -> b (c l) h p")
    return out + x * D.view(-1, 1)


def make_inputs(batch, seqlen, chunk_size, ngroups, nheads, headdim, dstate, device="cuda"):
    import torch
    nchunks = seqlen // chunk_size
    dt = torch.rand(batch, nheads, nchunks, chunk_size, device=device) * 0.1
    dA = -torch.rand(batch, nheads, nchunks, chunk_size, device=device) * 0.1
    return [t.half() for t in (
        torch.randn(batch, nchunks, ngroups, chunk_size, chunk_size, device=device) * 0.1,
        torch.randn(batch, seqlen, nheads, headdim, device=device), dt, dA.cumsum(-1),
        torch.randn(batch, seqlen, ngroups, dstate, device=device) * 0.1,
        torch.randn(batch, nchunks, nheads, headdim, dstate, device=device) * 0.1,
        torch.randn(nheads, device=device))]


def flops(batch, seqlen, chunk_size, nheads, headdim, dstate):
    """The reference benchmark's count (benchmark/mamba2/README.md)."""
    return 2 * batch * seqlen * chunk_size * nheads * headdim * 0.5 + 2 * batch * seqlen * nheads * headdim * dstate


def main(batch=8, heads=80, groups=1, seq_len=4096, chunk_size=256, dim=64, dstate=128):
    kernel = chunk_scan_fwd(batch, seq_len, chunk_size, groups, heads, dim, dstate)
    args = make_inputs(batch, seq_len, chunk_size, groups, heads, dim, dstate)
    out = kernel(*args)
    import torch
    torch.testing.assert_close(out.float(), ref_program(*args), rtol=2e-2, atol=5e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(*args))
    print(f"mamba2 chunk scan seq {seq_len}: {lat:.3f} ms, "
          f"{flops(batch, seq_len, chunk_size, heads, dim, dstate) / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--heads", type=int, default=80)
    p.add_argument("--groups", type=int, default=1)
    p.add_argument("--seq_len", type=int, default=4096)
    p.add_argument("--chunk_size", type=int, default=256)
    p.add_argument("--dim", type=int, default=64)
    p.add_argument("--dstate", type=int, default=128)
    a = p.parse_args()
    main(a.batch, a.heads, a.groups, a.seq_len, a.chunk_size, a.dim, a.dstate)
