"""FlashAttention-2 backward (reference: examples/flash_attention/example_mha_bwd_bshd.py,
examples/amd/example_amd_flash_attn_bwd.py) on MI355X, wired into ``torch.autograd``.

Three kernels, Q/K/V/O/dO all [batch, seq, heads, dim] (bshd):

* ``flashattn_fwd``       -- forward that also writes the base-2 log-sum-exp per row;
* ``flashattn_bwd_preprocess`` -- Delta = rowsum(O * dO) (one HBM pass);
* ``flashattn_bwd``       -- one block per (KV tile, head, batch).  K and V stay resident in
  LDS; Q/dO tiles stream through the LDS-DMA pipeline.  Per step (everything transposed so the
  KV rows are the MFMA M dimension and the per-KV-row accumulators dK/dV stay in AGPRs):
      P^T  = exp2(K Q^T * scale - lse)           (ss GEMM, FullRow: whole rows per wave)
      dP^T = V dO^T
      dV  += P^T dO                               (register-A GEMM: accumulator reused as operand)
      dS^T = P^T * (dP^T - Delta) * sm_scale
      dK  += dS^T Q
      dQ  += dS K     (dS^T staged through LDS, read transposed with ds_read_b64_tr_b16,
                       fp32 atomics into dQ -- many KV blocks contribute to one Q row)
* dQ (fp32) is cast back to the input dtype by a copy kernel.
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(out_idx=[3, 4], pass_configs=FAST_MATH)
def flashattn_fwd(batch, heads, seq_len, dim, is_causal, block_M=256, block_N=64, threads=None, dtype="float16",
                  groups=1, num_stages=2, dim_v=None, unroll=None, lpt=None):
    """Forward that also writes the base-2 LSE (the training forward).  Schedule as the sink
    kernel (examples/attention_sink): heads on the fastest grid axis and the heaviest causal
    query tiles first, KV tiles below the diagonal in an unmasked loop and the diagonal ones
    in a masked loop, lazy O rescale, 8 waves x 32 rows."""
    lpt = is_causal if lpt is None else lpt
    if threads is None:
        threads = min(512, 64 * (block_M // 16))  # FullRow: >= 16 query rows per wave
    scale = (1.0 / dim)**0.5 * LOG2E
    dv_ = dim if dim_v is None else dim_v  # V / O head dim (e.g. 192 / 128 in DeepSeek-style heads)
    shape = [batch, seq_len, heads, dim]
    kv_shape = [batch, seq_len, heads // groups, dim]
    v_shape = [batch, seq_len, heads // groups, dv_]
    o_shape = [batch, seq_len, heads, dv_]
    accum_dtype = "float"
    n_qt = (seq_len + block_M - 1) // block_M

    @T.macro
    def step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, m, m_prev, alpha, r_sum, l_sum, k, qt,
             by, bz, masked):
        T.copy(K[bz, k * block_N:(k + 1) * block_N, by // groups, :], K_shared)
        T.copy(V[bz, k * block_N:(k + 1) * block_N, by // groups, :], V_shared)
        if masked:
            for i, j in T.Parallel(block_M, block_N):
                acc_s[i, j] = T.if_then_else(((qt * block_M + i >= k * block_N + j) | (not is_causal)) &
                                             (k * block_N + j < seq_len), 0, -T.infinity(accum_dtype))
        else:
            T.clear(acc_s)
        T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
        T.copy(m, m_prev)
        T.reduce_max(acc_s, m_prev, dim=1, clear=False)
        rescale = T.alloc_var("int32")
        rescale = 0
        for i in T.Parallel(block_M):
            if (m_prev[i] - m[i]) * scale > 8.0:
                alpha[i] = T.exp2((m[i] - m_prev[i]) * scale)
                m[i] = m_prev[i]
                rescale = 1
            else:
                alpha[i] = 1.0
        if rescale != 0:
            for i, j in T.Parallel(block_M, dv_):
                acc_o[i, j] *= alpha[i]
        for i, j in T.Parallel(block_M, block_N):
            acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m[i] * scale)
        T.reduce_sum(acc_s, r_sum, dim=1)
        for i in T.Parallel(block_M):
            l_sum[i] = l_sum[i] * alpha[i] + r_sum[i]
        T.copy(acc_s, acc_s_cast)
        T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)

    @T.prim_func
    def flash_fwd(Q: T.Tensor(shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(v_shape, dtype),
                  Output: T.Tensor(o_shape, dtype), lse: T.Tensor([batch, heads, seq_len], accum_dtype)):
        # causal: the query-tile axis is the SLOWEST grid axis, so the heaviest tiles of every
        # (batch, head) are dispatched before any lighter one (longest-processing-time-first)
        with T.Kernel(heads, *((batch, n_qt) if lpt else (n_qt, batch)), threads=threads) as (by, g1, g2):
            bx, bz = (g2, g1) if lpt else (g1, g2)
            Q_shared = T.alloc_shared([block_M, dim], dtype)
            K_shared = T.alloc_shared([block_N, dim], dtype)
            V_shared = T.alloc_shared([block_N, dv_], dtype)
            acc_s = T.alloc_fragment([block_M, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_M, block_N], dtype)
            acc_o = T.alloc_fragment([block_M, dv_], accum_dtype)
            o_cast = T.alloc_fragment([block_M, dv_], dtype)
            m = T.alloc_fragment([block_M], accum_dtype)
            m_prev = T.alloc_fragment([block_M], accum_dtype)
            alpha = T.alloc_fragment([block_M], accum_dtype)
            r_sum = T.alloc_fragment([block_M], accum_dtype)
            l_sum = T.alloc_fragment([block_M], accum_dtype)
            qt = (n_qt - 1 - bx) if is_causal else bx  # heaviest causal tiles first
            T.copy(Q[bz, qt * block_M:(qt + 1) * block_M, by, :], Q_shared)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            if is_causal:
                end = T.min(T.ceildiv(seq_len, block_N), T.ceildiv((qt + 1) * block_M, block_N))
                full_end = T.min((qt * block_M + 1) // block_N, end)
            else:
                end = T.ceildiv(seq_len, block_N)
                full_end = seq_len // block_N
            for k in T.Pipelined(full_end, num_stages=num_stages, unroll=unroll):
                step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, m, m_prev, alpha, r_sum, l_sum, k,
                     qt, by, bz, False)
            for k in T.Pipelined(full_end, end, num_stages=num_stages):
                step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, m, m_prev, alpha, r_sum, l_sum, k,
                     qt, by, bz, True)
            for i, j in T.Parallel(block_M, dv_):
                o_cast[i, j] = acc_o[i, j] / l_sum[i]
            T.copy(o_cast, Output[bz, qt * block_M:(qt + 1) * block_M, by, :])
            for i in T.Parallel(block_M):
                l_sum[i] = T.log2(l_sum[i]) + m[i] * scale
            T.copy(l_sum, lse[bz, by, qt * block_M:(qt + 1) * block_M])

    return flash_fwd


@tilelang.jit(out_idx=[2], pass_configs=FAST_MATH)
def flashattn_bwd_preprocess(batch, heads, seq_len, dim, blk=32, threads=256, dtype="float16"):
    shape = [batch, seq_len, heads, dim]

    @T.prim_func
    def flash_bwd_prep(O: T.Tensor(shape, dtype), dO: T.Tensor(shape, dtype),
                       Delta: T.Tensor([batch, heads, seq_len], "float")):
        with T.Kernel(heads, T.ceildiv(seq_len, blk), batch, threads=threads) as (bx, by, bz):
            o = T.alloc_fragment([blk, dim], dtype)
            do = T.alloc_fragment([blk, dim], dtype)
            acc = T.alloc_fragment([blk, dim], "float")
            delta = T.alloc_fragment([blk], "float")
            T.copy(O[bz, by * blk:(by + 1) * blk, bx, :], o)
            T.copy(dO[bz, by * blk:(by + 1) * blk, bx, :], do)
            for i, j in T.Parallel(blk, dim):
                acc[i, j] = T.Cast("float", o[i, j]) * T.Cast("float", do[i, j])
            T.reduce_sum(acc, delta, 1)
            T.copy(delta, Delta[bz, bx, by * blk:(by + 1) * blk])

    return flash_bwd_prep


@tilelang.jit(out_idx=[1], pass_configs=FAST_MATH)
def flashattn_bwd_postprocess(batch, heads, seq_len, dim, blk=64, threads=256, dtype="float16"):
    shape = [batch, seq_len, heads, dim]

    @T.prim_func
    def flash_bwd_post(dQ: T.Tensor(shape, "float"), dQ_out: T.Tensor(shape, dtype)):
        with T.Kernel(T.ceildiv(seq_len, blk), heads, batch, threads=threads) as (bx, by, bz):
            t = T.alloc_fragment([blk, dim], "float")
            tc = T.alloc_fragment([blk, dim], dtype)
            T.copy(dQ[bz, bx * blk:(bx + 1) * blk, by, :], t)
            T.copy(t, tc)
            T.copy(tc, dQ_out[bz, bx * blk:(bx + 1) * blk, by, :])

    return flash_bwd_post


@tilelang.jit(pass_configs=FAST_MATH)
def flashattn_bwd(batch, heads, seq_len, dim, is_causal, block_M=128, block_N=64, threads=512, num_stages=2,
                  dtype="float16", dq_mode="atomic", groups=1, dim_v=None, kv_split=1, unroll=None, lpt=None,
                  mask_split=True):
    """``dq_mode``: "atomic" (fp32 atomics into dQ, one kernel) or "none" (dK/dV only; dQ comes from
    ``flashattn_bwd_dq``) -- the dQ atomics were 85% of the single-kernel time on MI355X.
    GQA (``groups`` query heads per KV head): one block per KV head walks the Q/dO tiles of all
    its query heads in ONE pipelined loop (head = it // n_q, tile = it % n_q), so dK/dV of the
    group accumulate in registers -- no atomics, no per-query-head dK/dV buffers.
    ``kv_split`` > 1 (few KV heads, e.g. 2 KV heads x 8 key tiles x batch 8 = 128 workgroups on
    256 CUs): each KV head's query heads are split over ``kv_split`` workgroups that write fp32
    partial dK/dV [kv_split, batch, seq, head_kv, d] (summed by the caller), so the grid fills
    the chip instead of serialising all ``groups`` heads in one workgroup."""
    lpt = is_causal if lpt is None else lpt
    sm_scale = (1.0 / dim)**0.5
    scale = sm_scale * LOG2E
    shape = [batch, seq_len, heads, dim]
    head_kv = heads // groups
    kv_shape = [batch, seq_len, head_kv, dim]
    dv_ = dim if dim_v is None else dim_v
    v_shape = [batch, seq_len, head_kv, dv_]
    o_shape = [batch, seq_len, heads, dv_]
    accum_dtype = "float"
    assert groups % kv_split == 0 and (kv_split == 1 or dq_mode == "none")
    gps = groups // kv_split  # query heads per workgroup
    if kv_split > 1:
        kv_shape_o = [kv_split, batch, seq_len, head_kv, dim]
        v_shape_o = [kv_split, batch, seq_len, head_kv, dv_]
        out_dtype = accum_dtype
    else:
        kv_shape_o, v_shape_o, out_dtype = kv_shape, v_shape, dtype

    @T.macro
    def body(Q, K, V, dO, lse, Delta, dQ, dK, dV):
        # causal: key tile on the SLOWEST grid axis -- tile 0 (the longest walk) of every (batch, head)
        # is dispatched first (longest-processing-time-first over the whole grid, not per batch)
        n_kt = (seq_len + block_M - 1) // block_M
        with T.Kernel(head_kv * kv_split, *((batch, n_kt) if lpt else (n_kt, batch)), threads=threads) as (
                bxs, g1, g2):
            by, bz = (g2, g1) if lpt else (g1, g2)
            bx, sp = (bxs // kv_split, bxs % kv_split) if kv_split > 1 else (bxs, 0)  # KV head, query-head slice
            K_shared = T.alloc_shared([block_M, dim], dtype)
            V_shared = T.alloc_shared([block_M, dv_], dtype)
            q = T.alloc_shared([block_N, dim], dtype)
            do = T.alloc_shared([block_N, dv_], dtype)
            dsT_shared = T.alloc_shared([block_M, block_N], dtype)
            lse_shared = T.alloc_shared([block_N], accum_dtype)
            delta = T.alloc_shared([block_N], accum_dtype)
            qkT = T.alloc_fragment([block_M, block_N], accum_dtype)
            dsT = T.alloc_fragment([block_M, block_N], accum_dtype)
            qkT_cast = T.alloc_fragment([block_M, block_N], dtype)
            dsT_cast = T.alloc_fragment([block_M, block_N], dtype)
            dv = T.alloc_fragment([block_M, dv_], accum_dtype)
            dk = T.alloc_fragment([block_M, dim], accum_dtype)
            dq = T.alloc_fragment([block_N, dim], accum_dtype)
            dv_cast = T.alloc_fragment([block_M, dv_], dtype)
            dk_cast = T.alloc_fragment([block_M, dim], dtype)

            T.copy(K[bz, by * block_M:(by + 1) * block_M, bx, :], K_shared)
            T.copy(V[bz, by * block_M:(by + 1) * block_M, bx, :], V_shared)
            T.clear(dv)
            T.clear(dk)
            loop_st = T.floordiv(by * block_M, block_N) if is_causal else 0
            loop_ed = T.ceildiv(seq_len, block_N)
            n_q = loop_ed - loop_st
            for it in T.Pipelined(n_q * gps, num_stages=num_stages, unroll=unroll):
                # clamped into range: provably in bounds, so the Q / dO / lse / Delta tiles are LDS-DMA
                # producers (division / modulo by a runtime count hides the range from the prover)
                hq0 = bx * groups + sp * gps if kv_split > 1 else bx * groups
                hq = T.max(T.min(hq0 + it // n_q, heads - 1), 0)
                k = T.max(T.min(loop_st + it % n_q, loop_ed - 1), 0)
                T.copy(Q[bz, k * block_N:(k + 1) * block_N, hq, :], q)
                T.clear(qkT)
                T.gemm(K_shared, q, qkT, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(lse[bz, hq, k * block_N:(k + 1) * block_N], lse_shared)
                # the causal mask selects the exponent (exp2(-inf) = 0); ``mask_split``: only tiles that
                # cross the diagonal take the select (a uniform branch: key tile and query tile are
                # workgroup-uniform), the ones wholly past it run the plain exponent
                if is_causal and mask_split:
                    if by * block_M + block_M - 1 <= k * block_N:
                        for i, j in T.Parallel(block_M, block_N):
                            qkT[i, j] = T.exp2(qkT[i, j] * scale - lse_shared[j])
                    else:
                        for i, j in T.Parallel(block_M, block_N):
                            qkT[i, j] = T.exp2(T.if_then_else(by * block_M + i <= k * block_N + j,
                                                              qkT[i, j] * scale - lse_shared[j],
                                                              -T.infinity(accum_dtype)))
                else:
                    for i, j in T.Parallel(block_M, block_N):
                        qkT[i, j] = T.exp2(T.if_then_else((by * block_M + i <= k * block_N + j) | (not is_causal),
                                                          qkT[i, j] * scale - lse_shared[j], -T.infinity(accum_dtype)))
                T.copy(dO[bz, k * block_N:(k + 1) * block_N, hq, :], do)
                T.clear(dsT)
                T.gemm(V_shared, do, dsT, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(qkT, qkT_cast)
                T.gemm(qkT_cast, do, dv, policy=T.GemmWarpPolicy.FullRow)
                T.copy(Delta[bz, hq, k * block_N:(k + 1) * block_N], delta)
                for i, j in T.Parallel(block_M, block_N):
                    dsT_cast[i, j] = qkT[i, j] * (dsT[i, j] - delta[j]) * sm_scale
                T.gemm(dsT_cast, q, dk, policy=T.GemmWarpPolicy.FullRow)
                if dq_mode == "atomic":
                    T.copy(dsT_cast, dsT_shared)
                    T.clear(dq)
                    T.gemm(dsT_shared, K_shared, dq, transpose_A=True)
                    T.atomic_add(dQ[bz, k * block_N:(k + 1) * block_N, hq, :], dq)
            if kv_split > 1:
                T.copy(dv, dV[sp, bz, by * block_M:(by + 1) * block_M, bx, :])
                T.copy(dk, dK[sp, bz, by * block_M:(by + 1) * block_M, bx, :])
            else:
                T.copy(dv, dv_cast)
                T.copy(dk, dk_cast)
                T.copy(dv_cast, dV[bz, by * block_M:(by + 1) * block_M, bx, :])
                T.copy(dk_cast, dK[bz, by * block_M:(by + 1) * block_M, bx, :])

    if dq_mode == "atomic":

        @T.prim_func
        def flash_bwd(Q: T.Tensor(shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(v_shape, dtype),
                      dO: T.Tensor(o_shape, dtype), lse: T.Tensor([batch, heads, seq_len], accum_dtype),
                      Delta: T.Tensor([batch, heads, seq_len], accum_dtype), dQ: T.Tensor(shape, accum_dtype),
                      dK: T.Tensor(kv_shape, dtype), dV: T.Tensor(v_shape, dtype)):
            body(Q, K, V, dO, lse, Delta, dQ, dK, dV)
    else:

        @T.prim_func
        def flash_bwd(Q: T.Tensor(shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(v_shape, dtype),
                      dO: T.Tensor(o_shape, dtype), lse: T.Tensor([batch, heads, seq_len], accum_dtype),
                      Delta: T.Tensor([batch, heads, seq_len], accum_dtype), dK: T.Tensor(kv_shape_o, out_dtype),
                      dV: T.Tensor(v_shape_o, out_dtype)):
            body(Q, K, V, dO, lse, Delta, None, dK, dV)

    return flash_bwd


@tilelang.jit(out_idx=[6], pass_configs=FAST_MATH)
def flashattn_bwd_dq(batch, heads, seq_len, dim, is_causal, block_M=128, block_N=64, threads=256, num_stages=2,
                     dtype="float16", groups=1, dim_v=None, unroll=None, lpt=None, fuse_delta=False, mask_split=True):
    """dQ without atomics: one block per (query tile, head, batch) walks the KV tiles, recomputing
    P and dP (2 extra GEMMs) and accumulating dQ = dS K in registers -- on MI355X this is ~4x
    faster than fp32 atomics from every KV block (measured: docs/RESULTS.md).
    ``fuse_delta``: the preprocess (Delta = rowsum(O * dO)) is done here for the block's own rows
    from its dO tile and an O tile (an extra trailing input ``O``), and Delta is written out for the
    dK/dV kernel, which then runs after this one -- one launch and one pass over dO fewer."""
    lpt = is_causal if lpt is None else lpt
    sm_scale = (1.0 / dim)**0.5
    scale = sm_scale * LOG2E
    shape = [batch, seq_len, heads, dim]
    kv_shape = [batch, seq_len, heads // groups, dim]
    dv_ = dim if dim_v is None else dim_v
    v_shape = [batch, seq_len, heads // groups, dv_]
    o_shape = [batch, seq_len, heads, dv_]
    accum_dtype = "float"

    @T.macro
    def body(Q, K, V, dO, lse, Delta, dQ, O):
        n_t = (seq_len + block_M - 1) // block_M
        # causal: the query-tile axis is the slowest, so the longest dQ rows (last query tiles) of
        # every (batch, head) are dispatched first
        with T.Kernel(heads, *((batch, n_t) if lpt else (n_t, batch)), threads=threads) as (bx, g1, g2):
            by_raw, bz = (g2, g1) if lpt else (g1, g2)
            by = (n_t - 1 - by_raw) if is_causal else by_raw
            q = T.alloc_shared([block_M, dim], dtype)
            do = T.alloc_shared([block_M, dv_], dtype)
            K_shared = T.alloc_shared([block_N, dim], dtype)
            V_shared = T.alloc_shared([block_N, dv_], dtype)
            lse_f = T.alloc_fragment([block_M], accum_dtype)
            delta_f = T.alloc_fragment([block_M], accum_dtype)
            s = T.alloc_fragment([block_M, block_N], accum_dtype)
            dp = T.alloc_fragment([block_M, block_N], accum_dtype)
            ds_cast = T.alloc_fragment([block_M, block_N], dtype)
            dq = T.alloc_fragment([block_M, dim], accum_dtype)
            dq_cast = T.alloc_fragment([block_M, dim], dtype)
            T.copy(Q[bz, by * block_M:(by + 1) * block_M, bx, :], q)
            T.copy(dO[bz, by * block_M:(by + 1) * block_M, bx, :], do)
            T.copy(lse[bz, bx, by * block_M:(by + 1) * block_M], lse_f)
            if fuse_delta:
                # Delta of this block's rows (the preprocess kernel's work), staged through LDS so the
                # reduction's row layout and the score tile's are each inferred on their own
                o_f = T.alloc_fragment([block_M, dv_], dtype)
                prod = T.alloc_fragment([block_M, dv_], accum_dtype)
                d_red = T.alloc_fragment([block_M], accum_dtype)
                d_s = T.alloc_shared([block_M], accum_dtype)
                T.copy(O[bz, by * block_M:(by + 1) * block_M, bx, :], o_f)
                for i, j in T.Parallel(block_M, dv_):
                    prod[i, j] = T.Cast(accum_dtype, o_f[i, j]) * T.Cast(accum_dtype, do[i, j])
                T.reduce_sum(prod, d_red, dim=1)
                T.copy(d_red, d_s)
                T.copy(d_s, delta_f)
                T.copy(d_s, Delta[bz, bx, by * block_M:(by + 1) * block_M])
            else:
                T.copy(Delta[bz, bx, by * block_M:(by + 1) * block_M], delta_f)
            T.clear(dq)
            loop_ed = T.ceildiv((by + 1) * block_M, block_N) if is_causal else T.ceildiv(seq_len, block_N)
            for k in T.Pipelined(loop_ed, num_stages=num_stages, unroll=unroll):
                T.copy(K[bz, k * block_N:(k + 1) * block_N, bx // groups, :], K_shared)
                T.copy(V[bz, k * block_N:(k + 1) * block_N, bx // groups, :], V_shared)
                T.clear(s)
                T.gemm(q, K_shared, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.clear(dp)
                T.gemm(do, V_shared, dp, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                if is_causal and mask_split:  # uniform branch: only diagonal tiles take the select
                    if by * block_M >= k * block_N + block_N - 1:
                        for i, j in T.Parallel(block_M, block_N):
                            ds_cast[i, j] = T.exp2(s[i, j] * scale - lse_f[i]) * (dp[i, j] - delta_f[i]) * sm_scale
                    else:
                        for i, j in T.Parallel(block_M, block_N):
                            pe = T.exp2(T.if_then_else(by * block_M + i >= k * block_N + j, s[i, j] * scale - lse_f[i],
                                                       -T.infinity(accum_dtype)))
                            ds_cast[i, j] = pe * (dp[i, j] - delta_f[i]) * sm_scale
                else:
                    for i, j in T.Parallel(block_M, block_N):
                        ds_cast[i, j] = T.exp2(T.if_then_else(
                            (by * block_M + i >= k * block_N + j) | (not is_causal),
                            s[i, j] * scale - lse_f[i], -T.infinity(accum_dtype))) * (dp[i, j] - delta_f[i]) * sm_scale
                T.gemm(ds_cast, K_shared, dq, policy=T.GemmWarpPolicy.FullRow)
            T.copy(dq, dq_cast)
            T.copy(dq_cast, dQ[bz, by * block_M:(by + 1) * block_M, bx, :])

    if fuse_delta:

        @T.prim_func
        def flash_bwd_dq(Q: T.Tensor(shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(v_shape, dtype),
                         dO: T.Tensor(o_shape, dtype), lse: T.Tensor([batch, heads, seq_len], accum_dtype),
                         Delta: T.Tensor([batch, heads, seq_len], accum_dtype), dQ: T.Tensor(shape, dtype),
                         O: T.Tensor(o_shape, dtype)):
            body(Q, K, V, dO, lse, Delta, dQ, O)
    else:

        @T.prim_func
        def flash_bwd_dq(Q: T.Tensor(shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(v_shape, dtype),
                         dO: T.Tensor(o_shape, dtype), lse: T.Tensor([batch, heads, seq_len], accum_dtype),
                         Delta: T.Tensor([batch, heads, seq_len], accum_dtype), dQ: T.Tensor(shape, dtype)):
            body(Q, K, V, dO, lse, Delta, dQ, None)

    return flash_bwd_dq


BWD_DQ_MODE = "separate"  # or "atomic" (single kernel, fp32 atomics into dQ)
BWD_FUSE_DELTA = True  # Delta computed inside the dQ kernel, which then runs before dK/dV
BWD_OVERLAP = False  # dQ on a side stream: measured slower (0.374 -> 0.509 ms, profiles/r3/s3/bwd/)


def _tiles(D, Dv, kind, causal=False, S=None):
    """Tile sizes that keep each kernel's LDS (operand tiles + 2-stage rings) under 160 KiB: the
    defaults are sized for D = Dv <= 128; wider heads (e.g. D=192 / Dv=128) halve the streamed tile.
    d64 heads use the winners of scripts/sweep_fa_bwd.py (b8 h32 s1024, profiles/r3/s3/bwd/):
    non-causal dK/dV 256x64 over 8 waves (209 -> 182 us), dQ 128x64 over 8 waves (150 -> 130 us);
    causal 64x32 / 64x64 over 4 waves (more, shorter workgroups balance the triangle).  The lowered
    main loops run under #pragma unroll where that measured faster (the ring slot of each copy a
    constant; outputs bitwise identical; profiles/r6/fa_bwd_unroll_ab.log, fa_train_unroll_ab.log):
    d64 dK/dV 173 -> 156 us, d128 dK/dV / dQ +8.5 / +9.4 %, forward +2-7 % non-causal; the causal
    d128 forward and dK/dV and the GQA d192 dK/dV lose 0.5-1.7 % and keep the plain loop.
    Causal d64 with the tile axis slowest in the grid (longest walks of every (batch, head) first,
    ``lpt``; profiles/r6/fa_bwd_lpt_ab*.log): dK/dV 128x32 over 4 waves up to S = 1024 (139.5 ->
    130.7 us at b8 h32 s1024), the non-causal 256x64 / 8-wave tile beyond (b2 h32 s4096 430 ->
    349 us); dQ 128x64 over 4 waves (98 -> 93 us, 304 -> 277 us)."""
    fwd = {} if causal else dict(unroll=2)
    if D + Dv <= 128:
        if causal:
            long_s = S is not None and S >= 2048
            bwd = dict(block_M=256, block_N=64, threads=512, unroll=4) if long_s else \
                dict(block_M=128, block_N=32, threads=256, unroll=2)
            return {"fwd": fwd, "bwd": bwd, "dq": dict(block_M=128, block_N=64, threads=256, unroll=2)}[kind]
        return {"fwd": fwd, "bwd": dict(block_M=256, block_N=64, threads=512, unroll=4),
                "dq": dict(block_M=128, block_N=64, threads=512, unroll=4)}[kind]
    if D + Dv <= 256:
        # causal dQ: 256x32 over 8 waves, 3.5-12 % faster than 128x64 (profiles/r6/fa_bwd_dq128_ab.log)
        dq = dict(block_M=256, block_N=32, threads=512) if causal else dict(unroll=2)
        return {"fwd": fwd, "bwd": {} if causal else dict(unroll=2), "dq": dq}[kind]
    return {"fwd": dict(block_M=128, **fwd), "bwd": dict(block_N=32), "dq": dict(block_N=32, unroll=2)}[kind]


def _kv_split(B, S, HKV, G, block_M, target_wgs=512):
    """Query-head split of the GQA dK/dV kernel so the grid reaches ~``target_wgs`` workgroups."""
    wgs = B * HKV * -(-S // block_M)
    split = 1
    while split < G and wgs * split < target_wgs and G % (split * 2) == 0:
        split *= 2
    return split


class _attention:
    """torch.autograd.Function built lazily (keeps this module importable without a GPU)."""
    fn = None

    @classmethod
    def get(cls):
        if cls.fn is None:
            import torch

            class Attn(torch.autograd.Function):

                @staticmethod
                def forward(ctx, q, k, v, causal):
                    B, S, H, D = q.shape
                    G = H // k.shape[2]
                    dt = "bfloat16" if q.dtype == torch.bfloat16 else "float16"
                    Dv = v.shape[-1]
                    fwd = flashattn_fwd(B, H, S, D, causal, dtype=dt, groups=G, dim_v=Dv,
                                        **_tiles(D, Dv, "fwd", causal, S))
                    o, lse = fwd(q, k, v)
                    ctx.save_for_backward(q, k, v, o, lse)
                    ctx.causal = causal
                    return o

                @staticmethod
                def backward(ctx, do):
                    q, k, v, o, lse = ctx.saved_tensors
                    B, S, H, D = q.shape
                    G = H // k.shape[2]
                    dt = "bfloat16" if q.dtype == torch.bfloat16 else "float16"
                    Dv = v.shape[-1]
                    do = do.contiguous()
                    fuse = BWD_FUSE_DELTA and BWD_DQ_MODE != "atomic" and not BWD_OVERLAP
                    if fuse:
                        # the dQ kernel computes Delta for its rows and runs first (no preprocess)
                        delta = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
                        dq = flashattn_bwd_dq(B, H, S, D, ctx.causal, dtype=dt, groups=G, dim_v=Dv, fuse_delta=True,
                                              **_tiles(D, Dv, "dq", ctx.causal, S))(q, k, v, do, lse, delta, o)
                    else:
                        delta = flashattn_bwd_preprocess(B, H, S, Dv, dtype=dt)(o, do)
                    dk = torch.empty_like(k)
                    dv = torch.empty_like(v)
                    bw = _tiles(D, Dv, "bwd", ctx.causal, S)
                    split = _kv_split(B, S, k.shape[2], G, bw.get("block_M", 128))
                    if BWD_DQ_MODE == "atomic":
                        dq = torch.zeros(B, S, H, D, dtype=torch.float32, device=q.device)
                        bwd = flashattn_bwd(B, H, S, D, ctx.causal, dtype=dt, groups=G, dim_v=Dv,
                                            **bw)
                        bwd(q, k, v, do, lse, delta, dq, dk, dv)
                        return flashattn_bwd_postprocess(B, H, S, D, dtype=dt)(dq), dk, dv, None
                    # dK/dV kernel without dQ + an atomic-free dQ kernel; they only share read-only
                    # inputs, so with BWD_OVERLAP the dQ kernel runs on a side stream and fills the
                    # CUs the dK/dV grid's tail leaves idle
                    bdq = None if fuse else flashattn_bwd_dq(B, H, S, D, ctx.causal, dtype=dt, groups=G, dim_v=Dv,
                                                             **_tiles(D, Dv, "dq", ctx.causal, S))
                    side = None
                    if BWD_OVERLAP and q.is_cuda:
                        main_s = torch.cuda.current_stream()
                        side = torch.cuda.Stream()
                        side.wait_stream(main_s)
                        with torch.cuda.stream(side):
                            dq = bdq(q, k, v, do, lse, delta)
                    if split > 1:
                        dkp = torch.empty((split, ) + tuple(k.shape), dtype=torch.float32, device=k.device)
                        dvp = torch.empty((split, ) + tuple(v.shape), dtype=torch.float32, device=v.device)
                        flashattn_bwd(B, H, S, D, ctx.causal, dtype=dt, dq_mode="none", groups=G, dim_v=Dv,
                                      kv_split=split, **bw)(q, k, v, do, lse, delta, dkp, dvp)
                        dk, dv = dkp.sum(0).to(k.dtype), dvp.sum(0).to(v.dtype)
                    else:
                        flashattn_bwd(B, H, S, D, ctx.causal, dtype=dt, dq_mode="none", groups=G, dim_v=Dv,
                                      **bw)(q, k, v, do, lse, delta, dk, dv)
                    if fuse:
                        pass  # dQ came out of the fused kernel above
                    elif side is None:
                        dq = bdq(q, k, v, do, lse, delta)
                    else:
                        main_s.wait_stream(side)
                        dq.record_stream(main_s)
                    return dq, dk, dv, None

            cls.fn = Attn
        return cls.fn


def attention(q, k, v, causal=False):
    return _attention.get().apply(q, k, v, causal)


def ref_program(Q, K, V, is_causal):
    import torch
    dim = Q.size(-1)
    G = Q.size(2) // K.size(2)
    K, V = K.repeat_interleave(G, 2), V.repeat_interleave(G, 2)
    scores = torch.einsum("bqhd,bkhd->bhqk", Q.float(), K.float()) / dim**0.5
    if is_causal:
        s = Q.size(1)
        mask = torch.tril(torch.ones(s, s, device=scores.device))
        scores = scores.masked_fill(mask == 0, float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", torch.softmax(scores, dim=-1), V.float()).to(Q.dtype)


def main(batch=8, heads=32, seq_len=1024, dim=64, causal=False):
    import torch
    flops = 5 * 2.0 * batch * heads * seq_len * seq_len * dim * (0.5 if causal else 1.0)
    Q = torch.randn(batch, seq_len, heads, dim, dtype=torch.half, device="cuda").requires_grad_()
    K = torch.randn_like(Q).requires_grad_()
    V = torch.randn_like(Q).requires_grad_()
    dO = torch.randn_like(Q)
    O = attention(Q, K, V, causal)
    O.backward(dO)
    grads = [t.grad.clone() for t in (Q, K, V)]
    for t in (Q, K, V):
        t.grad = None
    ref_program(Q, K, V, causal).backward(dO)
    for g, t in zip(grads, (Q, K, V)):
        torch.testing.assert_close(g, t.grad, rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    O = attention(Q, K, V, causal)  # the check above freed the first graph
    # same measurement as the reference example (examples/flash_attention/example_mha_bwd_bshd.py:333):
    # includes autograd's accumulation of dQ/dK/dV into the leaves' .grad (three elementwise adds)
    lat = do_bench(lambda: O.backward(dO, retain_graph=True))
    print(f"flash attention bwd: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")
    # the backward alone: torch.autograd.grad returns the gradients without accumulating them
    lat = do_bench(lambda: torch.autograd.grad(O, (Q, K, V), dO, retain_graph=True))
    print(f"flash attention bwd (no .grad accumulation): {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--h", type=int, default=32)
    p.add_argument("--n_ctx", type=int, default=1024)
    p.add_argument("--d_head", type=int, default=64)
    p.add_argument("--causal", action="store_true")
    a = p.parse_args()
    main(a.batch, a.h, a.n_ctx, a.d_head, a.causal)
