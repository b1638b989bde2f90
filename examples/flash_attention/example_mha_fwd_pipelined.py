"""FlashAttention forward with a user-specified software-pipeline schedule
(reference: examples/flash_attention/example_mha_fwd_bshd_wgmma_pipelined.py).

``T.Pipelined(order=, stage=, group=)`` (transform/stage_schedule.py) runs the QK^T GEMM of tile t
next to the rescale + PV GEMM of tile t-1, and the softmax of tile t last:

    iteration t:   S(t) = Q K(t)^T          stage 0, order 0   (MFMA)
                   O   *= scale(t-1)        stage 1, order 1   (VALU)
                   O   += P(t-1) V(t-1)     stage 1, order 2   (MFMA)
                   P(t) = softmax(S(t))     stage 0, order 3   (VALU + v_exp_f32)

Neither neighbouring pair depends on the other, so inside one wave the compiler can interleave
the MFMA stream of one tile with the exp/VALU stream of the other.  K/V tiles are LDS-DMA
producers (order = stage = -1) staged ``num_stages`` deep.
"""
import argparse

import tilelang
import tilelang.language as T
from tilelang.layout import PaddedLayout

from example_mha_fwd import FAST_MATH_NO_NANS, ref_program


@tilelang.jit(out_idx=[3], pass_configs=FAST_MATH_NO_NANS)
def flashattn_pipelined(batch, heads, seq_len, dim, is_causal=False, groups=1, block_M=256, block_N=64,
                        threads=512, num_stages=3, dtype="bfloat16", lazy_rescale=True, q_in_regs=True,
                        young_prio=False, staged_epilogue=False, seq_kv=None, layout="bshd", mfma="16x16",
                        sum_mfma=False, sink=False, sm_scale=None, fold_max=False, prescale_q=False,
                        pingpong=False, pk_scale=False, xcd_heads=False, skip_masked=True, unroll=None):
    """``young_prio``: the second-dispatched half of the waves runs at issue priority 1 (one
    ``s_setprio`` before the main loop; MI355X notes 'Two waves per SIMD', item 4).
    ``seq_kv`` (default ``seq_len``): key/value length; with ``is_causal`` the mask is aligned
    bottom-right (query i sees keys up to i + seq_kv - seq_len).  ``layout``: "bshd" or "bhsd"
    for Q/K/V/O (reference example_mha_fwd_bhsd.py).  ``mfma``: "16x16" (16x16x32) or "32x32"
    (32x32x16 tiles for both GEMMs: one query row per lane, P fed to P V in the accumulator's
    k order, and 24 of each MFMA's 32 cycles free for the softmax VALU stream).
    ``sum_mfma``: the softmax row sums come from the matrix cores: P times a ones tile (16 or 32
    columns) accumulates next to O, rescaled with it, so the per-tile VALU adds, their cross-lane
    reduction and the running-sum update leave the VALU stream (the loop is VALU-issue bound:
    an MFMA holds the SIMD's vector issue for half its cycles).
    ``sink``: a learned per-head logit ``Sinks[heads]`` joins every row's softmax normaliser (the
    gpt-oss attention of examples/attention_sink); it contributes nothing to the output.
    ``fold_max``: the running row max enters the QK^T MFMA chain as its initial accumulator, so
    the scores arrive max-subtracted and a probability is ``v_exp_f32(c * s)``; a row moves its
    max (lazy rescale, threshold 2^8) only on the first tile or when a score beats it by 8 in
    log2 units, and only then are that tile's scores shifted (skipped by an exec-mask branch
    otherwise).  Schedule: QK^T(t) | rescale(t-1) | max-and-decide(t) | PV(t-1) + exp(t), so the
    exponentials of tile t issue between the PV MFMAs of tile t-1.
    ``prescale_q`` (with ``fold_max``): the log2-domain scale c is folded into the Q registers
    once, so a probability is ONE ``v_exp_f32`` with no multiply; the price is Q rounded to bf16
    after scaling: a relative error of 2^-9 in every logit (at |c s| ~ 40 the probabilities of a
    row are off by ~5 %, against ~1.5 % without it).
    ``pingpong`` (with ``fold_max``): waves 4-7 run the same iteration in the order
    rescale(t-1) | PV(t-1) | QK^T(t) | decide(t) | exp(t) (``T.Pipelined(order_alt=)``), so on every
    SIMD one wave's softmax VALU phase sits under its partner's MFMAs instead of both waves
    reaching their VALU phase together after each barrier.
    ``xcd_heads`` (non-causal): workgroups are dealt round-robin over the 8 XCDs by dispatch id;
    the grid is decoded so that all query tiles of one head run on the same XCD (consecutive slots
    of that XCD), so the head's K/V stream is fetched into ONE XCD's L2 and read by all its tiles
    there, instead of into every XCD.
    ``skip_masked`` (causal, ``fold_max``): on a diagonal KV tile the waves whose query rows see
    none of its keys skip the QK^T, PV and row-sum MFMAs (``T.gemm(valid_m_min=)``): up to 6 of
    the 8 waves on the last diagonal tile.
    ``pk_scale`` (with ``fold_max``): the log2-domain scale is applied by its own element-wise loop
    before the exponentials, so the compiler pairs it into ``v_pk_mul_f32`` (16 instead of 32
    multiplies per wave and tile) instead of one ``v_mul_f32`` in front of every ``v_exp_f32``."""
    scale = ((1.0 / dim)**0.5 if sm_scale is None else sm_scale) * 1.44269504
    head_kv = heads // groups
    seq_kv = seq_len if seq_kv is None else seq_kv
    past = seq_kv - seq_len
    assert past >= 0, "seq_kv must be >= seq_len"
    # key-padding mask (reference example_mha_fwd_bshd.py:54): with seq_kv not a multiple of
    # block_N, keys at or past seq_kv get -inf in the LAST KV tile only (a uniform branch: the
    # interior tiles pay nothing); the causal mask already hides them from every stored row
    ragged_kv = seq_kv % block_N != 0 and not is_causal
    bhsd = layout == "bhsd"
    assert layout in ("bshd", "bhsd")
    q_shape = [batch, heads, seq_len, dim] if bhsd else [batch, seq_len, heads, dim]
    kv_shape = [batch, head_kv, seq_kv, dim] if bhsd else [batch, seq_kv, head_kv, dim]
    accum_dtype = "float"
    n_qt = (seq_len + block_M - 1) // block_M
    n_softmax = (8 if lazy_rescale else 7) - (2 if sum_mfma else 0)  # statements of the softmax group
    group = [[0], [1, 2], list(range(3, 3 + n_softmax))]
    group += [[3 + n_softmax], [4 + n_softmax], [5 + n_softmax] + ([6 + n_softmax] if sum_mfma else [])]
    n_ones = 16 if mfma == "16x16" else 32
    n_pv = 2 if sum_mfma else 1
    sc2 = 1.0 if prescale_q else scale  # scale still to apply to the (max-folded) scores
    thr = 8.0 / sc2  # lazy-rescale threshold in the scores' own units
    pk = pk_scale and not prescale_q
    xcd_h = xcd_heads and not is_causal and (heads * batch) % 8 == 0
    fold_group = [[0], [1, 2], [3], [4, 5, 6, 7], [8], list(range(9, 9 + n_pv)),
                  list(range(9 + n_pv, 9 + n_pv + (2 if sum_mfma else 4) + (1 if pk else 0)))]

    @T.macro
    def body(Q, K, V, Output, Sinks):
        # causal: heads on the fastest grid axis and the longest (last) query tiles first.  With few
        # query tiles (<= 4) the tile axis is the slowest, so the longest tiles of EVERY (batch, head)
        # go before any shorter one (b16 h16 s1024: 499 -> 604 TF); with more, the batch stays the
        # slowest axis, keeping a head's K/V shared by more co-resident tiles in L2 (b4 h32 s4096:
        # 1018 vs 995 TF, b8 h32 s2048: 863 vs 834; profiles/r6/fa_lpt_fwd_ab.log)
        lpt = is_causal and n_qt <= 4
        grid = (heads, batch, n_qt) if lpt else (heads, n_qt, batch) if is_causal else (n_qt, heads, batch)
        with T.Kernel(*grid, threads=threads) as (g0_, g1_, bz_):
            if xcd_h:
                pid = g0_ + n_qt * (g1_ + heads * bz_)  # dispatch id: XCD = pid % 8
                jj = pid // 8
                hb = (jj // n_qt) * 8 + pid % 8  # (batch, head) of this slot
                g0, g1, bz = jj % n_qt, hb % heads, hb // heads
            elif lpt:
                g0, g1, bz = g0_, bz_, g1_
            else:
                g0, g1, bz = g0_, g1_, bz_
            bx = (n_qt - 1 - g1) if is_causal else g0
            by = g0 if is_causal else g1
            if q_in_regs:
                Q_s = T.alloc_fragment([block_M, dim], dtype)
            else:
                Q_s = T.alloc_shared([block_M, dim], dtype)
            K_shared = T.alloc_shared([block_N, dim], dtype)
            V_shared = T.alloc_shared([block_N, dim], dtype)
            acc_s = T.alloc_fragment([block_M, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_M, block_N], dtype)
            acc_o = T.alloc_fragment([block_M, dim], accum_dtype)
            scores_max = T.alloc_fragment([block_M], accum_dtype)
            scores_max_prev = T.alloc_fragment([block_M], accum_dtype)
            scores_scale = T.alloc_fragment([block_M], accum_dtype)
            scores_sum = T.alloc_fragment([block_M], accum_dtype)
            logsum = T.alloc_fragment([block_M], accum_dtype)
            rescale = T.alloc_var("int32")
            if sum_mfma:
                ones_s = T.alloc_shared([block_N, n_ones], dtype)
                acc_l = T.alloc_fragment([block_M, n_ones], accum_dtype)
                T.fill(ones_s, 1)
                T.fill(acc_l, 0)

            if bhsd:
                T.copy(Q[bz, by, bx * block_M:(bx + 1) * block_M, :], Q_s)
            else:
                T.copy(Q[bz, bx * block_M:(bx + 1) * block_M, by, :], Q_s)
            T.fill(acc_o, 0)
            T.fill(logsum, 0)
            T.fill(scores_max, -(2.0**30) if lazy_rescale else -T.infinity(accum_dtype))
            rescale = 1
            if young_prio:
                if T.get_thread_binding() >= threads // 2:
                    T.set_priority(1)

            if is_causal:
                exact = past == 0 and seq_len % block_M == 0  # no tile runs past the last key tile
                loop_range = T.ceildiv((bx + 1) * block_M, block_N) if exact else T.min(
                    T.ceildiv((bx + 1) * block_M + past, block_N), T.ceildiv(seq_kv, block_N))
            else:
                loop_range = T.ceildiv(seq_kv, block_N)

            if fold_max:
                if prescale_q:  # log2-domain scale folded into the Q registers once: S' = (c Q) K^T
                    for i, j in T.Parallel(block_M, dim):
                        Q_s[i, j] = T.Cast(dtype, T.Cast(accum_dtype, Q_s[i, j]) * scale)
                T.fill(scores_max, 0)
                for k in T.Pipelined(loop_range, num_stages=num_stages, order=[-1, 0, 1, 2, -1, 3, 4],
                                     stage=[-1, 0, 1, 0, -1, 1, 0], group=fold_group,
                                     order_alt=[-1, 2, 0, 3, -1, 1, 4] if pingpong else None,
                                     alt_cond=(T.get_thread_binding() >= threads // 2) if pingpong else None,
                                     unroll=unroll):
                    # 0: K tile (producer)
                    if bhsd:
                        T.copy(K[bz, by // groups, k * block_N:(k + 1) * block_N, :], K_shared)
                    else:
                        T.copy(K[bz, k * block_N:(k + 1) * block_N, by // groups, :], K_shared)
                    # 1-2: acc_s = S' - m: the running max enters as the MFMA chain's initial
                    # accumulator, so exp2 needs no per-element subtraction
                    if is_causal:
                        if (k + 1) * block_N <= bx * block_M + past + 1:
                            for i, j in T.Parallel(block_M, block_N):
                                acc_s[i, j] = -scores_max[i]
                        else:
                            for i, j in T.Parallel(block_M, block_N):
                                acc_s[i, j] = T.if_then_else(bx * block_M + i + past >= k * block_N + j,
                                                             -scores_max[i], -T.infinity(acc_s.dtype))
                    elif ragged_kv:
                        if k == loop_range - 1:
                            for i, j in T.Parallel(block_M, block_N):
                                acc_s[i, j] = T.if_then_else(k * block_N + j < seq_kv, -scores_max[i],
                                                             -T.infinity(acc_s.dtype))
                        else:
                            for i, j in T.Parallel(block_M, block_N):
                                acc_s[i, j] = -scores_max[i]
                    else:
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = -scores_max[i]
                    # rows below m_lo see none of this tile's keys (causal diagonal)
                    m_lo = (k * block_N - bx * block_M - past) if (is_causal and skip_masked) else None
                    T.gemm(Q_s, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma,
                           valid_m_min=m_lo)
                    # 3: rescale group (one tile behind)
                    if rescale != 0:
                        for i, j in T.Parallel(block_M, dim):
                            acc_o[i, j] *= scores_scale[i]
                        if sum_mfma:
                            for i, j in T.Parallel(block_M, n_ones):
                                acc_l[i, j] *= scores_scale[i]
                    # 4-6: decide: a row moves its max only when a score beats it by 2^8 (or on the
                    # first tile); the rare move subtracts the shift from that tile's scores
                    T.reduce_max(acc_s, scores_max_prev, dim=1, clear=True)
                    rescale = 0
                    for i in T.Parallel(block_M):
                        if scores_max_prev[i] > thr or k == 0:
                            scores_scale[i] = T.if_then_else(k == 0, 1.0, T.exp2(-scores_max_prev[i] * sc2))
                            scores_max[i] = scores_max[i] + scores_max_prev[i]
                            rescale = 1
                        else:
                            scores_scale[i] = 1.0
                            scores_max_prev[i] = 0.0
                    if rescale != 0:
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = acc_s[i, j] - scores_max_prev[i]
                    # 7: V tile (producer); 8-9: O += P V (one tile behind)
                    if bhsd:
                        T.copy(V[bz, by // groups, k * block_N:(k + 1) * block_N, :], V_shared)
                    else:
                        T.copy(V[bz, k * block_N:(k + 1) * block_N, by // groups, :], V_shared)
                    T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma,
                           valid_m_min=m_lo)
                    if sum_mfma:
                        T.gemm(acc_s_cast, ones_s, acc_l, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma,
                               valid_m_min=m_lo)
                    # 10-11: P = exp2(acc_s) -> bf16
                    if pk:
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = acc_s[i, j] * sc2
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = T.exp2(acc_s[i, j])
                    else:
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = T.exp2(acc_s[i, j] * sc2) if not prescale_q else T.exp2(acc_s[i, j])
                    if not sum_mfma:
                        T.reduce_sum(acc_s, scores_sum, dim=1)
                        for i in T.Parallel(block_M):
                            logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                    T.copy(acc_s, acc_s_cast)
            else:
                for k in T.Pipelined(loop_range, num_stages=num_stages, order=[-1, 0, 3, 1, -1, 2],
                                     stage=[-1, 0, 0, 1, -1, 1], group=group):
                    # 0: K tile (producer)
                    if bhsd:
                        T.copy(K[bz, by // groups, k * block_N:(k + 1) * block_N, :], K_shared)
                    else:
                        T.copy(K[bz, k * block_N:(k + 1) * block_N, by // groups, :], K_shared)
                    # 1-2: S = Q K^T
                    if is_causal:
                        # only the diagonal blocks pay for the per-element mask (uniform branch)
                        if (k + 1) * block_N <= bx * block_M + past + 1:
                            T.clear(acc_s)
                        else:
                            for i, j in T.Parallel(block_M, block_N):
                                acc_s[i, j] = T.if_then_else(bx * block_M + i + past >= k * block_N + j, 0,
                                                             -T.infinity(acc_s.dtype))
                    elif ragged_kv:
                        if k == loop_range - 1:
                            for i, j in T.Parallel(block_M, block_N):
                                acc_s[i, j] = T.if_then_else(k * block_N + j < seq_kv, 0, -T.infinity(acc_s.dtype))
                        else:
                            T.clear(acc_s)
                    else:
                        T.clear(acc_s)
                    T.gemm(Q_s, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma)
                    # softmax group
                    T.copy(scores_max, scores_max_prev)
                    if lazy_rescale:
                        T.reduce_max(acc_s, scores_max_prev, dim=1, clear=False)
                        rescale = 0
                        for i in T.Parallel(block_M):
                            if (scores_max_prev[i] - scores_max[i]) * scale > 8.0:
                                scores_scale[i] = T.exp2((scores_max[i] - scores_max_prev[i]) * scale)
                                scores_max[i] = scores_max_prev[i]
                                rescale = 1
                            else:
                                scores_scale[i] = 1.0
                    else:
                        T.reduce_max(acc_s, scores_max, dim=1, clear=False)
                        for i in T.Parallel(block_M):
                            scores_scale[i] = T.exp2(scores_max_prev[i] * scale - scores_max[i] * scale)
                    for i, j in T.Parallel(block_M, block_N):
                        acc_s[i, j] = T.exp2(acc_s[i, j] * scale - scores_max[i] * scale)
                    if not sum_mfma:
                        T.reduce_sum(acc_s, scores_sum, dim=1)
                        for i in T.Parallel(block_M):
                            logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                    T.copy(acc_s, acc_s_cast)
                    # rescale group (one tile behind)
                    if rescale != 0:
                        for i, j in T.Parallel(block_M, dim):
                            acc_o[i, j] *= scores_scale[i]
                        if sum_mfma:
                            for i, j in T.Parallel(block_M, n_ones):
                                acc_l[i, j] *= scores_scale[i]
                    # V tile (producer) and O += P V (one tile behind)
                    if bhsd:
                        T.copy(V[bz, by // groups, k * block_N:(k + 1) * block_N, :], V_shared)
                    else:
                        T.copy(V[bz, k * block_N:(k + 1) * block_N, by // groups, :], V_shared)
                    T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma)
                    if sum_mfma:
                        T.gemm(acc_s_cast, ones_s, acc_l, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma)
            if sum_mfma:  # every column of acc_l holds the row sum: spread it in the row layout
                T.reduce_max(acc_l, logsum, dim=1)
            if sink:
                for i in T.Parallel(block_M):
                    logsum[i] += T.exp2(T.Cast(accum_dtype, Sinks[by]) * 1.44269504 -
                                        scores_max[i] * (sc2 if fold_max else scale))
            for i, j in T.Parallel(block_M, dim):
                acc_o[i, j] /= logsum[i]
            if staged_epilogue:  # O tile through row-padded LDS: 16-byte row-contiguous stores
                O_s = T.alloc_shared([block_M, dim], dtype)
                T.annotate_layout({O_s: PaddedLayout((block_M, dim), 8)})
                T.copy(acc_o, O_s)
                if bhsd:
                    T.copy(O_s, Output[bz, by, bx * block_M:(bx + 1) * block_M, :])
                else:
                    T.copy(O_s, Output[bz, bx * block_M:(bx + 1) * block_M, by, :])
            elif bhsd:
                T.copy(acc_o, Output[bz, by, bx * block_M:(bx + 1) * block_M, :])
            else:
                T.copy(acc_o, Output[bz, bx * block_M:(bx + 1) * block_M, by, :])

    if sink:

        @T.prim_func
        def main(Q: T.Tensor(q_shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(kv_shape, dtype),
                 Output: T.Tensor(q_shape, dtype), Sinks: T.Tensor([heads], dtype)):
            body(Q, K, V, Output, Sinks)
    else:

        @T.prim_func
        def main(Q: T.Tensor(q_shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(kv_shape, dtype),
                 Output: T.Tensor(q_shape, dtype)):
            body(Q, K, V, Output, None)

    return main


def main(batch=1, heads=64, seq_len=4096, dim=128, is_causal=False, groups=1):
    import torch
    flops = 4.0 * batch * heads * seq_len * seq_len * dim * (0.5 if is_causal else 1.0)
    kernel = flashattn_pipelined(batch, heads, seq_len, dim, is_causal, groups)
    q = torch.randn(batch, seq_len, heads, dim, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.bfloat16)
    o = kernel(q, k, v)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, is_causal, groups).float(), rtol=2e-2, atol=2e-2)
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v))
    print(f"flash attention fwd (order/stage pipelined): {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=64)
    p.add_argument("--seq_len", type=int, default=4096)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--is_causal", action="store_true")
    p.add_argument("--groups", type=int, default=1)
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_len, a.dim, a.is_causal, a.groups)
