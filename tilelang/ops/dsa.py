"""DeepSeek Sparse Attention (DSA) kernels: sparse MLA forward, fp8 lightning indexer, top-k selector.

Library home of the kernels used by ``tilelang.models.deepseek_v32`` and the examples in
``examples/deepseek_v32`` (reference: examples/deepseek_v32/{sparse_mla_fwd,fp8_lighting_indexer,
topk_selector}.py and inference/kernel.py).  Schedules are documented in the example files.
"""
import functools

import tilelang
import tilelang.language as T
from tilelang.layout import PaddedLayout

LOG2E = 1.44269504


# exp2 straight on v_exp_f32 (differs from the OCML expansion only below 2^-126): 772 -> 826 TF at the
# reference's benchmark shape (profiles/r6/smla_fast_math_ab.log; the expansion's range checks were
# 3 VALU per exponential in a VALU-issue-bound loop)
@tilelang.jit(out_idx=[3, 4], pass_configs={tilelang.PassConfigKey.TL_GEMM_FOLD_DEFAULT_GUARD: False,
                                            tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def sparse_mla_fwd(batch, seq_len, seq_len_kv, heads, dim, tail_dim, topk, kv_group=1, sm_scale=None, block_I=64,
                   threads=None, dtype="bfloat16", num_stages=2, block_H=None, xcd_pair=True, lazy_rescale=True,
                   wide=None, staged_out=True, sum_mfma=None):
    """Sparse MLA forward over the ``topk`` selected latent rows of every query token.

    Schedule (MI355X): one block per (token, 64-head slice); Q stays in registers (it is the
    MFMA A operand of both score GEMMs), so LDS holds only the gathered KV rows, double
    buffered: ``T.gather_rows`` becomes a lane-addressed buffer LDS-DMA issued one tile ahead
    of the MFMA work (``T.Pipelined``), i.e. the gather latency hides behind the GEMMs.
    ``wide`` (default for 64-head slices): 8 waves, S = Q K^T on a 4x2 wave grid, P through
    LDS and O = P V split over the 512 latent columns, so each wave holds a quarter of the O
    accumulator and two waves share every SIMD (656 TF vs 531 TF for the 4-wave FullRow
    form, where every wave owns 16 head rows and P never leaves registers).
    ``sum_mfma`` (default with ``wide``): the softmax row sums come from P (already in LDS for P V)
    times a ones tile on the MFMA, rescaled with O, instead of a per-tile cross-wave reduction
    through LDS and its barrier (examples/deepseek_mla/example_mla_decode.py, +4 % there)."""
    assert topk % block_I == 0
    if sm_scale is None:
        sm_scale = (1.0 / (dim + tail_dim))**0.5
    scale = sm_scale * LOG2E
    accum_dtype = "float"
    G = kv_group
    H = heads // G
    H_blk = block_H or min(64, max(16, H))
    assert H % H_blk == 0 or H < 16
    n_hblk = max(1, H // H_blk)
    valid_h = min(H, H_blk)
    if wide is None:
        wide = H_blk == 64  # measured: 656 TF wide vs 531 TF FullRow at the reference's shape
    use_sm = wide and (sum_mfma is None or sum_mfma)
    if threads is None:
        threads = 64 * (H_blk // 16) * (2 if wide else 1)  # FullRow: 16 head rows per wave
    # wide: 8 waves per 64-head slice -- S = Q K^T on a 4x2 wave grid, P through LDS, O = P V
    # split over D (each wave 64 of the 512 columns): half the O registers per wave, 2 waves/SIMD
    s_policy = T.GemmWarpPolicy.Square if wide else T.GemmWarpPolicy.FullRow
    D, DT = dim, tail_dim
    NI = topk // block_I
    if seq_len_kv is None:  # decode: one kernel for every cache length
        seq_len_kv = T.dynamic("seq_len_kv")
    past = seq_len_kv - seq_len
    pair_xcd = xcd_pair and n_hblk > 1 and seq_len % 8 == 0
    tau = 8.0 if lazy_rescale else 0.0

    @T.prim_func
    def main(Q: T.Tensor([batch, seq_len, heads, D + DT], dtype), KV: T.Tensor([batch, seq_len_kv, G, D + DT], dtype),
             Indices: T.Tensor([batch, seq_len, G, topk], "int32"), Output: T.Tensor([batch, seq_len, heads, D], dtype),
             Lse: T.Tensor([batch, seq_len, heads], accum_dtype)):
        with T.Kernel(seq_len * n_hblk, batch * G, threads=threads) as (pid, bz):
            if pair_xcd:
                # the head slices of one token run back to back on one XCD (block ids 8 apart:
                # workgroups go round-robin over the 8 XCDs), so the second slice's row gathers
                # hit the L2 the first one filled
                bx = (pid // (8 * n_hblk)) * 8 + pid % 8
                by = (pid // 8) % n_hblk
            else:
                bx = pid % seq_len
                by = pid // seq_len
            b = bz // G
            g = bz % G
            h0 = g * H + by * H_blk
            Q_frag = T.alloc_fragment([H_blk, D], dtype)
            Qt_frag = T.alloc_fragment([H_blk, DT], dtype)
            KV_shared = T.alloc_shared([block_I, D], dtype)
            Kt_shared = T.alloc_shared([block_I, DT], dtype)
            idx_s = T.alloc_shared([block_I], "int32")
            acc_s = T.alloc_fragment([H_blk, block_I], accum_dtype)
            acc_s_cast = T.alloc_fragment([H_blk, block_I], dtype)
            P_shared = T.alloc_shared([H_blk, block_I], dtype)
            alpha_s = T.alloc_shared([H_blk], accum_dtype)
            any_s = T.alloc_shared([2], "int32")  # wide: some row of this tile moved its max
            acc_o = T.alloc_fragment([H_blk, D], accum_dtype)
            o_cast = T.alloc_fragment([H_blk, D], dtype)
            m_cur = T.alloc_fragment([H_blk], accum_dtype)
            m_prev = T.alloc_fragment([H_blk], accum_dtype)
            alpha = T.alloc_fragment([H_blk], accum_dtype)
            l_sum = T.alloc_fragment([H_blk], accum_dtype)
            r_sum = T.alloc_fragment([H_blk], accum_dtype)

            T.clear(Q_frag)
            T.clear(Qt_frag)
            T.copy(Q[b, bx, h0:h0 + valid_h, 0:D], Q_frag[0:valid_h, :])
            T.copy(Q[b, bx, h0:h0 + valid_h, D:D + DT], Qt_frag[0:valid_h, :])
            if use_sm:
                ones_s = T.alloc_shared([block_I, 32], dtype)
                acc_l = T.alloc_fragment([H_blk, 32], accum_dtype)
                T.fill(ones_s, 1.0)
                T.clear(acc_l)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m_cur, -(2.0**30))
            # lazy-rescale flag, double-buffered by iteration parity: iteration t resets the slot
            # of t + 1 (ordered by the stage barrier against t - 1's readers and t + 1's setters)
            for z in T.Parallel(2):
                any_s[z] = 0
            for i in T.Pipelined(NI, num_stages=num_stages):
                # selected latent rows; indices outside the cache read zeros, causal ones are masked
                T.gather_rows(KV[b, :, g, 0:D], Indices[b, bx, g, i * block_I:(i + 1) * block_I], KV_shared)
                T.gather_rows(KV[b, :, g, D:D + DT], Indices[b, bx, g, i * block_I:(i + 1) * block_I], Kt_shared)
                T.copy(Indices[b, bx, g, i * block_I:(i + 1) * block_I], idx_s)  # prefetched a step ahead
                for h, r in T.Parallel(H_blk, block_I):
                    acc_s[h, r] = T.if_then_else((idx_s[r] <= bx + past) & (idx_s[r] >= 0), 0,
                                                 -T.infinity(accum_dtype))
                T.gemm(Q_frag, KV_shared, acc_s, transpose_B=True, policy=s_policy)
                T.gemm(Qt_frag, Kt_shared, acc_s, transpose_B=True, policy=s_policy)
                if wide:
                    for z in T.Parallel(1):  # previous tile's readers are past the stage barrier
                        any_s[z + (i + 1) % 2] = 0
                T.copy(m_cur, m_prev)
                T.reduce_max(acc_s, m_prev, dim=1, clear=False)
                # lazy rescale: a row keeps its running max until a new score exceeds it by
                # more than 2^8 (P <= 256 stays exact enough in fp32 / bf16), so after the
                # first tiles the 128-register O accumulator is almost never rescaled
                rescale = T.alloc_var("int32")
                rescale = 0
                for h in T.Parallel(H_blk):
                    if (m_prev[h] - m_cur[h]) * scale > tau:
                        alpha[h] = T.exp2((m_cur[h] - m_prev[h]) * scale)
                        m_cur[h] = m_prev[h]
                        rescale = 1
                        if wide:
                            any_s[i % 2] = 1
                    else:
                        alpha[h] = 1.0
                for h, r in T.Parallel(H_blk, block_I):
                    acc_s[h, r] = T.exp2(acc_s[h, r] * scale - m_cur[h] * scale)
                if not use_sm:
                    T.reduce_sum(acc_s, r_sum, dim=1)
                    for h in T.Parallel(H_blk):
                        l_sum[h] = l_sum[h] * alpha[h] + r_sum[h]
                if wide:
                    # O is partitioned over D, not over heads: alpha reaches its waves through LDS
                    T.copy(alpha, alpha_s)
                    T.copy(acc_s, P_shared)
                    # lazy rescale across the D-split waves: skipped (block-uniform flag) on the
                    # tiles where no row moved its max -- most of them after the first few
                    if any_s[i % 2] != 0:
                        for h, d in T.Parallel(H_blk, D):
                            acc_o[h, d] *= alpha_s[h]
                        if use_sm:
                            for h, j in T.Parallel(H_blk, 32):
                                acc_l[h, j] *= alpha_s[h]
                    T.gemm(P_shared, KV_shared, acc_o)
                    if use_sm:
                        T.gemm(P_shared, ones_s, acc_l)
                else:
                    if rescale != 0:  # per-thread flag: waves whose rows all kept their max skip it
                        for h, d in T.Parallel(H_blk, D):
                            acc_o[h, d] *= alpha[h]
                    T.copy(acc_s, acc_s_cast)
                    T.gemm(acc_s_cast, KV_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            if use_sm:
                for h, j in T.Parallel(H_blk, 32):  # every column of P x ones is the row sum
                    if j == 0:
                        alpha_s[h] = acc_l[h, j]
                for h in T.Parallel(H_blk):
                    l_sum[h] = alpha_s[h]
                for h, d in T.Parallel(H_blk, D):
                    o_cast[h, d] = acc_o[h, d] / alpha_s[h]
            elif wide:
                T.copy(l_sum, alpha_s)
                for h, d in T.Parallel(H_blk, D):
                    o_cast[h, d] = acc_o[h, d] / alpha_s[h]
            else:
                for h, d in T.Parallel(H_blk, D):
                    o_cast[h, d] = acc_o[h, d] / l_sum[h]
            for h in T.Parallel(H_blk):
                l_sum[h] = T.log2(l_sum[h]) + m_cur[h] * scale
            if staged_out:
                # the token's O rows leave as contiguous 16-byte row stores from a row-padded LDS
                # tile (the gathered-KV ring's bytes, dead after the loop): 756 -> 767 TF at the
                # reference's benchmark shape (profiles/r5/smla_epi/ab.log)
                O_s = T.alloc_shared([H_blk, D], dtype)
                T.annotate_layout({O_s: PaddedLayout((H_blk, D), 8)})
                T.copy(o_cast, O_s)
                T.copy(O_s[0:valid_h, :], Output[b, bx, h0:h0 + valid_h, :])
            else:
                T.copy(o_cast[0:valid_h, :], Output[b, bx, h0:h0 + valid_h, :])
            T.copy(l_sum[0:valid_h], Lse[b, bx, h0:h0 + valid_h])

    return main


@tilelang.jit(out_idx=[3])
def mqa_attn_return_logits(seq_len, seq_len_kv, heads, index_dim, block_N=128, threads=512, block_Q=None):
    """Lightning-indexer logits.  One block per ``block_Q`` query tokens (K tiles reused across
    them); per token and KV tile: S = K Q_t^T [block_N x heads] on the fp8 MFMA (FullRow: each
    wave owns whole key rows), relu * head weight in registers, then the sum over heads as an
    in-wave row reduction, and the key scale applied once per (token, key) after the sum
    (``k_scale[n]`` factors out of the head sum).  Before: the weighted scores went through LDS
    and one lane per (token, key) summed its heads serially."""
    if block_Q is None:
        block_Q = max(1, 128 // heads)
    if seq_len_kv is None:
        seq_len_kv = T.dynamic("seq_len_kv")
    dtype = "float8_e4m3fn"
    accum_dtype = "float"

    @T.prim_func
    def main(IndexQ: T.Tensor([seq_len * heads, index_dim], dtype), IndexK: T.Tensor([seq_len_kv, index_dim], dtype),
             IndexKScale: T.Tensor([seq_len_kv], accum_dtype), Logits: T.Tensor([seq_len, seq_len_kv], accum_dtype),
             Weights: T.Tensor([seq_len, heads], accum_dtype), CuSeqLenKS: T.Tensor([seq_len], "int32"),
             CuSeqLenKE: T.Tensor([seq_len], "int32")):
        with T.Kernel(T.ceildiv(seq_len, block_Q), threads=threads) as bx:
            q_s = [T.alloc_shared([heads, index_dim], dtype) for _ in range(block_Q)]
            k_shared = T.alloc_shared([block_N, index_dim], dtype)
            ks_shared = T.alloc_shared([block_N], accum_dtype)
            w_shared = T.alloc_shared([block_Q, heads], accum_dtype)
            s = [T.alloc_fragment([block_N, heads], accum_dtype) for _ in range(block_Q)]
            r = [T.alloc_fragment([block_N], accum_dtype) for _ in range(block_Q)]
            q0 = bx * block_Q
            for bq in list(range(block_Q)):  # trace-time unrolled (a plain range becomes a DSL loop)
                T.copy(IndexQ[(q0 + bq) * heads, 0], q_s[bq])
            T.copy(Weights[q0, 0], w_shared)
            for nb in T.Pipelined(T.ceildiv(seq_len_kv, block_N), num_stages=2):
                T.copy(IndexK[nb * block_N, 0], k_shared)
                T.copy(IndexKScale[nb * block_N], ks_shared)
                for bq in list(range(block_Q)):
                    T.clear(s[bq])
                    T.gemm(k_shared, q_s[bq], s[bq], transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                    for n, h in T.Parallel(block_N, heads):
                        s[bq][n, h] = T.max(s[bq][n, h], 0) * w_shared[bq, h]
                    T.reduce_sum(s[bq], r[bq], dim=1)
                    for n in T.Parallel(block_N):
                        kv_pos = nb * block_N + n
                        Logits[q0 + bq, kv_pos] = T.if_then_else(
                            (kv_pos >= CuSeqLenKS[q0 + bq]) & (kv_pos < CuSeqLenKE[q0 + bq]), r[bq][n] * ks_shared[n],
                            -T.infinity(accum_dtype))

    return main


@tilelang.jit(out_idx=[1])
def topk_selector(M, N, topk, threads=256):
    assert N % threads == 0

    @T.prim_func
    def main(Scores: T.Tensor([M, N], "float32"), Indices: T.Tensor([M, topk], "int32")):
        with T.Kernel(M, threads=threads) as r:
            keys = T.alloc_fragment([1, N], "int64")
            hit = T.alloc_fragment([1, N], "int32")
            cnt = T.alloc_fragment([1], "int32")
            lo = T.alloc_var("int64")
            hi = T.alloc_var("int64")
            mid = T.alloc_var("int64")
            pos = T.alloc_shared([2], "int32")
            for z, j in T.Parallel(1, N):
                bits = T.Cast("int64", T.reinterpret(Scores[r, j], "int32"))
                keys[z, j] = T.if_then_else(bits >= 0, bits + 2147483648, 2147483647 - (bits & 2147483647))
            lo = 0
            hi = 4294967295
            for _ in T.serial(32):
                mid = (lo + hi + 1) // 2
                for z, j in T.Parallel(1, N):
                    hit[z, j] = T.if_then_else(keys[z, j] >= mid, 1, 0)
                T.reduce_sum(hit, cnt, dim=1)
                if cnt[0] >= topk:
                    lo = mid
                else:
                    hi = mid - 1
            # lo is the key of the k-th largest value: take everything above it, then fill
            # the remaining slots with entries equal to it
            for z, j in T.Parallel(1, N):
                hit[z, j] = T.if_then_else(keys[z, j] > lo, 1, 0)
            T.reduce_sum(hit, cnt, dim=1)
            pos[0] = 0
            pos[1] = cnt[0]
            T.sync_threads()
            for z, j in T.Parallel(1, N):
                if keys[z, j] > lo:
                    slot_gt = T.atomic_add(pos[0], 1, return_prev=True)
                    Indices[r, slot_gt] = j
                elif keys[z, j] == lo:
                    slot = T.atomic_add(pos[1], 1, return_prev=True)
                    if slot < topk:
                        Indices[r, slot] = j

    return main


@functools.lru_cache(maxsize=None)
def for_target(name: str, target: str, *args):
    """The kernel ``name`` (one of this module's jit functions) compiled for ``target`` ("hip" /
    "cpu"): the model runs the same shapes on either device, the jit cache keys on shapes only."""
    impl = globals()[name]
    return tilelang.compile(impl.get_tir(*args), out_idx=impl.out_idx, target=target)
