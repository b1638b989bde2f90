"""Persistent FlashAttention forward (reference: examples/amd/example_amd_flash_attn_fwd.py).

``num_split_q`` workgroups per (batch, head) walk the query tiles with a ``T.While`` loop
instead of one workgroup per tile: the grid stays resident (one 8-wave workgroup per CU), and each
workgroup's K/V stream (LDS-DMA ring) moves on to its next query tile without a relaunch.  Tiles
are dealt in cost order along a snake, so causal heads are balanced exactly (see fast_flashattn).
The tile body is the staged FA kernel of examples/flash_attention/example_mha_fwd_pipelined.py
(T.Pipelined order/stage/group: QK^T(t) next to rescale + PV(t-1)): Q in registers, P kept in
registers as the PV operand, lazy rescale, fast exp2.
"""
import argparse

import tilelang
import tilelang.language as T

FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}


@tilelang.jit(out_idx=[3], pass_configs=FAST_MATH)
def fast_flashattn(batch, heads, seq_len, dim, is_causal=False, groups=1, block_M=256, block_N=64, num_split_q=None,
                   threads=512, num_stages=2, dtype="float16", mfma="16x16", unroll=2):
    """``num_split_q`` resident workgroups per (batch, head) (default: enough to put one 8-wave
    workgroup on each of the 256 CUs).  Work assignment in cost order: query tiles are ranked
    longest-first (causal: the last tiles see the most keys) and dealt to the workgroups of a head
    in a snake (``s, 2S-1-s, 2S+s, ...``), so every workgroup of a causal head gets the same number
    of KV blocks (tile pairs (i, n-1-i)) and no CU idles at the end.  ``unroll``: the KV loop is
    emitted twice per trip (constant LDS ring slots): 506 -> 539 TF at b1 h8 s4096 d128
    (profiles/r6/unroll_sweep_examples.log)."""
    scale = (1.0 / dim)**0.5 * 1.44269504
    head_kv = heads // groups
    q_shape = [batch, seq_len, heads, dim]
    kv_shape = [batch, seq_len, head_kv, dim]
    accum_dtype = "float"
    num_q_blocks = (seq_len + block_M - 1) // block_M
    # key-padding mask on the last KV tile when seq_len is not a multiple of block_N (reference
    # examples/flash_attention/example_mha_fwd_bshd.py:54); causal rows never see those keys
    ragged_kv = seq_len % block_N != 0 and not is_causal
    if num_split_q is None:  # one resident 8-wave workgroup per CU over the whole grid
        num_split_q = max(1, min(num_q_blocks, 256 // max(1, batch * heads)))
    group = [[0], [1, 2], list(range(3, 11)), [11], [12], [13]]  # as example_mha_fwd_pipelined

    @T.prim_func
    def main(Q: T.Tensor(q_shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(kv_shape, dtype),
             Output: T.Tensor(q_shape, dtype)):
        with T.Kernel(num_split_q, batch * heads, threads=threads) as (b_split, byz):
            bz = byz // heads
            by = byz % heads
            Q_r = T.alloc_fragment([block_M, dim], dtype)
            K_shared = T.alloc_shared([block_N, dim], dtype)
            V_shared = T.alloc_shared([block_N, dim], dtype)
            acc_s = T.alloc_fragment([block_M, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_M, block_N], dtype)
            acc_o = T.alloc_fragment([block_M, dim], accum_dtype)
            m_i = T.alloc_fragment([block_M], accum_dtype)
            m_prev = T.alloc_fragment([block_M], accum_dtype)
            alpha = T.alloc_fragment([block_M], accum_dtype)
            l_i = T.alloc_fragment([block_M], accum_dtype)
            r_sum = T.alloc_fragment([block_M], accum_dtype)
            rescale = T.alloc_var("int32")
            it = T.alloc_var("int32")
            it = 0
            while it < num_q_blocks:
                # snake over the cost-ranked tiles: rank r = it + (s | 2S-1-s), tile = n-1-r (causal)
                r = T.if_then_else((it // num_split_q) % 2 == 0, it + b_split, it + num_split_q - 1 - b_split)
                # clamped so the bounds prover sees the K/V tiles in range (LDS-DMA, not register staging)
                bx = T.max(T.min((num_q_blocks - 1 - r) if is_causal else r, num_q_blocks - 1), 0)
                if r < num_q_blocks:
                    T.copy(Q[bz, bx * block_M:(bx + 1) * block_M, by, :], Q_r)
                    T.fill(acc_o, 0)
                    T.fill(l_i, 0)
                    T.fill(m_i, -(2.0**30))
                    rescale = 1
                    loop_end = (T.min(T.ceildiv((bx + 1) * block_M, block_N), T.ceildiv(seq_len, block_N))
                                if is_causal else T.ceildiv(seq_len, block_N))
                    for k in T.Pipelined(loop_end, num_stages=num_stages, order=[-1, 0, 3, 1, -1, 2],
                                         stage=[-1, 0, 0, 1, -1, 1], group=group, unroll=unroll):
                        T.copy(K[bz, k * block_N:(k + 1) * block_N, by // groups, :], K_shared)
                        if is_causal:
                            if (k + 1) * block_N <= bx * block_M + 1:  # block fully visible: no mask
                                T.clear(acc_s)
                            else:
                                for i, j in T.Parallel(block_M, block_N):
                                    acc_s[i, j] = T.if_then_else(bx * block_M + i >= k * block_N + j, 0,
                                                                 -T.infinity(accum_dtype))
                        elif ragged_kv:
                            if k == loop_end - 1:
                                for i, j in T.Parallel(block_M, block_N):
                                    acc_s[i, j] = T.if_then_else(k * block_N + j < seq_len, 0,
                                                                 -T.infinity(accum_dtype))
                            else:
                                T.clear(acc_s)
                        else:
                            T.clear(acc_s)
                        T.gemm(Q_r, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow,
                               mfma_shape=mfma)
                        # softmax (lazy rescale: a row keeps its max until exceeded by 2^8)
                        T.copy(m_i, m_prev)
                        T.reduce_max(acc_s, m_prev, dim=1, clear=False)
                        rescale = 0
                        for i in T.Parallel(block_M):
                            if (m_prev[i] - m_i[i]) * scale > 8.0:
                                alpha[i] = T.exp2((m_i[i] - m_prev[i]) * scale)
                                m_i[i] = m_prev[i]
                                rescale = 1
                            else:
                                alpha[i] = 1.0
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m_i[i] * scale)
                        T.reduce_sum(acc_s, r_sum, dim=1)
                        for i in T.Parallel(block_M):
                            l_i[i] = l_i[i] * alpha[i] + r_sum[i]
                        T.copy(acc_s, acc_s_cast)
                        # one tile behind: rescale O, then O += P V
                        if rescale != 0:
                            for i, j in T.Parallel(block_M, dim):
                                acc_o[i, j] *= alpha[i]
                        T.copy(V[bz, k * block_N:(k + 1) * block_N, by // groups, :], V_shared)
                        T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow, mfma_shape=mfma)
                    for i, j in T.Parallel(block_M, dim):
                        acc_o[i, j] /= T.max(l_i[i], 1e-30)
                    T.copy(acc_o, Output[bz, bx * block_M:(bx + 1) * block_M, by, :])
                it = it + num_split_q

    return main


def ref_program(Q, K, V, is_causal, groups=1):
    import math
    import torch
    import torch.nn.functional as F
    dim = Q.size(-1)
    K = K.repeat_interleave(groups, dim=2)
    V = V.repeat_interleave(groups, dim=2)
    scores = torch.einsum("bqhd,bkhd->bhqk", Q.float(), K.float()) / math.sqrt(dim)
    if is_causal:
        s = Q.size(1)
        scores = scores.masked_fill(torch.tril(torch.ones(s, s, device=Q.device)) == 0, float("-inf"))
    return torch.einsum("bhqk,bkhd->bqhd", F.softmax(scores, -1), V.float()).to(Q.dtype)


def main(batch=1, heads=8, seq_len=4096, dim=128, is_causal=False, groups=1):
    import torch
    flops = 4.0 * batch * heads * seq_len * seq_len * dim * (0.5 if is_causal else 1.0)
    kernel = fast_flashattn(batch, heads, seq_len, dim, is_causal, groups)
    q = torch.randn(batch, seq_len, heads, dim, device="cuda", dtype=torch.float16)
    k = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.float16)
    v = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.float16)
    o = kernel(q, k, v)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, is_causal, groups).float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v))
    print(f"persistent flash attention fwd: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=8)
    p.add_argument("--seq_len", type=int, default=4096)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--is_causal", action="store_true")
    p.add_argument("--groups", type=int, default=1)
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_len, a.dim, a.is_causal, a.groups)
