"""FlashAttention-2 forward (reference: examples/flash_attention/example_mha_fwd_bshd.py,
examples/amd/example_amd_flash_attn_fwd.py) on MI355X.

Layout: Q/K/V/O are [batch, seq, heads, dim] (bshd).  One block computes ``block_M`` query
rows of one head; K/V tiles stream through a 2-stage LDS-DMA ring.  With
``policy=FullRow`` every wave owns whole rows of S = Q K^T, so the row softmax needs only
in-wave lane shuffles and P stays in registers: the accumulator layout of the first GEMM
*is* the (k-permuted) A-operand layout of the second, and V is read with
``ds_read_b64_tr_b16`` in the matching order.
"""
import argparse
import math

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}
# + no NaNs (-fno-honor-nans): the row max takes MFMA results straight into v_max_f32 (masked
# scores are -inf, never NaN, and every query row sees at least one unmasked key)
FAST_MATH_NO_NANS = {**FAST_MATH, tilelang.PassConfigKey.TL_NO_NANS: True,
                     # the unfolded wave guard: 0-4 % faster in this loop (scripts/guard_fold_ab.py, two runs)
                     tilelang.PassConfigKey.TL_GEMM_FOLD_DEFAULT_GUARD: False}


@tilelang.jit(out_idx=[3], pass_configs=FAST_MATH_NO_NANS)
def flashattn(batch, heads, seq_len, dim, is_causal=False, groups=1, block_M=128, block_N=64, threads=256,
              num_stages=2, dtype="bfloat16", lazy_rescale=True, q_in_regs=False):
    """``lazy_rescale``: a row keeps its running max until a new score exceeds it by 2^8, so the
    O accumulator is rescaled only on those (rare, after the first tiles) steps; a wave skips
    the rescale when none of its rows moved.  ``q_in_regs``: Q is loaded once into the MFMA
    A-operand registers of the wave that owns its rows (no per-tile LDS re-read of Q, and the
    LDS it used goes to deeper K/V staging)."""
    scale = (1.0 / dim)**0.5 * 1.44269504  # log2(e): softmax via exp2
    head_kv = heads // groups
    q_shape = [batch, seq_len, heads, dim]
    kv_shape = [batch, seq_len, head_kv, dim]
    accum_dtype = "float"
    # keys at or past seq_len in a ragged last KV tile are masked to -inf (reference
    # example_mha_fwd_bshd.py:54); causal rows never see them
    ragged_kv = seq_len % block_N != 0 and not is_causal

    @T.prim_func
    def main(
            Q: T.Tensor(q_shape, dtype),
            K: T.Tensor(kv_shape, dtype),
            V: T.Tensor(kv_shape, dtype),
            Output: T.Tensor(q_shape, dtype),
    ):
        with T.Kernel(T.ceildiv(seq_len, block_M), heads, batch, threads=threads) as (bx, by, bz):
            if q_in_regs:
                Q_shared = T.alloc_fragment([block_M, dim], dtype)
            else:
                Q_shared = T.alloc_shared([block_M, dim], dtype)
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

            T.copy(Q[bz, bx * block_M:(bx + 1) * block_M, by, :], Q_shared)
            T.fill(acc_o, 0)
            T.fill(logsum, 0)
            if lazy_rescale:
                T.fill(scores_max, -(2.0**30))  # finite: a fully masked tile keeps it (no inf - inf)
            else:
                T.fill(scores_max, -T.infinity(accum_dtype))

            # the causal range stops at the last key tile (a ragged last query tile would run past it)
            loop_range = (T.min(T.ceildiv((bx + 1) * block_M, block_N), T.ceildiv(seq_len, block_N))
                          if is_causal else T.ceildiv(seq_len, block_N))

            for k in T.Pipelined(loop_range, num_stages=num_stages):
                T.copy(K[bz, k * block_N:(k + 1) * block_N, by // groups, :], K_shared)
                if is_causal:
                    for i, j in T.Parallel(block_M, block_N):
                        acc_s[i, j] = T.if_then_else(bx * block_M + i >= k * block_N + j, 0,
                                                     -T.infinity(acc_s.dtype))
                elif ragged_kv:  # key-padding mask on the last KV tile only (uniform branch)
                    if k == loop_range - 1:
                        for i, j in T.Parallel(block_M, block_N):
                            acc_s[i, j] = T.if_then_else(k * block_N + j < seq_len, 0, -T.infinity(acc_s.dtype))
                    else:
                        T.clear(acc_s)
                else:
                    T.clear(acc_s)
                T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(V[bz, k * block_N:(k + 1) * block_N, by // groups, :], V_shared)
                T.copy(scores_max, scores_max_prev)
                if lazy_rescale:
                    T.reduce_max(acc_s, scores_max_prev, dim=1, clear=False)  # candidate max
                    rescale = T.alloc_var("int32")
                    rescale = 0
                    for i in T.Parallel(block_M):
                        if (scores_max_prev[i] - scores_max[i]) * scale > 8.0:
                            scores_scale[i] = T.exp2((scores_max[i] - scores_max_prev[i]) * scale)
                            scores_max[i] = scores_max_prev[i]
                            rescale = 1
                        else:
                            scores_scale[i] = 1.0
                    if rescale != 0:
                        for i, j in T.Parallel(block_M, dim):
                            acc_o[i, j] *= scores_scale[i]
                else:
                    T.reduce_max(acc_s, scores_max, dim=1, clear=False)
                    for i in T.Parallel(block_M):
                        scores_scale[i] = T.exp2(scores_max_prev[i] * scale - scores_max[i] * scale)
                    for i, j in T.Parallel(block_M, dim):
                        acc_o[i, j] *= scores_scale[i]
                for i, j in T.Parallel(block_M, block_N):
                    acc_s[i, j] = T.exp2(acc_s[i, j] * scale - scores_max[i] * scale)
                T.reduce_sum(acc_s, scores_sum, dim=1)
                for i in T.Parallel(block_M):
                    logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for i, j in T.Parallel(block_M, dim):
                acc_o[i, j] /= logsum[i]
            T.copy(acc_o, Output[bz, bx * block_M:(bx + 1) * block_M, by, :])

    return main


def ref_program(Q, K, V, is_causal=False, groups=1):
    import torch
    import torch.nn.functional as F
    dim = Q.size(-1)
    K = K.repeat_interleave(groups, dim=2)
    V = V.repeat_interleave(groups, dim=2)
    scores = torch.einsum("bqhd,bkhd->bhqk", Q.float(), K.float()) / math.sqrt(dim)
    if is_causal:
        s = Q.size(1)
        mask = torch.tril(torch.ones(s, s, device=scores.device))
        scores = scores.masked_fill(mask == 0, float("-inf"))
    p = F.softmax(scores, dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, V.float()).to(Q.dtype)


def main(batch=1, heads=8, seq_len=4096, dim=128, is_causal=False, groups=1):
    import torch
    flops = 4.0 * batch * heads * seq_len * seq_len * dim * (0.5 if is_causal else 1.0)
    kernel = flashattn(batch, heads, seq_len, dim, is_causal, groups)
    q = torch.randn(batch, seq_len, heads, dim, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.bfloat16)
    o = kernel(q, k, v)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, is_causal, groups).float(), rtol=2e-2, atol=2e-2)
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v))
    print(f"flash attention fwd: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


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
