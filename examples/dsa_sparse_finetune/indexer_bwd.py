"""Backward of the DSA indexer's KL loss (reference: examples/dsa_sparse_finetune/indexer_bwd.py).

loss_t = KL(attn_score_t || softmax(index logits over the top-k of t)), so the gradient at the
selected logit i is ``index_score_i - attn_score_i``; through logit_i = sum_h w_h relu(q_h . k_i * s):

    dw_h  += sum_i g_i relu_ih,      dqk_ih = g_i [relu_ih > 0] w_h
    dq_h  += s * sum_i dqk_ih k_i,   dk_i  += s * sum_h dqk_ih q_h   (fp32 atomics: keys are shared)

One block per packed token walks its top-k in 32-key tiles (rows gathered straight from global).
dq and dw are produced whole; dk is scattered with fp32 atomics into a zeroed fp32 buffer.
"""
import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[6, 7])
def indexer_bwd(seq_len, heads, dim, topk, sm_scale=None, block_I=32, threads=128, dtype="bfloat16"):
    scale = dim**-0.5 if sm_scale is None else sm_scale
    assert topk % block_I == 0 and heads % 16 == 0
    NI = topk // block_I

    @T.prim_func
    def main(IndexQ: T.Tensor([seq_len, heads, dim], dtype), Weights: T.Tensor([seq_len, heads], dtype),
             IndexK: T.Tensor([seq_len, dim], dtype), AttnScore: T.Tensor([seq_len, topk], "float32"),
             IndexScore: T.Tensor([seq_len, topk], "float32"), Idx: T.Tensor([seq_len, topk], "int32"),
             dIndexQ: T.Tensor([seq_len, heads, dim], dtype), dWeights: T.Tensor([seq_len, heads], "float32"),
             dIndexK: T.Tensor([seq_len, dim], "float32")):
        with T.Kernel(seq_len, threads=threads) as t:
            q_s = T.alloc_shared([heads, dim], dtype)
            qf_s = T.alloc_shared([heads, dim], "float32")
            w_s = T.alloc_shared([heads], "float32")
            k_s = T.alloc_shared([block_I, dim], dtype)
            g_s = T.alloc_shared([block_I], "float32")
            idx_s = T.alloc_shared([block_I], "int32")
            dqk_s = T.alloc_shared([block_I, heads], dtype)
            dqkf_s = T.alloc_shared([block_I, heads], "float32")
            rw_s = T.alloc_shared([block_I, heads], "float32")
            dw_s = T.alloc_shared([heads], "float32")
            lg = T.alloc_fragment([block_I, heads], "float32")
            dq = T.alloc_fragment([heads, dim], "float32")
            dk = T.alloc_fragment([block_I, dim], "float32")
            for h, d in T.Parallel(heads, dim):
                v = T.cast(IndexQ[t, h, d], "float32") * scale
                q_s[h, d] = v
                qf_s[h, d] = v
            for h in T.Parallel(heads):
                w_s[h] = T.cast(Weights[t, h], "float32")
                dw_s[h] = 0.0
            T.clear(dq)
            for ib in T.serial(NI):
                for i in T.Parallel(block_I):
                    idx = Idx[t, ib * block_I + i]
                    ok = (idx >= 0) & (idx <= t)
                    idx_s[i] = T.if_then_else(ok, idx, -1)
                    g_s[i] = T.if_then_else(ok, IndexScore[t, ib * block_I + i] - AttnScore[t, ib * block_I + i], 0.0)
                for i, d in T.Parallel(block_I, dim):
                    k_s[i, d] = T.if_then_else(idx_s[i] >= 0, IndexK[T.max(idx_s[i], 0), d], 0)
                T.clear(lg)
                T.gemm(k_s, q_s, lg, transpose_B=True)
                for i, h in T.Parallel(block_I, heads):
                    r = T.max(lg[i, h], 0)
                    rw_s[i, h] = g_s[i] * r
                    v = T.if_then_else(r > 0, g_s[i] * w_s[h], 0.0)
                    dqk_s[i, h] = v
                    dqkf_s[i, h] = v
                for h in T.Parallel(heads):
                    acc = T.alloc_var("float32")
                    acc = 0.0
                    for i in T.serial(block_I):
                        acc = acc + rw_s[i, h]
                    dw_s[h] = dw_s[h] + acc
                T.gemm(dqk_s, k_s, dq, transpose_A=True)
                T.clear(dk)
                T.gemm(dqkf_s, qf_s, dk)
                for i, d in T.Parallel(block_I, dim):
                    if idx_s[i] >= 0:
                        T.atomic_add(dIndexK[idx_s[i], d], dk[i, d])
            for h, d in T.Parallel(heads, dim):
                dq[h, d] = dq[h, d] * scale
            T.copy(dq, dIndexQ[t, :, :])
            for h in T.Parallel(heads):
                dWeights[t, h] = dw_s[h]

    return main


def indexer_bwd_interface(q, weights, k, attn_score, index_score, idx_abs, sm_scale=None):
    """(dq [S,H,D] in q's dtype, dweights fp32 [S,H], dk fp32 [S,D])."""
    import torch
    S, H, D = q.shape
    dk = torch.zeros(S, D, dtype=torch.float32, device=q.device)
    dq, dw = indexer_bwd(S, H, D, idx_abs.shape[-1], sm_scale)(q, weights.to(q.dtype), k, attn_score, index_score,
                                                               idx_abs, dk)
    return dq, dw, dk
