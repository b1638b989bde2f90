"""DSA indexer for sparse fine-tuning: index scores, top-k selection and the top-k softmax
(reference: examples/dsa_sparse_finetune/indexer_topk_reducesum.py).

For packed token t (sequence start ``bos``) and every key n of its sequence with n <= t:

    logit[t, n] = scale * sum_h w[t, h] relu(q[t, h] . k[n])           (bf16 MFMA, fp32 sum)
    idx[t, :]   = top-k positions of logit[t, :]                       (library topk_selector)
    score[t, :] = softmax(logit[t, idx[t, :]])                          (unselectable: score 0, idx -1)

MI355X decomposition (the reference fuses everything with a bitonic merge per token):
``index_logits`` -- one block per ``128 / H`` tokens makes the (tokens x heads) rows the MFMA N
dimension against 64-key K tiles streamed by LDS-DMA, then reduces the heads through LDS;
``topk_selector`` -- exact bisection on the fp32 bit pattern, the row in registers
(tilelang.ops.dsa); ``topk_softmax`` -- one wave-sized block per token gathers the k logits.
Indices come back relative to the sequence (as the reference) and absolute (packed) for the
sparse MLA kernels.
"""
import math

import tilelang
import tilelang.language as T

from index import prepare_token_indices  # noqa: F401  (re-exported for callers)


@tilelang.jit(out_idx=[5])
def index_logits(seq_len, heads, dim, block_N=64, threads=256, sm_scale=None, dtype="bfloat16"):
    """Indexer logits of ``block_Q`` query tokens per block: per token, S = K Q_t^T [block_N x
    heads] (FullRow MFMA: whole key rows per wave), relu * weight, and the head sum as an in-wave
    row reduction (the scores used to go through LDS and one lane per (token, key) summed its heads
    serially -- the same change took the fp8 lightning indexer from 282 to ~1.4 PF)."""
    block_Q = max(1, 128 // heads)
    scale = dim**-0.5 if sm_scale is None else sm_scale

    @T.prim_func
    def main(IndexQ: T.Tensor([seq_len * heads, dim], dtype), IndexK: T.Tensor([seq_len, dim], dtype),
             Weights: T.Tensor([seq_len, heads], dtype), Offsets: T.Tensor([seq_len + 1], "int32"),
             TokenIndices: T.Tensor([seq_len, 2], "int32"), Logits: T.Tensor([seq_len, seq_len], "float32")):
        with T.Kernel(T.ceildiv(seq_len, block_Q), threads=threads) as bx:
            q_s = [T.alloc_shared([heads, dim], dtype) for _ in range(block_Q)]
            k_s = T.alloc_shared([block_N, dim], dtype)
            s = [T.alloc_fragment([block_N, heads], "float32") for _ in range(block_Q)]
            r = [T.alloc_fragment([block_N], "float32") for _ in range(block_Q)]
            w_s = T.alloc_shared([block_Q, heads], "float32")
            lo_s = T.alloc_shared([block_Q], "int32")
            q0 = bx * block_Q
            for bq in list(range(block_Q)):  # trace-time unrolled (a plain range becomes a DSL loop)
                T.copy(IndexQ[(q0 + bq) * heads, 0], q_s[bq])
            for u, h in T.Parallel(block_Q, heads):
                t = T.min(q0 + u, seq_len - 1)
                w_s[u, h] = T.cast(Weights[t, h], "float32") * scale
            for u in T.Parallel(block_Q):
                t = T.min(q0 + u, seq_len - 1)
                lo_s[u] = Offsets[TokenIndices[t, 0]]
            t_hi = T.min(q0 + block_Q, seq_len) - 1
            for nb in T.Pipelined(T.ceildiv(seq_len, block_N), num_stages=2):
                T.copy(IndexK[nb * block_N, 0], k_s)
                if nb * block_N <= t_hi:
                    for bq in list(range(block_Q)):
                        T.clear(s[bq])
                        T.gemm(k_s, q_s[bq], s[bq], transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                        for n, h in T.Parallel(block_N, heads):
                            s[bq][n, h] = T.max(s[bq][n, h], 0) * w_s[bq, h]
                        T.reduce_sum(s[bq], r[bq], dim=1)
                        for n in T.Parallel(block_N):
                            key = nb * block_N + n
                            if (q0 + bq < seq_len) & (key < seq_len):
                                Logits[q0 + bq, key] = T.if_then_else((key >= lo_s[bq]) & (key <= q0 + bq),
                                                                      r[bq][n], -T.infinity("float32"))
                else:  # every key of the tile is after every query of the block: causally masked
                    for u, n in T.Parallel(block_Q, block_N):
                        key = nb * block_N + n
                        if (q0 + u < seq_len) & (key < seq_len):
                            Logits[q0 + u, key] = -T.infinity("float32")

    return main


@tilelang.jit(out_idx=[3, 4, 5], pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def topk_softmax(seq_len, N, topk, threads=64):
    """Selected logits -> softmax; picks of masked keys (logit -inf) get score 0 and index -1."""

    @T.prim_func
    def main(Logits: T.Tensor([seq_len, N], "float32"), Idx: T.Tensor([seq_len, topk], "int32"),
             Bos: T.Tensor([seq_len], "int32"), IdxRel: T.Tensor([seq_len, topk], "int32"),
             IdxAbs: T.Tensor([seq_len, topk], "int32"), Score: T.Tensor([seq_len, topk], "float32")):
        with T.Kernel(seq_len, threads=threads) as t:
            lv = T.alloc_fragment([1, topk], "float32")
            v = T.alloc_fragment([1, topk], "float32")
            mx = T.alloc_fragment([1], "float32")
            sm = T.alloc_fragment([1], "float32")
            for z, i in T.Parallel(1, topk):
                lv[z, i] = Logits[t, Idx[t, i]]
            T.reduce_max(lv, mx, dim=1)
            for z, i in T.Parallel(1, topk):
                v[z, i] = T.if_then_else(lv[z, i] > -T.infinity("float32"), T.exp(lv[z, i] - mx[0]), 0.0)
            T.reduce_sum(v, sm, dim=1)
            for z, i in T.Parallel(1, topk):
                ok = lv[z, i] > -T.infinity("float32")
                Score[t, i] = v[z, i] / sm[0]
                IdxAbs[t, i] = T.if_then_else(ok, Idx[t, i], -1)
                IdxRel[t, i] = T.if_then_else(ok, Idx[t, i] - Bos[t], -1)

    return main


def indexer_topk_reducesum_interface(q, weights, k, topk, offsets, return_abs=False):
    """q [S, H, D] bf16, weights [S, H], k [S, D], offsets [B+1] -> (topk_indices [S, topk]
    relative to the sequence (-1 = none), topk_score [S, topk] fp32)."""
    import torch
    from tilelang.ops.dsa import topk_selector
    S, H, D = q.shape
    tok = prepare_token_indices(offsets)
    offs = torch.zeros(S + 1, dtype=torch.int32, device=q.device)
    offs[:offsets.numel()] = offsets.to(torch.int32)
    logits = index_logits(S, H, D)(q.reshape(S * H, D).contiguous(), k, weights.to(q.dtype), offs, tok)
    n_pad = int(math.ceil(S / 256) * 256)
    if n_pad != S:
        logits = torch.nn.functional.pad(logits, (0, n_pad - S), value=float("-inf"))
    idx = topk_selector(S, n_pad, topk)(logits.contiguous())
    bos = offsets.to(torch.int32)[tok[:, 0].long()].contiguous()
    idx_rel, idx_abs, score = topk_softmax(S, n_pad, topk)(logits, idx, bos)
    return (idx_rel, score, idx_abs) if return_abs else (idx_rel, score)


def ref_index_score(q, weights, k, topk, offsets):
    """fp32 reference: same logits; top-k by torch.topk (ties may pick different positions)."""
    import torch
    out_idx, out_score = [], []
    for i in range(offsets.numel() - 1):
        a, b = int(offsets[i]), int(offsets[i + 1])
        qq, kk, ww = q[a:b].float(), k[a:b].float(), weights[a:b].float()
        s = b - a
        logits = torch.einsum("thd,nd->thn", qq, kk).relu()
        logits = (logits * ww[..., None]).sum(1) * q.shape[-1]**-0.5
        logits = logits.masked_fill(~torch.ones(s, s, dtype=torch.bool, device=q.device).tril(), float("-inf"))
        val, idx = logits.topk(min(topk, s), -1)
        sc = torch.softmax(val, -1).nan_to_num(0.0)
        if idx.shape[-1] < topk:
            idx = torch.nn.functional.pad(idx, (0, topk - idx.shape[-1]), value=-1)
            sc = torch.nn.functional.pad(sc, (0, topk - sc.shape[-1]), value=0.0)
        out_idx.append(idx)
        out_score.append(sc)
    return torch.cat(out_idx), torch.cat(out_score), logits
