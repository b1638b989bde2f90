"""Attention mass of every selected key, summed over heads and renormalised over the top-k
(reference: examples/dsa_sparse_finetune/sparse_mla_topk_reducesum.py) -- the target
distribution the DSA indexer is trained towards.

    attn_score[t, i] = sum_h P[t, h, idx_i] / sum_{i'} sum_h P[t, h, idx_i'],
    P = exp2(q_h . kv_idx * scale - lse_h)    (lse: the sparse MLA forward's base-2 LSE)

One block per packed token; the selected latent rows (D + rope tail, 576) are gathered 32 at a time
(``T.gather_rows``: LDS-DMA) and S^T = KV Q^T puts the keys on the MFMA M dimension so the head
sum is a row reduction.  Heads are walked in slices of 64.
"""
import tilelang
import tilelang.language as T

LOG2E = 1.44269504


@tilelang.jit(out_idx=[4], pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def sparse_mla_topk_reducesum(seq_len, heads, dqk, topk, sm_scale=None, block_I=32, threads=256,
                              dtype="bfloat16"):
    scale = (dqk**-0.5 if sm_scale is None else sm_scale) * LOG2E
    H_blk = min(64, heads)
    assert heads % H_blk == 0 and topk % block_I == 0 and H_blk % 16 == 0
    NI = topk // block_I

    @T.prim_func
    def main(Q: T.Tensor([seq_len, heads, dqk], dtype), KV: T.Tensor([seq_len, dqk], dtype),
             Idx: T.Tensor([seq_len, topk], "int32"), Lse: T.Tensor([seq_len, heads], "float32"),
             AttnScore: T.Tensor([seq_len, topk], "float32")):
        with T.Kernel(seq_len, threads=threads) as t:
            q_s = T.alloc_shared([H_blk, dqk], dtype)
            kv_s = T.alloc_shared([block_I, dqk], dtype)
            lse_s = T.alloc_shared([H_blk], "float32")
            acc = T.alloc_shared([topk], "float32")
            st = T.alloc_fragment([block_I, H_blk], "float32")
            cs = T.alloc_fragment([block_I], "float32")
            tot = T.alloc_fragment([1, topk], "float32")
            tsum = T.alloc_fragment([1], "float32")
            for i in T.Parallel(topk):
                acc[i] = 0.0
            for hb in T.serial(heads // H_blk):
                T.copy(Q[t, hb * H_blk:(hb + 1) * H_blk, :], q_s)
                T.copy(Lse[t, hb * H_blk:(hb + 1) * H_blk], lse_s)
                for ib in T.Pipelined(NI, num_stages=2):
                    T.gather_rows(KV[:, :], Idx[t, ib * block_I:(ib + 1) * block_I], kv_s)
                    T.clear(st)
                    T.gemm(kv_s, q_s, st, transpose_B=True)
                    for i, h in T.Parallel(block_I, H_blk):
                        idx = Idx[t, ib * block_I + i]
                        st[i, h] = T.exp2(T.if_then_else((idx >= 0) & (idx <= t), st[i, h] * scale - lse_s[h],
                                                         -T.infinity("float32")))
                    T.reduce_sum(st, cs, dim=1)
                    for i in T.Parallel(block_I):
                        acc[ib * block_I + i] = acc[ib * block_I + i] + cs[i]
            for z, i in T.Parallel(1, topk):
                tot[z, i] = acc[i]
            T.reduce_sum(tot, tsum, dim=1)
            for z, i in T.Parallel(1, topk):
                AttnScore[t, i] = tot[z, i] / T.max(tsum[0], 1e-30)

    return main


def sparse_mla_topk_reducesum_interface(q, kv, idx_abs, lse, sm_scale=None):
    """q [S, H, 576], kv [S, 576] (one latent group), idx_abs [S, topk] packed positions (-1 = none),
    lse [S, H] base-2 from the sparse MLA forward -> attn_score [S, topk]."""
    S, H, DQK = q.shape
    return sparse_mla_topk_reducesum(S, H, DQK, idx_abs.shape[-1], sm_scale)(q, kv, idx_abs, lse)
