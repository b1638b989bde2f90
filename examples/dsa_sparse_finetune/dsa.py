"""DeepSeek Sparse Attention training step: indexer + sparse MLA, differentiable end to end
(reference: examples/dsa_sparse_finetune/dsa.py).

forward   idx, index_score = indexer top-k (indexer_topk_reducesum.py)
          o, lse           = sparse MLA forward over the selected rows (tilelang.ops.dsa)
backward  attn_score       = per-key attention mass (sparse_mla_topk_reducesum.py), the indexer target
          dq, dkv          = sparse MLA backward (examples/deepseek_v32/sparse_mla_bwd.py)
          d(index q/k/w)   = KL(attn_score || index distribution) backward (indexer_bwd.py)

Sequences are packed ([S, ...] with ``offsets`` [B+1]); the sparse MLA kernels run on the packed
tensor as one sequence with absolute row indices, masked per sequence by the indexer (a token
only ever selects rows of its own sequence at or before it).
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "deepseek_v32"))

from indexer_topk_reducesum import indexer_topk_reducesum_interface  # noqa: E402
from indexer_bwd import indexer_bwd_interface  # noqa: E402
from sparse_mla_topk_reducesum import sparse_mla_topk_reducesum_interface  # noqa: E402


def _sparse_mla_fwd(q, kv, idx_abs, dim_v, sm_scale):
    from tilelang.ops.dsa import sparse_mla_fwd
    S, H, DQK = q.shape
    k = sparse_mla_fwd(1, S, S, H, dim_v, DQK - dim_v, idx_abs.shape[-1], 1, sm_scale)
    o, lse = k(q[None].contiguous(), kv[None, :, None].contiguous(), idx_abs[None, :, None].contiguous())
    return o[0], lse[0]


class DSAFunction:

    @staticmethod
    def apply(q, kv, index_q, index_k, weights, offsets, topk, dim_v, sm_scale=None):
        import torch

        class _Fn(torch.autograd.Function):

            @staticmethod
            def forward(ctx, q, kv, index_q, index_k, weights):
                idx_rel, index_score, idx_abs = indexer_topk_reducesum_interface(index_q, weights, index_k, topk,
                                                                                 offsets, return_abs=True)
                o, lse = _sparse_mla_fwd(q, kv, idx_abs, dim_v, sm_scale)
                ctx.save_for_backward(q, kv, index_q, index_k, weights, idx_abs, index_score, o, lse)
                ctx.mark_non_differentiable(idx_rel)
                return o, idx_rel

            @staticmethod
            def backward(ctx, do, _unused):
                from sparse_mla_bwd import sparse_mla_bwd
                q, kv, index_q, index_k, weights, idx_abs, index_score, o, lse = ctx.saved_tensors
                attn_score = sparse_mla_topk_reducesum_interface(q, kv, idx_abs, lse, sm_scale)
                dq, dkv = sparse_mla_bwd(q[None], kv[None, :, None], o[None], do.contiguous().to(q.dtype)[None],
                                         idx_abs[None, :, None].contiguous(), lse[None], sm_scale)
                diq, dw, dik = indexer_bwd_interface(index_q, weights, index_k, attn_score, index_score, idx_abs)
                return (dq[0], dkv[0, :, 0].to(kv.dtype), diq, dik.to(index_k.dtype), dw.to(weights.dtype))

        return _Fn.apply(q, kv, index_q, index_k, weights)


def deepseek_sparse_attention(q, kv, index_q, index_k, weights, offsets, topk, dim_v, sm_scale=None):
    """-> (o [S, H, dim_v], topk indices [S, topk] relative to each sequence, -1 = none)."""
    return DSAFunction.apply(q, kv, index_q, index_k, weights, offsets, topk, dim_v, sm_scale)


# ----------------------------------------------------------------------------- fp32 references


def ref_sparse_attention(q, kv, idx_abs, dim_v, sm_scale=None):
    """Dense masked softmax over the selected rows (differentiable, fp32)."""
    import torch
    S, H, DQK = q.shape
    sm_scale = DQK**-0.5 if sm_scale is None else sm_scale
    sel = torch.zeros(S, S, dtype=torch.bool, device=q.device)
    rows = torch.arange(S, device=q.device)[:, None].expand_as(idx_abs)
    valid = idx_abs >= 0
    sel[rows[valid], idx_abs[valid].long()] = True
    s = torch.einsum("thd,nd->thn", q.float(), kv.float()) * sm_scale
    s = s.masked_fill(~sel[:, None, :], float("-inf"))
    p = torch.softmax(s, -1)
    return torch.einsum("thn,nd->thd", p, kv[:, :dim_v].float()), p


def ref_attn_score(p, idx_abs):
    import torch
    ps = p.sum(1)
    g = torch.gather(ps, 1, idx_abs.clamp(min=0).long()) * (idx_abs >= 0)
    return g / g.sum(-1, keepdim=True)


def ref_indexer_loss(index_q, weights, index_k, idx_abs, attn_score):
    """sum_t KL(attn_score_t || softmax(selected index logits_t)) as in the reference."""
    import torch
    import torch.nn.functional as F
    D = index_q.shape[-1]
    logits = torch.einsum("thd,nd->thn", index_q.float(), index_k.float()) * D**-0.5
    score = (logits.relu() * weights.float()[..., None]).sum(1)
    sel = torch.gather(score, 1, idx_abs.clamp(min=0).long()).masked_fill(idx_abs < 0, float("-inf"))
    logp = F.log_softmax(sel, -1)
    valid = idx_abs >= 0
    return (attn_score[valid] * (attn_score[valid].clamp(min=1e-30).log() - logp[valid])).sum()
