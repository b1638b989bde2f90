"""Backward kernels of the sequence-model families, checked against torch fp32 autograd of the
forward definition."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("linear_attention", "gdn", "deepseek_nsa", "flash_attention", "dsa_sparse_finetune"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import tilelang  # noqa: E402


def _close(name, got, want, tol=2e-2):
    scale = max(1.0, want.abs().max().item())
    err = (got.float() - want.float()).abs().max().item()
    assert err <= tol * scale, f"{name}: max err {err:.4g} (ref max {scale:.4g})"


# --------------------------------------------------------------------------- linear attention


def _linear_inputs(B, S, H, D, device):
    g = torch.Generator().manual_seed(0)
    mk = lambda: torch.nn.functional.normalize(torch.randn(B, S, H, D, generator=g), dim=-1)  # noqa: E731
    q, k = mk().half(), mk().half()
    v = torch.randn(B, S, H, D, generator=g).half()
    do = torch.randn(B, S, H, D, generator=g).half()
    return [x.to(device) for x in (q, k, v, do)]


def _linear_check(device, B, S, H, D):
    from example_linear_attn_bwd import linear_attn_bwd, ref_program
    q, k, v, do = _linear_inputs(B, S, H, D, device)
    f = linear_attn_bwd.get_tir(B, S, H, D, D, 64, 128 if device == "cpu" else 256)
    kern = tilelang.compile(f, out_idx=[4, 5, 6], target="cpu" if device == "cpu" else "hip")
    dq, dk, dv = kern(q, k, v, do)
    qr, kr, vr = (x.float().requires_grad_(True) for x in (q, k, v))
    ref_program(qr, kr, vr).backward(do.float())
    _close("dq", dq, qr.grad)
    _close("dk", dk, kr.grad)
    _close("dv", dv, vr.grad)


def test_linear_attn_bwd_cpu():
    _linear_check("cpu", 1, 128, 2, 64)


@pytest.mark.gpu
def test_linear_attn_bwd_gpu():
    _linear_check("cuda", 2, 512, 4, 128)


@pytest.mark.gpu
def test_linear_attn_autograd_gpu():
    from example_linear_attn_bwd import LinearAttention, ref_program
    q, k, v, do = _linear_inputs(1, 256, 2, 128, "cuda")
    qa, ka, va = (x.clone().requires_grad_(True) for x in (q, k, v))
    o = LinearAttention.apply(qa, ka, va)
    o.backward(do)
    qr, kr, vr = (x.float().requires_grad_(True) for x in (q, k, v))
    ref_program(qr, kr, vr).backward(do.float())
    _close("o", o, ref_program(q, k, v))
    for n, a, r in (("dq", qa, qr), ("dk", ka, kr), ("dv", va, vr)):
        _close(n, a.grad, r.grad)


# --------------------------------------------------------------------------- gated delta rule


def _gdn_check(device, S, H, D, block_DV):
    from example_gdn import make_inputs
    from example_gdn_bwd import chunk_gated_delta_rule_bwd, reference_grads
    q, k, v, g, beta = make_inputs(1, S, H, D, D, device)
    do = torch.randn(1, S, H, D, generator=torch.Generator().manual_seed(1)).to(torch.bfloat16).to(device)
    got = chunk_gated_delta_rule_bwd(q, k, v, g, beta, do, block_DV=block_DV)[:5]
    ref = reference_grads(q, k, v, g, beta, do)
    for n, a, r in zip(("dq", "dk", "dv", "dg", "dbeta"), got, ref):
        _close(n, a.cpu(), r)


def test_gdn_bwd_cpu():
    _gdn_check("cpu", 128, 2, 32, 32)


@pytest.mark.gpu
def test_gdn_bwd_gpu():
    _gdn_check("cuda", 256, 2, 128, 32)


@pytest.mark.gpu
def test_gdn_autograd_gpu():
    from example_gdn import make_inputs, naive_recurrent
    from example_gdn_bwd import ChunkGatedDeltaRule
    q, k, v, g, beta = make_inputs(1, 192, 2, 64, 64, "cuda")
    xs = [x.clone().requires_grad_(True) for x in (q, k, v, g, beta)]
    o = ChunkGatedDeltaRule.apply(*xs)
    do = torch.randn_like(o)
    o.backward(do)
    rs = [x.detach().float().cpu().requires_grad_(True) for x in (q, k, v, g, beta)]
    o_ref, _ = naive_recurrent(*rs)
    o_ref.backward(do.float().cpu())
    _close("o", o.cpu(), o_ref, 5e-2)
    for n, a, r in zip(("dq", "dk", "dv", "dg", "dbeta"), xs, rs):
        _close(n, a.grad.cpu(), r.grad, 5e-2)


# --------------------------------------------------------------------------- NSA


def _nsa_check(device, B, SQ, HQ, H, D, S, BS):
    from example_nsa_fwd import make_block_indices
    from example_nsa_bwd import nsa_fwd_lse, nsa_backward, ref_attention
    g = torch.Generator().manual_seed(0)
    q = torch.randn(B, SQ, HQ, D, generator=g).bfloat16().to(device)
    k = torch.randn(B, SQ, H, D, generator=g).bfloat16().to(device)
    v = torch.randn(B, SQ, H, D, generator=g).bfloat16().to(device)
    bi = make_block_indices(B, SQ, SQ, H, S, BS, device)
    o, lse = nsa_fwd_lse(B, HQ, SQ, SQ, D, True, None, BS, HQ // H, S)(q, k, v, bi)
    do = torch.randn(o.shape, generator=g).bfloat16().to(device)
    dq, dk, dv = nsa_backward(q, k, v, bi, o, lse, do, BS)
    qr, kr, vr = (x.float().cpu().requires_grad_(True) for x in (q, k, v))
    orf = ref_attention(qr, kr, vr, bi, BS)
    _close("o", o.cpu(), orf)
    orf.backward(do.float().cpu())
    _close("dq", dq.cpu(), qr.grad)
    _close("dk", dk.cpu(), kr.grad)
    _close("dv", dv.cpu(), vr.grad)


def test_nsa_bwd_cpu():
    _nsa_check("cpu", 1, 96, 16, 1, 64, 2, 32)


@pytest.mark.gpu
def test_nsa_bwd_gpu():
    _nsa_check("cuda", 2, 512, 32, 2, 128, 4, 64)


# --------------------------------------------------------------------------- varlen FlashAttention


def _varlen_check(device, lens_q, lens_k, H, G, D, causal, small):
    from example_mha_fwd_varlen import make_varlen
    from example_mha_bwd_varlen import (flashattn_varlen_fwd_lse, reference_grads, varlen_bwd_dkv, varlen_bwd_dq,
                                        varlen_bwd_preprocess)
    torch.manual_seed(0)
    q, k, v, cu_q, cu_k = make_varlen(lens_q, lens_k, H, H // G, D, device)
    B, TQ, TK = len(lens_q), q.shape[0], k.shape[0]
    cfg = (64, 32, 128) if small else (128, 64, 256)
    o, lse = flashattn_varlen_fwd_lse(B, H, TQ, TK, max(lens_q), D, causal, G, *cfg)(q, k, v, cu_q, cu_k)
    do = torch.randn_like(o)
    delta = varlen_bwd_preprocess(H, TQ, D)(o, do)
    kv_cfg = (64, 32, 128) if small else (128, 64, 512)
    dk, dv = varlen_bwd_dkv(B, H, TQ, TK, max(lens_k), D, causal, G, *kv_cfg)(q, k, v, do, lse, delta, cu_q, cu_k)
    dq = varlen_bwd_dq(B, H, TQ, TK, max(lens_q), D, causal, G, *cfg)(q, k, v, do, lse, delta, cu_q, cu_k)
    orf, gq, gk, gv = reference_grads(q, k, v, cu_q, cu_k, do, causal)
    _close("o", o.cpu(), orf)
    _close("dq", dq.cpu(), gq)
    _close("dk", dk.cpu(), gk)
    _close("dv", dv.cpu(), gv)


@pytest.mark.parametrize("causal", [True, False])
def test_varlen_attn_bwd_cpu(causal):
    _varlen_check("cpu", [40, 100, 64], [72, 100, 64], 4, 2, 64, causal, True)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [True, False])
def test_varlen_attn_bwd_gpu(causal):
    _varlen_check("cuda", [300, 1000, 64, 513], [300, 1200, 64, 700], 8, 4, 128, causal, False)


# --------------------------------------------------------------------------- DSA sparse fine-tuning


def _dsa_check(device, S, H, HI, topk, lens):
    from dsa import deepseek_sparse_attention, ref_sparse_attention, ref_attn_score, ref_indexer_loss
    from indexer_topk_reducesum import indexer_topk_reducesum_interface, ref_index_score
    g = torch.Generator().manual_seed(0)
    DQK, DV, DI = 576, 512, 64
    mk = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).bfloat16().to(device)  # noqa: E731
    q, kv, iq, ik, w = mk(S, H, DQK, sc=0.5), mk(S, DQK, sc=0.5), mk(S, HI, DI), mk(S, DI), mk(S, HI)
    offsets = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=device)
    xs = [x.clone().requires_grad_(True) for x in (q, kv, iq, ik, w)]
    o, idx = deepseek_sparse_attention(*xs, offsets, topk, DV)
    do = torch.randn(o.shape, generator=g).to(device)
    o.backward(do)
    # the selection matches torch.topk as sets with the same softmax scores
    idx_rel, score, idx_abs = indexer_topk_reducesum_interface(iq, w, ik, topk, offsets, return_abs=True)
    ridx, rscore, _ = ref_index_score(iq.cpu(), w.cpu(), ik.cpu(), topk, offsets.cpu())
    for t in range(0, S, 7):
        a = sorted(float(s) for i, s in zip(idx_rel[t].cpu(), score[t].cpu()) if i >= 0)
        b = sorted(float(s) for s in rscore[t] if s > 0)
        assert len(a) == len(b) and max((abs(x - y) for x, y in zip(a, b)), default=0) < 2e-3, t
    rs = [x.float().cpu().clone().requires_grad_(True) for x in (q, kv, iq, ik, w)]
    idx_c = idx_abs.cpu()
    orf, p = ref_sparse_attention(rs[0], rs[1], idx_c, DV)
    _close("o", o.cpu(), orf)
    orf.backward(do.float().cpu())
    ref_indexer_loss(rs[2], rs[4], rs[3], idx_c, ref_attn_score(p.detach(), idx_c)).backward()
    for n, a, r in zip(("dq", "dkv", "d_index_q", "d_index_k", "d_weights"), xs, rs):
        _close(n, a.grad.cpu(), r.grad)


def test_dsa_finetune_cpu():
    _dsa_check("cpu", 128, 16, 16, 64, [50, 78])


@pytest.mark.gpu
def test_dsa_finetune_gpu():
    _dsa_check("cuda", 512, 64, 32, 128, [200, 312])
