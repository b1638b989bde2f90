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
