"""NSA variants: packed variable-length forward and single-token decode (CPU plumbing + MI355X)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "deepseek_nsa"))

import tilelang  # noqa: E402


def _both(jf, *a, **kw):
    f = jf.get_tir(*a, **kw)
    kh = tilelang.compile(f, out_idx=jf.out_idx, target="hip", pass_configs=jf.pass_configs)
    assert len(kh.code[0]) > 0
    return tilelang.compile(f, out_idx=jf.out_idx, target="cpu", pass_configs=jf.pass_configs)


def _varlen_check(device, lens, HQ, H, D, S, bs):
    import example_nsa_fwd_varlen as m
    q, k, v, idx, cnt, off, ti = m.make_inputs(lens, HQ, H, D, S, bs, device)
    args = (len(lens), HQ, q.shape[0], D, True, None, bs, HQ // H, S)
    kern = _both(m.native_sparse_attention_varlen, *args) if device == "cpu" else \
        m.native_sparse_attention_varlen(*args)
    o = torch.empty_like(q)
    kern(q, k, v, o, idx, cnt, off, ti)
    ref = m.ref_program(q, k, v, idx, cnt, off, bs)
    torch.testing.assert_close(o.float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)


def test_nsa_varlen_cpu():
    _varlen_check("cpu", [70, 130, 33], 32, 2, 64, 3, 32)


@pytest.mark.gpu
def test_nsa_varlen_gpu():
    _varlen_check("cuda", [300, 517, 64, 200], 32, 2, 128, 4, 64)


def _decode_check(device, B, SL, HQ, H, D, S, bs):
    import example_nsa_fwd as mf
    if device == "cpu":
        kern = _both(mf.nsa_fwd, B, HQ, 1, SL, D, False, None, bs, HQ // H, S, dtype="float16")
    else:
        from example_nsa_decode import native_sparse_attention
        kern = native_sparse_attention(B, HQ, SL, D, block_size=bs, groups=HQ // H, selected_blocks=S)
    q = torch.randn(B, 1, HQ, D).half().to(device)
    k = torch.randn(B, SL, H, D).half().to(device)
    v = torch.randn_like(k)
    idx = torch.stack([torch.randperm(SL // bs)[:S].sort()[0] for _ in range(B * H)]).view(B, 1, H, S).int()
    idx[0, 0, 0, -1] = SL  # the reference pads with seq_len: skipped
    idx = idx.to(device)
    o = kern(q, k, v, idx)
    torch.testing.assert_close(o.float().cpu(), mf.ref_program(q, k, v, idx, bs, is_causal=False).float(), rtol=2e-2,
                               atol=2e-2)


def test_nsa_decode_cpu():
    _decode_check("cpu", 2, 128, 32, 2, 64, 3, 32)


@pytest.mark.gpu
def test_nsa_decode_gpu():
    _decode_check("cuda", 4, 2048, 64, 4, 128, 8, 64)
