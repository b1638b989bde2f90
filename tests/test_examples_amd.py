"""examples/amd: persistent (T.While) FlashAttention forward and the autograd backward."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "amd"))

import tilelang  # noqa: E402
from example_amd_flash_attn_fwd import fast_flashattn, ref_program  # noqa: E402


@pytest.mark.parametrize("causal", [False, True])
def test_persistent_fa_cpu(causal):
    f = fast_flashattn.get_tir(1, 2, 256, 64, causal, 1, 64, 32, 3, 128)
    k = tilelang.compile(f, out_idx=[3], target="cpu")
    q = torch.randn(1, 256, 2, 64, dtype=torch.float16)
    kk, v = torch.randn_like(q), torch.randn_like(q)
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, causal).float(), rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("causal,groups", [(False, 1), (True, 1), (True, 4)])
def test_persistent_fa_gpu(causal, groups):
    B, H, S, D = 2, 8, 1024, 128
    k = fast_flashattn(B, H, S, D, causal, groups)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16)
    kk = torch.randn(B, S, H // groups, D, device="cuda", dtype=torch.float16)
    v = torch.randn_like(kk)
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, causal, groups).float(), rtol=2e-2,
                               atol=2e-2)


@pytest.mark.gpu
def test_amd_fa_bwd_gpu():
    from example_amd_flash_attn_bwd import main
    main(batch=1, heads=4, seq_len=512, dim=64, is_causal=True)
