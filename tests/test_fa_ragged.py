"""Ragged sequence lengths in the FlashAttention forward kernels: keys at or past seq_len in the
last KV tile are masked (reference examples/flash_attention/example_mha_fwd_bshd.py:54), query
rows past seq_len are neither computed into nor stored.  Every case is checked against the fp32
definition (example_mha_fwd.ref_program); s=192/256 run beside the ragged ones as controls."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "flash_attention"))
sys.path.insert(0, os.path.join(ROOT, "examples", "amd"))

import tilelang  # noqa: E402
from example_mha_fwd import flashattn, ref_program  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined  # noqa: E402


def _check(out, q, k, v, causal, groups=1):
    ref = ref_program(q, k, v, causal, groups).float()
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    # the scaled-row symptom of a missing mask (all rows ~0.93x): the median error stays small
    assert (out.float() - ref).abs().median().item() < 5e-3


def _inputs(b, s, h, d, groups=1, device="cpu", dtype=torch.bfloat16):
    q = torch.randn(b, s, h, d, device=device, dtype=dtype)
    k = torch.randn(b, s, h // groups, d, device=device, dtype=dtype)
    return q, k, torch.randn_like(k)


@pytest.mark.parametrize("s", [200, 192, 333])
@pytest.mark.parametrize("causal", [False, True])
def test_mha_fwd_ragged_cpu(s, causal):
    f = flashattn.get_tir(2, 2, s, 64, causal, 1, 64, 32, 128, 2)
    k = tilelang.compile(f, out_idx=[3], target="cpu")
    q, kk, v = _inputs(2, s, 2, 64)
    _check(k(q, kk, v), q, kk, v, causal)


@pytest.mark.parametrize("s", [200, 333])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("fold_max,sum_mfma", [(False, False), (True, True)])
def test_pipelined_fwd_ragged_cpu(s, causal, fold_max, sum_mfma):
    f = flashattn_pipelined.get_tir(1, 2, s, 64, causal, 1, 64, 32, 128, 2, "bfloat16", True, True,
                                    fold_max=fold_max, sum_mfma=sum_mfma)
    k = tilelang.compile(f, out_idx=[3], target="cpu")
    q, kk, v = _inputs(1, s, 2, 64)
    _check(k(q, kk, v), q, kk, v, causal)


@pytest.mark.parametrize("causal", [False, True])
def test_persistent_fwd_ragged_cpu(causal):
    from example_amd_flash_attn_fwd import fast_flashattn
    f = fast_flashattn.get_tir(1, 2, 200, 64, causal, 1, 64, 32, 3, 128)
    k = tilelang.compile(f, out_idx=[3], target="cpu")
    q, kk, v = _inputs(1, 200, 2, 64, dtype=torch.float16)
    _check(k(q, kk, v), q, kk, v, causal)


@pytest.mark.gpu
@pytest.mark.parametrize("s", [200, 333, 4000])
@pytest.mark.parametrize("causal", [False, True])
def test_pipelined_fwd_ragged_gpu(s, causal):
    """The bench kernel's configuration (fold_max, sum_mfma, 256x64 tile, 8 waves) at ragged s."""
    k = flashattn_pipelined(2, 4, s, 128, causal, 2, 256, 64, 512, 2, q_in_regs=True, fold_max=True,
                            sum_mfma=True, young_prio=True)
    q, kk, v = _inputs(2, s, 4, 128, groups=2, device="cuda")
    _check(k(q, kk, v), q, kk, v, causal, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("s", [200, 333])
@pytest.mark.parametrize("causal", [False, True])
def test_mha_fwd_ragged_gpu(s, causal):
    k = flashattn(2, 4, s, 128, causal)
    q, kk, v = _inputs(2, s, 4, 128, device="cuda")
    _check(k(q, kk, v), q, kk, v, causal)


@pytest.mark.gpu
@pytest.mark.parametrize("causal", [False, True])
def test_persistent_fwd_ragged_gpu(causal):
    from example_amd_flash_attn_fwd import fast_flashattn
    k = fast_flashattn(2, 8, 1000, 128, causal)
    q, kk, v = _inputs(2, 1000, 8, 128, device="cuda", dtype=torch.float16)
    _check(k(q, kk, v), q, kk, v, causal)
