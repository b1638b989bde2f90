"""Block-scaled fp8 linear (tilelang/ops/fp8_gemm.py) against an fp32 dequant reference, and the
DeepSeek-V3.2 model with fp8 weights on the GPU."""
import pytest
import torch

from tilelang.ops import fp8_gemm as F
from tilelang.ops.quant import act_quant


def _dequant_act(xq, xs, group=128):
    return xq.float() * xs.repeat_interleave(group, -1)[..., :xq.shape[-1]]


def _check(M, N, K, device):
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g).to(device=device, dtype=torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.05).to(device)
    wq, ws = F.weight_quant(w)
    assert ws.shape == ((N + 127) // 128, K // 128)
    y = F.fp8_linear(x, wq, ws)
    xq, xs = act_quant(x.contiguous(), 128)
    ref = _dequant_act(xq, xs) @ F.weight_dequant(wq, ws).t()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    # and close to the unquantised product (fp8 rounding only)
    full = x.float() @ w.float().t()
    assert (y.float() - full).norm() / full.norm() < 0.08


@pytest.mark.parametrize("M,N,K", [(4, 256, 256), (70, 384, 512)])
def test_fp8_linear_cpu(M, N, K):
    _check(M, N, K, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1, 512, 1024), (64, 2048, 7168), (200, 1536, 512), (1024, 4096, 2048)])
def test_fp8_linear_gpu(M, N, K):
    _check(M, N, K, "cuda")
    src = F.fp8_gemm_kernel(M, N, K).get_kernel_source()
    assert "gemm_ss_f8" in src


@pytest.mark.gpu
def test_deepseek_v32_fp8_model_gpu():
    from tilelang.models.deepseek_v32 import ModelArgs, Transformer
    toks = torch.randint(0, 512, (2, 16), generator=torch.Generator().manual_seed(7)).cuda()
    ref = Transformer(ModelArgs.tiny(), seed=0, device="cuda")(toks, 0)
    m = Transformer(ModelArgs.tiny(gemm_impl="fp8"), seed=0, device="cuda")
    out = m(toks, 0)
    rel = (out.float() - ref.float()).norm() / ref.float().norm()
    assert rel < 0.15, rel
