"""BitNet b1.58: int8 x int2 GEMM (raw and dequantising), fused RMSNorm + int8 quantisation, and a
decoder layer against the reference's fp32-simulated BitLinear math."""
import pytest
import torch

from tilelang.models import bitnet as B
from tilelang.ops import bitnet as K


def _raw(device, M, N, Kd):
    A = torch.randint(-128, 128, (M, Kd), dtype=torch.int8, device=device)
    codes = torch.randint(0, 4, (N, Kd), device=device)
    for zero in (0, 1):
        C = K.int2_gemm(A, K.pack_int2(codes), zero=zero)
        ref = (A.double() @ (codes.double() - zero).t()).int()
        torch.testing.assert_close(C, ref, rtol=0, atol=0)


def test_int2_gemm_cpu():
    _raw("cpu", 32, 64, 256)
    _raw("cpu", 3, 64, 192)  # decode-sized tile, K a multiple of 64 only


def _norm_quant(device):
    x = torch.randn(37, 512, device=device).half()
    w = (torch.rand(512, device=device) + 0.5).half()
    q, s = K.rms_norm_quant(x, w, 1e-5)
    rq, rs = K.activation_quant(B._ref_rms(x, w, 1e-5))
    assert int((q.int() - rq.int()).abs().max()) <= 1  # fp32 rounding ties at most
    torch.testing.assert_close(s, rs, rtol=1e-5, atol=0)


def test_rms_norm_quant_cpu():
    _norm_quant("cpu")


def _layer(device, tokens):
    torch.manual_seed(0)
    cfg = B.BitnetConfig.tiny()
    layer = B.BitnetDecoderLayer(cfg).to(device)
    x = torch.randn(2, tokens, cfg.hidden_size, device=device, dtype=cfg.dtype)
    cos, sin = B.rope_tables(cfg.hidden_size // cfg.num_attention_heads, tokens, cfg.rope_theta, device, cfg.dtype)
    y = layer(x, cos, sin)
    r = B.reference_layer(layer, x, cos, sin)
    assert (y.float() - r.float()).abs().max().item() < 0.03 * r.abs().max().item()


def test_bitnet_layer_cpu():
    _layer("cpu", 64)


def test_bitnet_model_generate_cpu():
    cfg = B.BitnetConfig.tiny()
    m = B.BitnetForCausalLM(cfg)
    ids = torch.randint(0, cfg.vocab_size, (1, 8))
    out = m.generate(ids, 2)
    assert out.shape == (1, 10) and torch.equal(out[:, :8], ids)


@pytest.mark.gpu
def test_int2_gemm_gpu():
    _raw("cuda", 1, 3200, 3200)
    _raw("cuda", 300, 1000, 1024)


@pytest.mark.gpu
def test_rms_norm_quant_gpu():
    _norm_quant("cuda")


@pytest.mark.gpu
def test_bitnet_layer_gpu():
    _layer("cuda", 128)


def _gemv(device, M, N, Kd):
    Kp = -(-Kd // 256) * 256
    x = torch.randint(-128, 128, (M, Kd), dtype=torch.int8, device=device)
    codes = torch.randint(0, 3, (N, Kd), device=device)
    wq = K.pack_int2(torch.nn.functional.pad(codes, (0, Kp - Kd), value=1))
    sx, sw = torch.rand(M, device=device) + 0.5, torch.rand(N, device=device) + 0.5
    out = K.int2_gemm(x, wq, sx, sw, out_dtype=torch.float32, zero=1)
    ref = (x.double() @ (codes.double() - 1).t()) / (sx.double()[:, None] * sw.double()[None])
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-3)


def test_int2_gemv_decode_cpu():
    _gemv("cpu", 1, 48, 320)
    _gemv("cpu", 3, 64, 512)


@pytest.mark.gpu
def test_int2_gemv_decode_gpu():
    _gemv("cuda", 1, 3200, 3200)
    _gemv("cuda", 4, 3200, 8640)


@pytest.mark.gpu
def test_bitnet_layer_decode_gpu():
    _layer("cuda", 1)
