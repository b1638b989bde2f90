"""BitNet b1.58 int8 x int2 kernels, decode and prefill (reference:
examples/bitnet-1.58b/kernel_benchmark/tilelang_bitnet_158_int8xint2_{decode,prefill}.py), plus one
BitNet-3B decoder layer end to end (reference: examples/bitnet-1.58b/modeling_bitnet.py).

The kernels are ``tilelang.ops.bitnet`` (int8 activations x 2-bit weight codes on
``v_mfma_i32_16x16x64_i8``, int32 accumulation, optional dequantising epilogue); see that module
for the schedule.  ``bitnet_158_int8xint2_decode`` / ``_prefill`` keep the reference's contract:
C [M, N] int32 = A int8 [M, K] @ B^T with B the unsigned 2-bit codes packed four per byte.
"""
import argparse

import tilelang
from tilelang.ops.bitnet import int2_gemm_kernel, int2_gemv_kernel, pack_int2


def bitnet_158_int8xint2_decode(M, N, K, in_dtype="int8", out_dtype="float32", accum_dtype="int32"):
    """Decode (M <= 8): the weight-streaming GEMV kernel; with unit scales its fp32 output is the
    exact int32 product.  Call as kernel(A, qw, ones(M), ones(N))."""
    assert (in_dtype, accum_dtype) == ("int8", "int32") and M <= 8
    return int2_gemv_kernel(M, N, K, -(-K // 256) * 256, 0, out_dtype)


def bitnet_158_int8xint2_prefill(M, N, K, in_dtype="int8", out_dtype="int32", accum_dtype="int32"):
    assert (in_dtype, out_dtype, accum_dtype) == ("int8", "int32", "int32")
    return int2_gemm_kernel(M, N, K, 0, "int32")


def check(M, N, K):
    import torch
    A = torch.randint(0, 4, (M, K), device="cuda", dtype=torch.int8)
    B = torch.randint(0, 2, (N, K), device="cuda")
    ref = (A.double() @ B.double().t())
    if M <= 8:
        kern = bitnet_158_int8xint2_decode(M, N, K)
        Kp = -(-K // 256) * 256
        qw = pack_int2(torch.nn.functional.pad(B, (0, Kp - K)))
        args = (A, qw, torch.ones(M, device="cuda"), torch.ones(N, device="cuda"))
        torch.testing.assert_close(kern(*args).double(), ref, rtol=0, atol=0)
    else:
        kern = bitnet_158_int8xint2_prefill(M, N, K)
        args = (A, pack_int2(B))
        torch.testing.assert_close(kern(*args), ref.int(), rtol=0, atol=0)
    qw = args[1]
    lat = tilelang.profiler.do_bench(lambda: kern(*args))
    print(f"int8 x int2 M{M} N{N} K{K}: {lat * 1e3:.1f} us, {2 * M * N * K / lat * 1e-9:.1f} TOPS, "
          f"{N * K / 4 / lat * 1e-6:.0f} GB/s weights")


def layer_bench(tokens=2048):
    import torch
    from tilelang.models.bitnet import BitnetConfig, BitnetDecoderLayer, rope_tables, reference_layer
    cfg = BitnetConfig.bitnet_3b()
    layer = BitnetDecoderLayer(cfg).cuda()
    x = torch.randn(1, tokens, cfg.hidden_size, device="cuda", dtype=cfg.dtype)
    cos, sin = rope_tables(cfg.hidden_size // cfg.num_attention_heads, tokens, cfg.rope_theta, "cuda", cfg.dtype)
    y = layer(x, cos, sin)
    r = reference_layer(layer, x, cos, sin)
    err = (y.float() - r.float()).abs().max().item()
    print(f"BitNet-3B layer vs fp32-simulated reference: max abs err {err:.3e} (ref max {r.abs().max().item():.2f})")
    lat = tilelang.profiler.do_bench(lambda: layer(x, cos, sin))
    print(f"BitNet-3B decoder layer, {tokens} tokens: {lat:.3f} ms")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--layer_tokens", type=int, default=2048)
    a = p.parse_args()
    for shape in ((1, 3200, 3200), (1, 17280, 3200), (1, 3200, 8640), (256, 256, 256), (2048, 17280, 3200),
                  (2048, 3200, 8640)):
        check(*shape)
    layer_bench(a.layer_tokens)
