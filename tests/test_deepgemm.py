"""Block-scaled fp8 GEMM with 2xAcc promotion (DeepGEMM recipe): CPU-target numerics + gfx950 compile,
and the MI355X kernel against the dequantised fp32 product."""
import pytest
import torch

import tilelang


@pytest.mark.parametrize("M,N,K,bn,kw", [(256, 256, 512, 128, {}),
                                         (256, 512, 384, 256, dict(block_M=256, threads=512)),
                                         (200, 192, 256, 128, {})])
def test_deepgemm_fp8_cpu(M, N, K, bn, kw):
    import example_deepgemm_fp8_2xAcc as m
    f = m.tl_gemm.get_tir(M, N, K, bn, **kw)
    assert len(tilelang.compile(f, target="hip").code[0]) > 0
    k = tilelang.compile(f, target="cpu")
    A, B = torch.randn(M, K).bfloat16(), torch.randn(N, K).bfloat16()
    a8, sa = m.per_token_cast_to_fp8(A)
    b8, sb = m.per_block_cast_to_fp8(B)
    C = torch.zeros(M, N, dtype=torch.bfloat16)
    k(a8, b8, C, sa, sb)
    assert m.calc_diff(C, m.ref_deepgemm_fp8(a8, b8, sa, sb, torch.float32)) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("out_dtype", ["bfloat16", "float32"])
@pytest.mark.parametrize("bn", [128, 256])
def test_deepgemm_fp8_gpu(out_dtype, bn):
    import example_deepgemm_fp8_2xAcc as m
    assert m.assert_tl_gemm_correctness(1024, 1024, 4096, bn, out_dtype=out_dtype, bench=False) < 1e-3
