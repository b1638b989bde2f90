"""Block-scaled MX GEMM (T.gemm_scaled -> v_mfma_scale_f32_16x16x128_f8f6f4) against an fp32 PyTorch
dequantise-then-matmul reference, with non-unit e8m0 scales (MXFP8 e4m3/e5m2, MXFP4 e2m1, mixed)."""
import pytest
import torch

import tilelang

FMTS = [("e4m3", "e4m3"), ("e2m1", "e2m1"), ("e4m3", "e2m1"), ("e5m2", "e4m3")]


def _check(c, a, b, sa, sb, af, bf):
    import example_tilelang_gemm_mx as m
    ref = m.ref_program(a.cpu(), b.cpu(), sa.cpu(), sb.cpu(), af, bf)
    torch.testing.assert_close(c.float().cpu(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())


@pytest.mark.parametrize("af,bf", FMTS)
def test_mx_gemm_cpu(af, bf):
    import example_tilelang_gemm_mx as m
    M = N = 64
    K = 256
    f = m.mx_matmul.get_tir(M, N, K, 64, 64, 128, 128, 2, af, bf)
    k = tilelang.compile(f, out_idx=[-1], target="cpu")
    a, sa = m.quantize(torch.randn(M, K) * 3, af)
    b, sb = m.quantize(torch.randn(N, K) * 0.2, bf)
    assert len(set(sa.flatten().tolist())) > 1  # genuinely non-unit, varying scales
    _check(k(a, b, sa, sb), a, b, sa, sb, af, bf)
    kh = tilelang.compile(f, out_idx=[-1], target="hip")
    src = kh.get_kernel_source()
    assert "gemm_ss_mx" in src and len(kh.code[0]) > 0


def test_mx_gemm_rejects_bad_scales():
    import example_tilelang_gemm_mx as m
    import tilelang.language as T

    @T.prim_func
    def bad(A: T.Tensor((64, 128), "float8_e4m3fn"), B: T.Tensor((64, 128), "float8_e4m3fn"),
            SA: T.Tensor((64, 8), "uint8"), SB: T.Tensor((64, 4), "uint8"), C: T.Tensor((64, 64), "float32")):
        with T.Kernel(1, threads=256):
            A_s = T.alloc_shared((64, 128), "float8_e4m3fn")
            B_s = T.alloc_shared((64, 128), "float8_e4m3fn")
            C_l = T.alloc_fragment((64, 64), "float32")
            T.copy(A, A_s)
            T.copy(B, B_s)
            T.clear(C_l)
            T.gemm_scaled(A_s, B_s, C_l, SA, SB, transpose_B=True)
            T.copy(C_l, C)

    with pytest.raises(Exception, match="scales must be"):
        tilelang.compile(bad, target="hip")
    assert m is not None


FP6_FMTS = [("e2m3", "e2m3"), ("e3m2", "e3m2"), ("e2m3", "e4m3"), ("e2m1", "e2m3")]


@pytest.mark.gpu
@pytest.mark.parametrize("af,bf", FMTS + FP6_FMTS)
def test_mx_gemm_gpu(af, bf):
    import example_tilelang_gemm_mx as m
    M, N, K = 512, 512, 1024
    k = m.mx_matmul(M, N, K, 256, 256, 128, 512, 2, af, bf)
    a, sa = m.quantize(torch.randn(M, K, device="cuda") * 3, af)
    b, sb = m.quantize(torch.randn(N, K, device="cuda") * 0.2, bf)
    assert len(set(sa.flatten().tolist())) > 1
    _check(k(a, b, sa, sb), a, b, sa, sb, af, bf)


@pytest.mark.gpu
def test_mxfp4_native_weight_gemm_gpu():
    """bf16 activations quantised to MXFP8 on the fly x stored MXFP4 weights on the scaled MFMA."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                                    "dequantize_gemm"))
    from example_dequant_gemm_mxfp4 import mxfp4_gemm_native, ref_program
    from tilelang.quantize import quantize_mxfp4
    torch.manual_seed(0)
    A = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)
    Bq, S = quantize_mxfp4(torch.randn(768, 1024, device="cuda"))
    c = mxfp4_gemm_native(A, Bq, S)
    ref = ref_program(A, Bq, S).float()
    assert ((c.float() - ref).norm() / ref.norm()).item() < 0.05


def test_preshuffle_mx_scales_order():
    """Byte ((((kk * R/64 + q) * 4 + g) * 16 + r) * 4 + b) of a tile holds the scale of row
    64 q + 16 b + r, column 4 kk + g (tl/gemm.h gemm_ss_mx SCALE_PS)."""
    from tilelang.quantize import preshuffle_mx_scales
    R, C, bk = 128, 16, 256  # one 128-row tile, two K tiles of 8 scale columns
    s = torch.arange(R * C, dtype=torch.int32).reshape(R, C)
    p = preshuffle_mx_scales(s, R, bk).reshape(-1)
    tile = bk // 32
    for row in (0, 17, 63, 64, 100, 127):
        for col in (0, 3, 5, 7, 8, 15):
            tk, kb = divmod(col, tile)
            kk, g = divmod(kb, 4)
            q, rem = divmod(row, 64)
            b, r = divmod(rem, 16)
            idx = tk * R * tile + ((((kk * (R // 64) + q) * 4 + g) * 16 + r) * 4 + b)
            assert p[idx].item() == s[row, col].item()
    with pytest.raises(ValueError):
        preshuffle_mx_scales(s[:96], 96, bk)


@pytest.mark.parametrize("af,bf", [("e4m3", "e4m3"), ("e2m1", "e2m1")])
def test_mx_gemm_preshuffled_cpu(af, bf):
    import example_tilelang_gemm_mx as m
    from tilelang.quantize import preshuffle_mx_scales
    M, N, K, bm, bn, bk = 128, 128, 512, 128, 128, 256
    f = m.mx_matmul.get_tir(M, N, K, bm, bn, bk, 256, 2, af, bf, preshuffle_scales=True)
    k = tilelang.compile(f, out_idx=[-1], target="cpu")
    a, sa = m.quantize(torch.randn(M, K) * 3, af)
    b, sb = m.quantize(torch.randn(N, K) * 0.2, bf)
    c = k(a, b, preshuffle_mx_scales(sa, bm, bk), preshuffle_mx_scales(sb, bn, bk))
    _check(c, a, b, sa, sb, af, bf)
    kh = tilelang.compile(f, out_idx=[-1], target="hip")
    assert "gemm_ss_mx" in kh.get_kernel_source() and len(kh.code[0]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("af,bf", [("e4m3", "e4m3"), ("e2m1", "e2m1"), ("e4m3", "e2m1")])
def test_mx_gemm_preshuffled_gpu(af, bf):
    import example_tilelang_gemm_mx as m
    from tilelang.quantize import preshuffle_mx_scales
    M, N, K = 512, 512, 1024
    bk = 256 if af == bf == "e2m1" else 128
    k = m.mx_matmul(M, N, K, 256, 256, bk, 512, 2, af, bf, preshuffle_scales=True)
    a, sa = m.quantize(torch.randn(M, K, device="cuda") * 3, af)
    b, sb = m.quantize(torch.randn(N, K, device="cuda") * 0.2, bf)
    _check(k(a, b, preshuffle_mx_scales(sa, 256, bk), preshuffle_mx_scales(sb, 256, bk)), a, b, sa, sb, af, bf)


def test_mx_gemm_rejects_high_row_bit_swizzle():
    """gemm_ss_mx derives each lane's swizzled address from row bits 0..3 only: an annotated LDS
    swizzle on a higher row bit is a lowering error naming the tile, not a hipcc static_assert."""
    import tilelang.language as T
    from tilelang.layout.layout import SwizzleLayout

    @T.prim_func
    def prog(A: T.Tensor((64, 128), "float8_e4m3fn"), B: T.Tensor((64, 128), "float8_e4m3fn"),
             SA: T.Tensor((64, 4), "uint8"), SB: T.Tensor((64, 4), "uint8"), C: T.Tensor((64, 64), "float32")):
        with T.Kernel(1, threads=256):
            A_s = T.alloc_shared((64, 128), "float8_e4m3fn")
            B_s = T.alloc_shared((64, 128), "float8_e4m3fn")
            C_l = T.alloc_fragment((64, 64), "float32")
            T.annotate_layout({A_s: SwizzleLayout((64, 128), 1, [(5, 0), (1, 1)])})
            T.copy(A, A_s)
            T.copy(B, B_s)
            T.clear(C_l)
            T.gemm_scaled(A_s, B_s, C_l, SA, SB, transpose_B=True)
            T.copy(C_l, C)

    with pytest.raises(Exception, match="A_s.*row bit 5"):
        tilelang.compile(prog, target="hip")


@pytest.mark.parametrize("af,bf", [("e2m3", "e2m3"), ("e3m2", "e4m3"), ("e2m1", "e3m2")])
def test_mx_gemm_fp6_cpu(af, bf):
    """Packed MXFP6 operands (4 elements per 3 bytes) against the fp32 dequantised product."""
    import example_tilelang_gemm_mx as m
    M = N = 64
    K = 256
    f = m.mx_matmul.get_tir(M, N, K, 64, 64, 128, 128, 2, af, bf)
    k = tilelang.compile(f, out_idx=[-1], target="cpu")
    a, sa = m.quantize(torch.randn(M, K) * 3, af)
    b, sb = m.quantize(torch.randn(N, K) * 0.2, bf)
    assert len(set(sa.flatten().tolist())) > 1
    _check(k(a, b, sa, sb), a, b, sa, sb, af, bf)
    kh = tilelang.compile(f, out_idx=[-1], target="hip")
    assert f"gemm_ss_mx<{'234'['e2m3 e3m2 e2m1'.split().index(af)] if af != 'e4m3' else 0}" in \
        kh.get_kernel_source() and len(kh.code[0]) > 0


def test_fp6_pack_and_grid():
    from tilelang.quantize import (dequantize_mxfp6, fp6_grid, pack_fp6, quantize_mxfp6, unpack_fp6)
    assert fp6_grid("e2m3")[-1] == 7.5 and fp6_grid("e3m2")[-1] == 28.0
    assert fp6_grid("e2m3")[1] == 0.125 and fp6_grid("e3m2")[1] == 0.0625  # subnormals
    c = torch.randint(0, 64, (3, 64), dtype=torch.uint8)
    p = pack_fp6(c)
    assert p.shape == (3, 48) and torch.equal(unpack_fp6(p), c)
    # element k at bits 6k..6k+5 of the row's little-endian bit stream
    one = torch.zeros(1, 4, dtype=torch.uint8)
    one[0, 1] = 63
    assert pack_fp6(one).tolist() == [[0b11000000, 0b00001111, 0]]
    w = torch.randn(4, 128)
    for fmt, tol in (("e2m3", 0.05), ("e3m2", 0.09)):
        q, s = quantize_mxfp6(w, fmt)
        assert ((dequantize_mxfp6(q, s, fmt) - w).norm() / w.norm()).item() < tol
