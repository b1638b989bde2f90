"""Dequant GEMM variants: W4A8 (int8 MFMA), fp16 x int4 GEMV, grouped MoE bf16 x MXFP4 — CPU plumbing
target + gfx950 compile, and MI355X numerics, against PyTorch fp32/int references."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "dequantize_gemm"))

import tilelang  # noqa: E402


def _build(device, jf, *a, **kw):
    if device != "cpu":
        return jf(*a, **kw)
    f = jf.get_tir(*a, **kw)
    kh = tilelang.compile(f, out_idx=jf.out_idx, target="hip", pass_configs=jf.pass_configs)
    assert len(kh.code[0]) > 0
    return tilelang.compile(f, out_idx=jf.out_idx, target="cpu", pass_configs=jf.pass_configs)


def _w4a8(device, m, n, k, *tile):
    import example_dequant_gemm_w4a8 as w
    kern = _build(device, w.matmul_int8xint4, m, n, k, *tile)
    A = torch.randint(-128, 128, (m, k), dtype=torch.int8, device=device)
    qB = torch.randint(0, 256, (n, k // 2), dtype=torch.uint8, device=device)
    torch.testing.assert_close(kern(A, qB).cpu(), w.ref_program(A.cpu(), qB.cpu()), rtol=0, atol=0)


def test_w4a8_cpu():
    _w4a8("cpu", 64, 128, 256, 64, 64, 128, 2, 256)


@pytest.mark.gpu
def test_w4a8_gpu():
    _w4a8("cuda", 256, 1024, 2048)


def _gemv(device, M, N, K, fmt, scaled, **kw):
    import example_dequant_gemv_fp16xint4 as g
    kern = _build(device, g.dequantize_gemv, M, N, K, source_format=fmt, group_size=128, with_scaling=scaled, **kw)
    A = torch.randn(M, K, dtype=torch.float16, device=device)
    qB = torch.randint(0, 256, (N, K // 2), dtype=torch.uint8, device=device)
    args, s = [A, qB], None
    if scaled:
        s = (torch.rand(N, K // 128, device=device) * 0.02).half()
        args.append(s)
    ref = g.ref_program(A, qB, fmt, s, 128)
    torch.testing.assert_close(kern(*args).float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))


@pytest.mark.parametrize("fmt,scaled", [("uint", False), ("int", True)])
def test_gemv_int4_cpu(fmt, scaled):
    _gemv("cpu", 2, 64, 2048, fmt, scaled)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,scaled", [("uint", False), ("int", True)])
def test_gemv_int4_gpu(fmt, scaled):
    _gemv("cuda", 1, 4096, 8192, fmt, scaled)
    _gemv("cuda", 4, 1000, 4096, fmt, scaled)


def _grouped(device, m, n, k, topk, E, bm, wb, **kw):
    import example_dequant_groupedgemm_bf16_mxfp4 as gg
    A, qB, S, Bias, tw, sids, eids, pm = gg.get_data(m, n, k, 32, topk, E, bm, device=device)
    kern = _build(device, gg.matmul, m, n, k, topk, E, pm, with_bias=wb, block_M=bm, **kw)
    out = kern(A, qB, S, Bias, tw, sids, eids)
    ref = gg.ref_moe(A, qB, S, Bias, tw, sids, eids, bm, wb)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))


@pytest.mark.parametrize("wb", [False, True])
def test_grouped_mxfp4_cpu(wb):
    _grouped("cpu", 64, 128, 256, 2, 4, 32, wb, block_N=64)


@pytest.mark.gpu
@pytest.mark.parametrize("wb", [False, True])
def test_grouped_mxfp4_gpu(wb):
    _grouped("cuda", 256, 512, 1024, 4, 8, 128, wb)
