"""User-level MFMA emitter (tilelang.intrinsics) and examples/gemm/example_gemm_intrinsics.py."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm"))

import tilelang  # noqa: E402
from tilelang.intrinsics import MatrixCoreIntrinEmitter, mfma_layout  # noqa: E402
from example_gemm_intrinsics import tl_matmul  # noqa: E402


def test_lane_maps_cover_tiles():
    for kp in (8, 16):
        a = {mfma_layout.a_coord(l, j, kp) for l in range(64) for j in range(kp)}
        b = {mfma_layout.b_coord(l, j, kp) for l in range(64) for j in range(kp)}
        assert a == {(r, k) for r in range(16) for k in range(4 * kp)}
        assert b == {(k, c) for k in range(4 * kp) for c in range(16)}
    c = {mfma_layout.c_coord(l, v) for l in range(64) for v in range(4)}
    assert c == {(r, n) for r in range(16) for n in range(16)}


def test_emitter_validation():
    with pytest.raises(NotImplementedError):
        MatrixCoreIntrinEmitter("float32", "float32")
    with pytest.raises(ValueError):
        MatrixCoreIntrinEmitter("float16", "float16", warp_row_tiles=24)


@pytest.mark.parametrize("dt", ["float16", "int8"])
def test_intrinsics_gemm_compiles(dt):
    out, acc = ("int32", "int32") if dt == "int8" else ("float16", "float32")
    src = tilelang.lower(tl_matmul.get_tir(256, 256, 256, dt, out, acc), target="hip").kernel_source
    assert src.count("tl::mfma_16x16") == 16  # 4 x 4 warp tiles per K step


@pytest.mark.gpu
@pytest.mark.parametrize("dt", ["float16", "bfloat16", "int8"])
def test_intrinsics_gemm_gpu(dt):
    out, acc = ("int32", "int32") if dt == "int8" else (dt, "float32")
    M, N, K = 512, 384, 256
    k = tl_matmul(M, N, K, dt, out, acc)
    if dt == "int8":
        a = torch.randint(-8, 8, (M, K), device="cuda", dtype=torch.int8)
        b = torch.randint(-8, 8, (N, K), device="cuda", dtype=torch.int8)
        torch.testing.assert_close(k(a, b).cpu(), (a.cpu().long() @ b.cpu().long().T).int())
    else:
        tdt = getattr(torch, dt)
        a = torch.randn(M, K, device="cuda", dtype=tdt)
        b = torch.randn(N, K, device="cuda", dtype=tdt)
        torch.testing.assert_close(k(a, b).float(), a.float() @ b.float().T, rtol=2e-2, atol=2e-2)
