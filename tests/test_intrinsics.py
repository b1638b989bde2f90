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
        MatrixCoreIntrinEmitter("float8_e4m3fnuz", "float8_e4m3fnuz")
    with pytest.raises(ValueError):
        MatrixCoreIntrinEmitter("float16", "float16", warp_row_tiles=24)
    with pytest.raises(ValueError):
        MatrixCoreIntrinEmitter("int8", "int8", "float32")
    e = MatrixCoreIntrinEmitter("float8_e4m3fn", "float8_e5m2", chunk=128)
    assert (e.k_dim, e.local_size_a) == (128, 32)  # the scaled f8f6f4 form
    e = MatrixCoreIntrinEmitter("float8_e4m3fn", "float8_e4m3fn", micro_size=32, fp8_k_dim=16, chunk=64, k_pack=2)
    assert (e.k_dim, e.local_size_a, e.local_size_out) == (16, 16, 16)
    e = MatrixCoreIntrinEmitter("float32", "float32", chunk=4)
    assert (e.k_dim, e.local_size_a) == (4, 1)


def test_shuffle_weight_tile_major():
    from tilelang.intrinsics import shuffle_weight
    b = torch.arange(64 * 96).view(64, 96)
    s = shuffle_weight(b, (16, 32), is_transpose=True)
    assert s.shape == (4, 3, 16, 32)
    assert s[2, 1, 5, 7] == b[2 * 16 + 5, 1 * 32 + 7]
    s = shuffle_weight(b, (16, 32), is_transpose=False)  # [K=64, N=96]
    assert s.shape == (2, 6, 32, 16) and s[1, 4, 3, 9] == b[32 + 3, 4 * 16 + 9]


_CASES = [("float16", {}), ("float16", dict(micro_size=16, block_col_warps=2, warp_row_tiles=64)),
          ("bfloat16", dict(k_pack=2)), ("float16", dict(b_transposed=False)), ("float16", dict(b_preshuffle=True)),
          ("int8", {}), ("int8", dict(micro_size=16, block_col_warps=2, warp_row_tiles=64)),
          ("float8_e4m3fn", {}), ("float8_e4m3fn", dict(micro_size=16, block_col_warps=2, warp_row_tiles=64)),
          ("float8_e5m2", dict(fp8_k_dim=16)), ("float8_e4m3fn", dict(b_preshuffle=True))]


def _types(dt):
    return ("int32", "int32") if dt == "int8" else (("float16" if dt == "float16" else "float32"), "float32")


@pytest.mark.parametrize("dt,kw", _CASES)
def test_intrinsics_gemm_compiles(dt, kw):
    out, acc = _types(dt)
    src = tilelang.compile(tl_matmul.get_tir(512, 512, 512, dt, out, acc, **kw), out_idx=[2],
                           target="hip").get_kernel_source()
    assert "tl::mfma_emit<%d, " % kw.get("micro_size", 32) in src
    assert "tl::ld_run<" in src


@pytest.mark.gpu
@pytest.mark.parametrize("dt,kw", _CASES)
def test_intrinsics_gemm_gpu(dt, kw):
    from tilelang.intrinsics import shuffle_weight
    out, acc = _types(dt)
    M, N, K = 512, 768, 1024
    k = tl_matmul(M, N, K, dt, out, acc, **kw)
    if dt == "int8":
        a = torch.randint(-8, 8, (M, K), device="cuda", dtype=torch.int8)
        b = torch.randint(-8, 8, (N, K), device="cuda", dtype=torch.int8)
    else:
        tdt = getattr(torch, dt)
        a = torch.randn(M, K, device="cuda").to(tdt)
        b = torch.randn(N, K, device="cuda").to(tdt)
    bt = b.t().contiguous() if kw.get("b_transposed", True) is False else b
    if kw.get("b_preshuffle"):
        e = MatrixCoreIntrinEmitter(dt, dt, acc, micro_size=kw.get("micro_size", 32), chunk=1 << 20)
        bt = shuffle_weight(b, (kw.get("micro_size", 32), e.micro_size_k), is_transpose=True)
    c = k(a, bt)
    ref = a.cpu().float() @ b.cpu().float().T
    if dt == "int8":
        torch.testing.assert_close(c.cpu(), ref.int())
    else:
        torch.testing.assert_close(c.float().cpu(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))


_RK_CASES = [dict(reduce_k=2, block_row_warps=2, block_col_warps=2, warp_row_tiles=64, warp_col_tiles=64),
             dict(reduce_k=4, micro_size=16, block_row_warps=1, block_col_warps=2, warp_row_tiles=64,
                  warp_col_tiles=64, chunk=32)]


@pytest.mark.parametrize("kw", _RK_CASES)
def test_intrinsics_reduce_k_compiles(kw):
    """reduce_k: the block runs (waves, reduce_k) threads, each wave group takes its K slice of
    every stage, and the partial accumulators are summed through LDS behind a barrier."""
    k = tilelang.compile(tl_matmul.get_tir(512, 512, 512, "float16", "float16", "float32", **kw), out_idx=[2],
                         target="hip")
    src = k.get_kernel_source()
    assert "__launch_bounds__(%d)" % (64 * kw["block_row_warps"] * kw["block_col_warps"] * kw["reduce_k"]) in src
    body = src[src.index("C_red"):]
    first_store = body.index("C_red[")
    assert "sync_threads" in body[first_store:] or "barrier" in body[first_store:]


@pytest.mark.gpu
@pytest.mark.parametrize("kw", _RK_CASES)
def test_intrinsics_reduce_k_gpu(kw):
    M, N, K = 512, 768, 1024
    k = tl_matmul(M, N, K, "float16", "float16", "float32", **kw)
    a = torch.randn(M, K, device="cuda").half()
    b = torch.randn(N, K, device="cuda").half()
    ref = a.cpu().float() @ b.cpu().float().T
    torch.testing.assert_close(k(a, b).float().cpu(), ref, rtol=2e-2, atol=2e-2 * (K ** 0.5))
