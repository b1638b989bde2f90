"""Numerics of compiled gfx950 kernels against PyTorch fp32 references (needs an MI355X)."""
import pytest
import torch

import tilelang
import tilelang.language as T

pytestmark = pytest.mark.gpu


def _native_loaded():
    from tilelang import _native
    _native.runtime()  # raises loudly if the in-tree extension is missing


@pytest.mark.parametrize("M,N,K,bm,bn,bk,threads,stages,trans_b,dtype", [
    (1024, 1024, 1024, 128, 128, 32, 256, 3, False, "float16"),
    (512, 768, 256, 64, 64, 32, 256, 2, False, "float16"),
    (1024, 1024, 512, 128, 128, 64, 256, 2, True, "float16"),
    (1024, 1024, 1024, 256, 256, 64, 512, 2, False, "float16"),
    (512, 512, 512, 128, 128, 32, 256, 2, False, "bfloat16"),
    (512, 512, 512, 128, 128, 64, 256, 1, True, "bfloat16"),
    (1024, 768, 512, 256, 256, 64, 512, 2, "staged", "float16"),
])
def test_gemm(M, N, K, bm, bn, bk, threads, stages, trans_b, dtype):
    _native_loaded()
    from example_gemm import matmul
    staged = trans_b == "staged"  # LDS-staged epilogue (padded C tile, 16-byte row stores)
    trans_b = False if staged else trans_b
    k = matmul(M, N, K, bm, bn, bk, threads, stages, dtype, trans_B=trans_b, staged_epilogue=staged)
    tdt = getattr(torch, dtype)
    a = torch.randn(M, K, device="cuda", dtype=tdt)
    b = torch.randn((N, K) if trans_b else (K, N), device="cuda", dtype=tdt)
    ref = a.float() @ (b.float().t() if trans_b else b.float())
    torch.testing.assert_close(k(a, b).float(), ref, rtol=2e-2, atol=2e-1)


@pytest.mark.parametrize("b,h,s,d,causal,cfg", [
    (1, 2, 256, 128, False, dict(block_M=128, block_N=64, threads=256)),
    (2, 4, 512, 64, True, dict(block_M=128, block_N=64, threads=256)),
    (1, 8, 1024, 128, False, dict(block_M=256, block_N=64, threads=512)),
    (1, 4, 512, 128, True, dict(block_M=64, block_N=64, threads=256)),
])
def test_flash_attention(b, h, s, d, causal, cfg):
    _native_loaded()
    from example_mha_fwd import flashattn, ref_program
    k = flashattn(b, h, s, d, causal, 1, **cfg)
    q = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, causal).float(), rtol=2e-2, atol=2e-2)


@tilelang.jit(out_idx=[-1])
def _add(M, N, bm, bn, dtype):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), threads=256) as (bx, by):
            for i, j in T.Parallel(bm, bn):
                C[by * bm + i, bx * bn + j] = A[by * bm + i, bx * bn + j] + B[by * bm + i, bx * bn + j]

    return main


@pytest.mark.parametrize("dtype", ["float32", "float16", "bfloat16"])
def test_elementwise_add(dtype):
    _native_loaded()
    k = _add(1024, 1024, 64, 64, dtype)
    tdt = getattr(torch, dtype)
    a = torch.randn(1024, 1024, device="cuda", dtype=tdt)
    b = torch.randn(1024, 1024, device="cuda", dtype=tdt)
    torch.testing.assert_close(k(a, b), a + b)


@tilelang.jit(out_idx=[-1])
def _row_softmax(M, N, bm):

    @T.prim_func
    def main(X: T.Tensor((M, N), "float32"), Y: T.Tensor((M, N), "float32")):
        with T.Kernel(T.ceildiv(M, bm), threads=256) as bx:
            x = T.alloc_fragment((bm, N), "float32")
            mx = T.alloc_fragment((bm, ), "float32")
            sm = T.alloc_fragment((bm, ), "float32")
            T.copy(X[bx * bm, 0], x)
            T.reduce_max(x, mx, dim=1)
            for i, j in T.Parallel(bm, N):
                x[i, j] = T.exp(x[i, j] - mx[i])
            T.reduce_sum(x, sm, dim=1)
            for i, j in T.Parallel(bm, N):
                x[i, j] = x[i, j] / sm[i]
            T.copy(x, Y[bx * bm, 0])

    return main


def test_reduce_softmax():
    _native_loaded()
    k = _row_softmax(512, 256, 16)
    x = torch.randn(512, 256, device="cuda")
    torch.testing.assert_close(k(x), torch.softmax(x, dim=1), rtol=1e-4, atol=1e-5)


def test_dynamic_shape_gemm():
    _native_loaded()
    m = T.dynamic("m")

    @T.prim_func
    def dyn(A: T.Tensor((m, 256), "float16"), B: T.Tensor((256, 256), "float16"), C: T.Tensor((m, 256), "float16")):
        with T.Kernel(2, T.ceildiv(m, 128), threads=256) as (bx, by):
            A_s = T.alloc_shared((128, 32), "float16")
            B_s = T.alloc_shared((32, 128), "float16")
            C_l = T.alloc_fragment((128, 128), "float")
            T.clear(C_l)
            for k in T.Pipelined(8, num_stages=2):
                T.copy(A[by * 128, k * 32], A_s)
                T.copy(B[k * 32, bx * 128], B_s)
                T.gemm(A_s, B_s, C_l)
            T.copy(C_l, C[by * 128, bx * 128])

    k = tilelang.compile(dyn, out_idx=[-1])
    for M in (128, 384, 200):
        a = torch.randn(M, 256, device="cuda", dtype=torch.float16)
        b = torch.randn(256, 256, device="cuda", dtype=torch.float16)
        torch.testing.assert_close(k(a, b).float(), a.float() @ b.float(), rtol=2e-2, atol=2e-1)


def test_runtime_facade():
    """tilelang.runtime: device properties and runtime-owned (uncached) workspace memory."""
    from tilelang import runtime as R
    info = R.device_info(0)
    assert info["gcnArchName"].startswith("gfx950") and info["multiProcessorCount"] >= 1
    ws = R.Workspace(4096, 0, uncached=True)
    assert ws.ptr != 0
    ws.zero()
    ws.close()
    assert ws.ptr == 0
