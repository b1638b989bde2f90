"""CPU ("c"/"llvm"/"cpu") plumbing target — BASELINE config 1 and friends (no GPU needed)."""
import pytest
import torch

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1], target="cpu")
def elementwise_add(M, N, bm, bn, dtype="float32"):

    @T.prim_func
    def main(A: T.Tensor((M, N), dtype), B: T.Tensor((M, N), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), is_cpu=True) as (bx, by):
            for i, j in T.Parallel(bm, bn):
                C[by * bm + i, bx * bn + j] = A[by * bm + i, bx * bn + j] + B[by * bm + i, bx * bn + j]

    return main


def test_elementwise_add_1024():
    k = elementwise_add(1024, 1024, 32, 32)
    a, b = torch.randn(1024, 1024), torch.randn(1024, 1024)
    torch.testing.assert_close(k(a, b), a + b)


@tilelang.jit(out_idx=[-1], target="cpu")
def cpu_gemm(M, N, K, bm, bn, bk, dtype="float16"):

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), C: T.Tensor((M, N), "float32")):
        with T.Kernel(T.ceildiv(N, bn), T.ceildiv(M, bm), is_cpu=True) as (bx, by):
            A_s = T.alloc_shared((bm, bk), dtype)
            B_s = T.alloc_shared((bk, bn), dtype)
            C_l = T.alloc_fragment((bm, bn), "float")
            T.clear(C_l)
            for k in T.Pipelined(T.ceildiv(K, bk), num_stages=2):
                T.copy(A[by * bm, k * bk], A_s)
                T.copy(B[k * bk, bx * bn], B_s)
                T.gemm(A_s, B_s, C_l)
            T.copy(C_l, C[by * bm, bx * bn])

    return main


def test_cpu_gemm_matches_torch():
    k = cpu_gemm(128, 96, 64, 32, 32, 32)
    a = torch.randn(128, 64).half()
    b = torch.randn(64, 96).half()
    torch.testing.assert_close(k(a, b), a.float() @ b.float(), rtol=1e-3, atol=1e-3)


@tilelang.jit(out_idx=[-1], target="cpu")
def cpu_rowmax(M, N):

    @T.prim_func
    def main(A: T.Tensor((M, N), "float32"), O: T.Tensor((M, ), "float32")):
        with T.Kernel(1, is_cpu=True):
            A_l = T.alloc_fragment((M, N), "float32")
            m = T.alloc_fragment((M, ), "float32")
            T.copy(A, A_l)
            T.reduce_max(A_l, m, dim=1)
            T.copy(m, O)

    return main


def test_cpu_reduce_max():
    k = cpu_rowmax(16, 40)
    a = torch.randn(16, 40)
    torch.testing.assert_close(k(a), a.max(dim=1).values)


def test_runtime_argument_checks():
    k = elementwise_add(64, 64, 32, 32)
    a = torch.randn(64, 64)
    with pytest.raises(ValueError, match="dtype"):
        k(a, torch.randn(64, 64, dtype=torch.float64))
    with pytest.raises(ValueError, match="dim 1"):
        k(a, torch.randn(64, 32))
    with pytest.raises(ValueError, match="expected 2 inputs"):
        k(a)
    with pytest.raises(ValueError, match="contiguous"):
        k(a, torch.randn(64, 64).t())
