"""``@tilelang.lazy_jit`` argument binding (tilelang/jit/lazy.py); behaviour follows the reference's
``testing/python/language/test_tilelang_language_lazy_jit.py``."""
from typing import Any

import pytest
import torch

import tilelang
import tilelang.language as T


@T.macro
def _copy_tiles(A, B):
    M, N = A.shape
    with T.Kernel(T.ceildiv(M, 32), T.ceildiv(N, 32), threads=64) as (bx, by):
        T.copy(A[bx * 32:bx * 32 + 32, by * 32:by * 32 + 32], B[bx * 32:bx * 32 + 32, by * 32:by * 32 + 32])


@T.macro
def _gemm_body(A, B, C, out_dtype, bm, bn, bk):
    M, K = A.shape
    K, N = B.shape
    with T.Kernel(T.ceildiv(M, bm), T.ceildiv(N, bn), threads=64) as (bx, by):
        A_s = T.alloc_shared((bm, bk), A.dtype)
        B_s = T.alloc_shared((bk, bn), A.dtype)
        C_l = T.alloc_fragment((bm, bn), "float32")
        T.clear(C_l)
        for k in T.Pipelined(T.ceildiv(K, bk), num_stages=2):
            T.copy(A[bx * bm, k * bk], A_s)
            T.copy(B[k * bk, by * bn], B_s)
            T.gemm(A_s, B_s, C_l)
        T.copy(C_l, C[bx * bm, by * bn])


@tilelang.lazy_jit(target="cpu")
def gemm_annot(A: T.Tensor[[int, int], Any], B: T.Tensor[[int, int], Any], out_dtype: T.dtype = T.float32,
               bm: int = 32, bn: int = 32, bk: int = 32):
    M, K = A.shape
    K, N = B.shape
    C = T.empty(M, N, dtype=out_dtype)
    _gemm_body(A, B, C, out_dtype, bm, bn, bk)
    return C


@tilelang.lazy_jit(target="cpu")
def gemm_ptr(A: T.ptr, B: T.ptr, C: T.ptr, M: int, N: int, K: int, dtype: T.dtype, out_dtype: T.dtype):
    A = T.make_tensor(A, (M, K), dtype)
    B = T.make_tensor(B, (K, N), dtype)
    C = T.make_tensor(C, (M, N), out_dtype)
    _gemm_body(A, B, C, out_dtype, 32, 32, 32)


def test_annotated_gemm_specialises_per_dtype():
    cfgs = [{"A": T.Tensor((64, 64), dt), "B": T.Tensor((64, 64), dt), "out_dtype": T.float32}
            for dt in (T.float16, T.float32)]
    ks = gemm_annot.par_compile(cfgs)
    assert len({id(k) for k in ks}) == 2
    for dt in (torch.float16, torch.float32):
        a, b = torch.randn(64, 64, dtype=dt), torch.randn(64, 64, dtype=dt)
        c = gemm_annot(a, b)
        assert c.dtype == torch.float32 and c.shape == (64, 64)
        torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-2, atol=1e-2)
    # same shapes/dtypes: no new specialisation
    n = len(gemm_annot._cache)
    gemm_annot(torch.randn(64, 64, dtype=torch.float16), torch.randn(64, 64, dtype=torch.float16))
    assert len(gemm_annot._cache) == n


def test_ptr_gemm():
    a, b = torch.randn(64, 32, dtype=torch.float16), torch.randn(32, 96, dtype=torch.float16)
    c = torch.zeros(64, 96)
    assert gemm_ptr(a, b, c, 64, 96, 32, T.float16, T.float32) is None
    torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-2, atol=1e-2)


@tilelang.lazy_jit(target="cpu")
def copy_static(A: T.Tensor[[int, int], T.float32], B: T.Tensor[[int, int], T.float32]):
    _copy_tiles(A, B)


@tilelang.lazy_jit(target="cpu")
def copy_fixed(A: T.Tensor[[64, 64], T.float32], B: T.Tensor[[64, 64], T.float32]):
    _copy_tiles(A, B)


@tilelang.lazy_jit(target="cpu")
def copy_dyn(A: T.Tensor[[T.dyn, int], T.float32], B: T.Tensor[[T.dyn, int], T.float32]):
    _copy_tiles(A, B)


@tilelang.lazy_jit(target="cpu")
def copy_strided(A: T.StridedTensor[[int, int], [int, int], T.float32],
                 B: T.StridedTensor[[int, int], [int, int], T.float32]):
    _copy_tiles(A, B)


@tilelang.lazy_jit(target="cpu")
def copy_ret(A: T.Tensor[[T.dyn, 64], Any]):
    M, N = A.shape
    B = T.empty(M, N, dtype=A.dtype)
    _copy_tiles(A, B)
    return B


@pytest.mark.parametrize("fn", [copy_static, copy_fixed, copy_dyn])
def test_copy_annotations(fn):
    a = torch.randn(64, 64)
    b = torch.empty(64, 64)
    fn(a, b)
    assert torch.equal(a, b)


def test_dyn_dim_one_kernel_for_all_sizes():
    for m in (32, 64, 96):
        a = torch.randn(m, 64)
        b = torch.empty(m, 64)
        copy_dyn(a, b)
        assert torch.equal(a, b)
    assert len(copy_dyn._cache) == 1


def test_strided_views_and_return():
    x = torch.randn(64, 2, 64, 2)
    y = torch.zeros(64, 2, 64, 2)
    copy_strided(x[:, 0, :, 0], y[:, 0, :, 0])
    assert torch.equal(x[:, 0, :, 0], y[:, 0, :, 0])
    for dt in (torch.float32, torch.float16):
        a = torch.randn(96, 64).to(dt)
        assert torch.equal(copy_ret(a), a)


def test_binding_errors():
    with pytest.raises(TypeError):
        copy_fixed(torch.randn(32, 64), torch.randn(32, 64))   # literal dims must match
    with pytest.raises(TypeError):
        copy_static(torch.randn(64, 64).half(), torch.randn(64, 64).half())  # dtype fixed to float32
    with pytest.raises(TypeError):
        copy_static(torch.randn(64, 128)[:, ::2], torch.randn(64, 64))  # non-contiguous needs StridedTensor
    with pytest.raises(TypeError):
        copy_ret(torch.randn(64, 32))   # literal trailing dim 64


@tilelang.lazy_jit
def gemm_gpu(A: T.Tensor[[int, int], Any], B: T.Tensor[[int, int], Any], out_dtype: T.dtype = T.float32):
    M, K = A.shape
    K, N = B.shape
    C = T.empty(M, N, dtype=out_dtype)
    _gemm_body(A, B, C, out_dtype, 32, 32, 32)
    return C


@pytest.mark.gpu
def test_lazy_jit_gpu():
    for dt in (torch.float16, torch.bfloat16):
        a = torch.randn(256, 128, dtype=dt, device="cuda")
        b = torch.randn(128, 192, dtype=dt, device="cuda")
        torch.testing.assert_close(gemm_gpu(a, b), a.float() @ b.float(), rtol=1e-2, atol=1e-2)
