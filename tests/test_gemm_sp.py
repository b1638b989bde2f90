"""T.gemm_sp: 2:4 structured-sparse GEMM (gfx950 v_smfmac_f32_16x16x64).

Reference coverage: examples/gemm_sp/test_example_gemm_sp.py, testing/python/tilelang/
test_tilelang_tilelibrary_gemm_sp.py (compress -> kernel -> dense torch reference)."""
import os
import sys

import pytest
import torch

import tilelang
from tilelang.utils.sparse import compress, decompress, randn_semi_sparse

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "examples", "gemm_sp"))
from example_gemm_sp import matmul_sp, ref_program  # noqa: E402


def test_compress_roundtrip():
    a = randn_semi_sparse(64, 256, device="cpu")
    s, e = compress(a)
    assert s.shape == (64, 128) and e.shape == (64, 16) and e.dtype == torch.int16
    assert torch.equal(decompress(s, e), a)
    st, et = compress(a.t().contiguous(), transposed=True)
    assert st.shape == (128, 64) and torch.equal(decompress(st, et, transposed=True), a.t())
    dense = torch.randn(4, 16)
    with pytest.raises(ValueError, match="2:4"):
        compress(dense)


@pytest.mark.parametrize("trans_B", [False, True])
def test_gemm_sp_cpu(trans_B):
    M, N, K = 64, 64, 256
    f = matmul_sp.get_tir(M, N, K, block_M=64, block_N=64, block_K=64, num_stages=2, threads=256, trans_B=trans_B)
    k = tilelang.compile(f, out_idx=[-1], target="cpu")
    a = randn_semi_sparse(M, K, device="cpu")
    b = torch.randn((N, K) if trans_B else (K, N), dtype=torch.float16)
    s, e = compress(a)
    c = k(s, e, b)
    torch.testing.assert_close(c.float(), ref_program(a, b, trans_B).float(), rtol=1e-2, atol=5e-2)


@pytest.mark.parametrize("trans_B", [False, True])
def test_gemm_sp_hip_source(trans_B):
    f = matmul_sp.get_tir(256, 256, 512, trans_B=trans_B)
    src = tilelang.compile(f, out_idx=[-1], target="hip").get_kernel_source()
    assert "tl::gemm_sp_ss<half_t, 256, 256, 64, 4, 2" in src
    assert "tl::glds16" in src  # A_sparse / B stream through the LDS-DMA ring


def test_gemm_sp_rejects_bad_metadata():
    import tilelang.language as T

    @T.prim_func
    def bad(A: T.Tensor((64, 32), "float16"), E: T.Tensor((64, 8), "int16"), B: T.Tensor((64, 64), "float16"),
            C: T.Tensor((64, 64), "float32")):
        with T.Kernel(1, threads=256):
            A_s = T.alloc_shared((64, 32), "float16")
            E_s = T.alloc_shared((64, 8), "int16")
            B_s = T.alloc_shared((64, 64), "float16")
            C_f = T.alloc_fragment((64, 64), "float32")
            T.copy(A, A_s)
            T.copy(E, E_s)
            T.copy(B, B_s)
            T.clear(C_f)
            T.gemm_sp(A_s, E_s, B_s, C_f)
            T.copy(C_f, C)

    with pytest.raises(Exception, match="K/16"):
        tilelang.compile(bad, target="hip")


@pytest.mark.gpu
@pytest.mark.parametrize("trans_B", [False, True])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gemm_sp_gpu(trans_B, dtype):
    M, N, K = 512, 768, 1024
    dn = "float16" if dtype == torch.float16 else "bfloat16"
    k = matmul_sp(M, N, K, dtype=dn, out_dtype=dn, trans_B=trans_B)
    a = randn_semi_sparse(M, K, device="cuda", dtype=dtype)
    b = torch.randn((N, K) if trans_B else (K, N), device="cuda", dtype=dtype)
    s, e = compress(a)
    c = k(s, e, b)
    ref = a.float() @ (b.float().t() if trans_B else b.float())
    torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=2e-1)


@pytest.mark.gpu
def test_gemm_sp_gpu_small_tile():
    M, N, K = 256, 256, 512
    k = matmul_sp(M, N, K, block_M=128, block_N=128, block_K=128, num_stages=2, threads=256)
    a = randn_semi_sparse(M, K, device="cuda")
    b = torch.randn((K, N), device="cuda", dtype=torch.float16)
    s, e = compress(a)
    torch.testing.assert_close(k(s, e, b).float(), (a.float() @ b.float()), rtol=2e-2, atol=2e-1)
