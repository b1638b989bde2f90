"""GPU numerics for the fp8 GEMM and DeepSeek MLA decode examples."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,bm,bn,bk,threads", [(1024, 1024, 1024, 128, 128, 128, 256),
                                                   (512, 512, 512, 128, 128, 64, 256),
                                                   (1024, 512, 768, 256, 256, 128, 512)])
@pytest.mark.parametrize("dtype", ["float8_e4m3fn", "float8_e5m2"])
def test_fp8_gemm(M, N, K, bm, bn, bk, threads, dtype):
    from example_tilelang_gemm_fp8 import matmul, calc_diff
    k = matmul(M, N, K, bm, bn, bk, threads, 2, dtype)
    tdt = getattr(torch, dtype)
    a = torch.randn(M, K, device="cuda").to(tdt)
    b = torch.randn(N, K, device="cuda").to(tdt)
    c = k(a, b)
    ref = a.float() @ b.float().t()
    assert calc_diff(c, ref) < 1e-3
    torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=1.0)


@pytest.mark.parametrize("batch,heads,kv_ctx,num_split", [(4, 64, 512, 2), (2, 128, 1024, 4), (3, 64, 256, 1)])
def test_mla_decode(batch, heads, kv_ctx, num_split):
    from example_mla_decode import mla_decode, ref_program
    k = mla_decode(batch, heads, 1, kv_ctx, 512, 64, num_split=num_split)
    q = torch.randn(batch, heads, 512, device="cuda", dtype=torch.float16)
    q_pe = torch.randn(batch, heads, 64, device="cuda", dtype=torch.float16)
    kv = torch.randn(batch, kv_ctx, 1, 512, device="cuda", dtype=torch.float16)
    k_pe = torch.randn(batch, kv_ctx, 1, 64, device="cuda", dtype=torch.float16)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, 512, device="cuda")
    out = k(q, q_pe, kv, k_pe, glse, part)
    torch.testing.assert_close(out.float(), ref_program(q, q_pe, kv, k_pe).float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("batch,heads,kv_ctx,num_split", [(4, 128, 1024, 4), (3, 64, 512, 2)])
def test_mla_decode_persistent(batch, heads, kv_ctx, num_split):
    from example_mla_decode_persistent import mla_decode_persistent
    from example_mla_decode import ref_program
    k = mla_decode_persistent(batch, heads, 1, kv_ctx, 512, 64, num_split=num_split)
    q = torch.randn(batch, heads, 512, device="cuda", dtype=torch.float16)
    q_pe = torch.randn(batch, heads, 64, device="cuda", dtype=torch.float16)
    kv = torch.randn(batch, kv_ctx, 1, 512, device="cuda", dtype=torch.float16)
    k_pe = torch.randn(batch, kv_ctx, 1, 64, device="cuda", dtype=torch.float16)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, 512, device="cuda")
    out = k(q, q_pe, kv, k_pe, glse, part)
    torch.testing.assert_close(out.float(), ref_program(q, q_pe, kv, k_pe).float(), rtol=2e-2, atol=2e-2)
