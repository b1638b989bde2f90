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


@pytest.mark.parametrize("batch,heads,kv_ctx,num_split,block_N,stages,qk_fp8,pv_fp8",
                         [(4, 128, 1024, 2, 64, 1, True, True), (3, 64, 512, 1, 32, 2, True, True),
                          (2, 128, 2048, 4, 32, 2, True, True), (2, 128, 1024, 2, 32, 2, False, False),
                          (4, 128, 1024, 2, 64, 1, True, False), (4, 128, 2048, 2, 128, 1, True, True),
                          (4, 128, 1024, 2, 64, 2, True, True)])
def test_mla_decode_kv_fp8(batch, heads, kv_ctx, num_split, block_N, stages, qk_fp8, pv_fp8):
    """fp8 (OCP e4m3) latent cache: scaled-MFMA scores and (pv_fp8) e4m3 P x fp8 V on the fp8 MFMA
    vs an fp32 reference over the dequantised cache."""
    from example_mla_decode_kv_fp8 import mla_decode_kv_fp8, quantize_kv, ref_program
    k = mla_decode_kv_fp8(batch, heads, kv_ctx, 512, 64, block_N=block_N, num_split=num_split, num_stages=stages,
                          qk_fp8=qk_fp8, pv_fp8=pv_fp8)
    src = k.get_kernel_source()
    assert ("gemm_ss_f8" in src) == qk_fp8
    q = torch.randn(batch, heads, 512, device="cuda", dtype=torch.bfloat16)
    q_pe = torch.randn(batch, heads, 64, device="cuda", dtype=torch.bfloat16)
    # unit-variance cache: with a much sharper softmax, rounding ties of the in-kernel Q quantisation
    # (fast-math division vs torch's) flip single fp8 steps and move outputs by a few 1e-2
    kv8, s = quantize_kv(torch.randn(batch, kv_ctx, 1, 512, device="cuda"))
    k_pe = torch.randn(batch, kv_ctx, 1, 64, device="cuda", dtype=torch.bfloat16)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, 512, device="cuda")
    out = k(q, q_pe, kv8, k_pe, s, glse, part)
    rq = ref_program(q, q_pe, kv8, s, k_pe, qk_fp8)
    if pv_fp8:  # e4m3 probabilities: ~2 % relative error in the norm (tests/test_examples_cpu.py)
        assert (out.float() - rq).norm() / rq.norm() < 3e-2
        assert (out.float() - rq).abs().max() < 0.08 * rq.abs().max()
        assert "u, false>" in src  # the PV GEMM reads the fp8 V tile transposed (ds_read_b64_tr_b8)
    else:
        torch.testing.assert_close(out.float(), rq, rtol=3e-2, atol=3e-2)
    ref = ref_program(q, q_pe, kv8, s, k_pe)
    assert (out.float() - ref).norm() / ref.norm() < (4e-2 if pv_fp8 else 3e-2)


def test_group_per_split_token_cast_gpu():
    from example_group_per_split_token_cast_to_fp8 import group_per_split_token_cast_to_fp8, ref_program
    sizes = [100, 0, 257, 64]
    M, N, M_max = sum(sizes), 1024, 320
    x = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    bs = torch.tensor(sizes, dtype=torch.int32, device="cuda")
    k = group_per_split_token_cast_to_fp8(M, M_max, N, len(sizes), 8)
    q, s = k(x, bs)
    rq, rs = ref_program(x, bs, M_max)
    torch.testing.assert_close(s, rs, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(q.float(), rq.float(), rtol=0.13, atol=0.01)  # one e4m3 ulp (rounding ties)
    assert q[1].float().abs().max() == 0 and q[0, 100:].float().abs().max() == 0  # padding rows are zero
