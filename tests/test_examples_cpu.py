"""Example kernels (elementwise / norm / softmax / top-k / fp8 cast / GEMV / split-K / Hadamard)
traced from the same DSL programs as the GPU build, executed on the CPU plumbing target against
PyTorch fp32 references, and compiled for gfx950 (hipcc cross-compiles without a GPU)."""
import pytest
import torch

import tilelang


def _both(jitf, *args, out_idx="default", **kw):
    f = jitf.get_tir(*args, **kw)
    oi = jitf.out_idx if out_idx == "default" else out_idx
    kh = tilelang.compile(f, out_idx=oi, target="hip")
    assert len(kh.code[0]) > 0
    return tilelang.compile(f, out_idx=oi, target="cpu")


def test_elementwise_add():
    import example_elementwise_add as m
    k = _both(m.elementwise_add, 256, 512, 32, 256, 256)
    a, b = torch.randn(256, 512), torch.randn(256, 512)
    torch.testing.assert_close(k(a, b), a + b)


def test_rms_norm():
    import rms_norm as m
    k = _both(m.rms_norm, 64, 512, 4)
    x = torch.randn(64, 512)
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-4)
    k = _both(m.rms_norm_splitk, 64, 2048, 4, 512)
    x = torch.randn(64, 2048)
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-4)


def test_online_softmax():
    import online_softmax as m
    k = _both(m.online_softmax, 16, 4096, 4, 1024)
    x = torch.randn(16, 4096)
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-6)
    k = _both(m.softmax_rows, 16, 1024, 4)
    x = torch.randn(16, 1024)
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-6)


def test_topk():
    import example_topk as m
    k = _both(m.tl_topk, 64, 128, 6, 16)
    x = torch.rand(64, 128)
    g, i = k(x)
    rg, ri = m.ref_program(x, 6)
    torch.testing.assert_close(g, rg)
    torch.testing.assert_close(i, ri)


def test_per_token_cast_fp8():
    import example_per_token_cast_to_fp8 as m
    k = _both(m.per_token_cast_to_fp8, 64, 512, 8)
    x = torch.randn(64, 512)
    q, s = k(x)
    rq, rs = m.ref_program(x)
    torch.testing.assert_close(s, rs)
    torch.testing.assert_close(q.float(), rq.float(), rtol=0, atol=0)


def test_gemv():
    import example_gemv as m
    k = _both(m.gemv, 64, 1024, 8, 256)
    A, x = torch.randn(64, 1024).half(), torch.randn(1024).half()
    torch.testing.assert_close(k(A, x).float(), m.ref_program(A, x).float(), rtol=1e-2, atol=1e-1)


@pytest.mark.parametrize("variant", ["tile", "elementwise"])
def test_splitk(variant):
    import example_tilelang_gemm_splitk as m
    fn = m.matmul_splitk if variant == "tile" else m.matmul_splitk_elementwise
    k = _both(fn, 128, 128, 256, 64, 64, 32, 4)
    a, b = torch.randn(128, 256).half(), torch.randn(256, 128).half()
    c = torch.zeros(128, 128)
    k(a, b, c)
    torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-3, atol=1e-3)


def test_hadamard():
    import example_hadamard as m
    k = _both(m.hadamard, 4, 1024)
    x = torch.randn(4, 1024)
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("causal", [False, True])
def test_flash_attention_bwd(causal):
    import example_mha_bwd as m
    B, S, H, D = 1, 128, 2, 64
    q, k, v, do = [torch.randn(B, S, H, D).half() for _ in range(4)]
    o, lse = _both(m.flashattn_fwd, B, H, S, D, causal, 64, 64)(q, k, v)
    qf, kf, vf = [t.float().requires_grad_() for t in (q, k, v)]
    ro = m.ref_program(qf, kf, vf, causal)
    ro.backward(do.float())
    torch.testing.assert_close(o.float(), ro.detach(), rtol=1e-2, atol=1e-2)
    delta = _both(m.flashattn_bwd_preprocess, B, H, S, D)(o, do)
    dq = torch.zeros(B, S, H, D)
    dk, dv = torch.empty_like(q), torch.empty_like(q)
    _both(m.flashattn_bwd, B, H, S, D, causal, 64, 64, 256)(q, k, v, do, lse, delta, dq, dk, dv)
    dqh = _both(m.flashattn_bwd_postprocess, B, H, S, D)(dq)
    for a, r in ((dqh, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(a.float(), r, rtol=1e-2, atol=1e-2)


def test_gqa_decode_contiguous_and_paged():
    import example_gqa_decode as m
    b, h, g, s, d, ns = 2, 8, 2, 256, 64, 2
    q = torch.randn(b, h, d).half()
    k, v = torch.randn(b, s, g, d).half(), torch.randn(b, s, g, d).half()
    lens = torch.tensor([200, 256], dtype=torch.int32)
    glse, part = torch.empty(b, h, ns), torch.empty(b, h, ns, d)
    o = _both(m.gqa_decode, b, h, g, s, d, 64, 16, ns)(q, k, v, lens, glse, part)
    torch.testing.assert_close(o, m.ref_program(q, k, v, lens), rtol=1e-2, atol=1e-2)
    ps, mp, npg = 64, 4, 10
    table = torch.randperm(npg)[:b * mp].view(b, mp).int()
    kc, vc = torch.randn(npg, ps, g, d).half(), torch.randn(npg, ps, g, d).half()
    o = _both(m.gqa_decode_paged, b, h, g, npg, ps, mp, d, 64, 16, ns)(q, kc, vc, lens, table, glse, part)
    ref = m.ref_program(q, m.paged_to_contiguous(kc, table, mp, ps), m.paged_to_contiguous(vc, table, mp, ps), lens)
    torch.testing.assert_close(o, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("sq,skv,win", [(256, 256, None), (192, 320, None), (256, 256, 128)])
def test_attention_sink(sq, skv, win):
    import example_gqa_sink_fwd_bhsd as m
    k = _both(m.flashattn_sink, 1, 8, sq, skv, 64, 4, win, None, 64, 64, 2, 256, "float16")
    q = torch.randn(1, 8, sq, 64).half()
    kk, v = torch.randn(1, 2, skv, 64).half(), torch.randn(1, 2, skv, 64).half()
    s = torch.randn(8).half()
    torch.testing.assert_close(k(q, kk, v, s).float(), m.ref_program(q, kk, v, s, win).float(), rtol=1e-2, atol=1e-2)


def test_linear_attention_fwd():
    import example_linear_attn_fwd as m
    k = _both(m.linear_attn_fwd, 1, 256, 2, 64, 64)
    q = torch.nn.functional.normalize(torch.randn(1, 256, 2, 64), dim=-1).half()
    kk = torch.nn.functional.normalize(torch.randn(1, 256, 2, 64), dim=-1).half()
    v = torch.randn(1, 256, 2, 64).half()
    o, h = k(q, kk, v)
    ro, rh = m.ref_program(q, kk, v)
    torch.testing.assert_close(o.float(), ro, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(h, rh, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("xcd_group,lean,factored,xscale", [(False, False, False, False), (True, False, False, False),
                                                            (True, True, False, False), (False, False, True, False),
                                                            (False, False, False, True)])
def test_mamba_chunk_scan(xcd_group, lean, factored, xscale):
    """xcd_group: the grid decoded so every workgroup of a (batch, chunk) shares one XCD."""
    import example_mamba_chunk_scan as m
    B = 2 if xcd_group else 1
    args = m.make_inputs(B, 2048, 128, 1, 2, 64, 64, device="cpu") if xcd_group else \
        m.make_inputs(1, 512, 128, 1, 2, 64, 64, device="cpu")
    k = _both(m.chunk_scan_fwd, B, 2048 if xcd_group else 512, 128, 1, 2, 64, 64, xcd_group=xcd_group, lean=lean,
              factored=factored, xscale=xscale, **({"block_M": 64, "block_K": 32} if xscale else {}))
    torch.testing.assert_close(k(*args).float(), m.ref_program(*args), rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("mask_split,heavy_first", [(True, False), (False, True), (True, True)])
def test_mamba_chunk_scan_mask_split(mask_split, heavy_first):
    """Diagonal-only causal select (uniform branch) and reversed row-tile order."""
    import example_mamba_chunk_scan as m
    args = m.make_inputs(1, 512, 128, 1, 2, 64, 64, device="cpu")
    k = _both(m.chunk_scan_fwd, 1, 512, 128, 1, 2, 64, 64, block_M=64, block_K=32, mask_split=mask_split,
              heavy_first=heavy_first)
    torch.testing.assert_close(k(*args).float(), m.ref_program(*args), rtol=1e-2, atol=2e-2)


def test_mamba_chunk_scan_factored_strong_decay():
    """The factored decay exp(a_i - c) exp(c - b_j) where the per-element decays span far beyond
    fp32's exponent range inside a chunk (dA down to -4 per step: -500 over a chunk): the row
    factor underflows exactly where the true decay is below fp32 range as well."""
    import example_mamba_chunk_scan as m
    args = m.make_inputs(1, 512, 128, 1, 2, 64, 64, device="cpu")
    dA = -torch.rand(1, 2, 4, 128) * 4.0
    args[3] = dA.cumsum(-1).half()
    for kw in (dict(factored=True), dict(xscale=True, block_M=64, block_K=32)):
        k = _both(m.chunk_scan_fwd, 1, 512, 128, 1, 2, 64, 64, **kw)
        out = k(*args).float()
        assert torch.isfinite(out).all()
        torch.testing.assert_close(out, m.ref_program(*args), rtol=1e-2, atol=2e-2)


def test_dequant_gemm_w4a16():
    import example_dequant_gemm_w4a16 as m
    k = _both(m.dequant_gemm_w4a16, 64, 256, 256)
    A, W = torch.randn(64, 256).half(), torch.randn(256, 256).half()
    Bq, s = m.quantize_int4(W)
    assert (m.dequantize_int4(Bq, s) - W.float()).abs().max() < 0.5
    torch.testing.assert_close(k(A, Bq, s).float(), m.ref_program(A, Bq, s).float(), rtol=1e-2, atol=5e-2)


@pytest.mark.parametrize("n,c,h,w,f,k,s,d,p", [(2, 32, 8, 8, 64, 3, 1, 1, 1), (1, 32, 9, 9, 64, 3, 2, 2, 2)])
def test_convolution_im2col(n, c, h, w, f, k, s, d, p):
    import example_convolution as m
    kern = _both(m.convolution, n, c, h, w, f, k, s, d, p, 64, 64, 32)
    a, b = torch.randn(n, h, w, c).half(), torch.randn(k, k, c, f).half()
    torch.testing.assert_close(kern(a, b).float(), m.ref_program(s, p, d)(a, b).float(), rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash_attention_bwd_atomic_free_dq(causal):
    import example_mha_bwd as m
    B, S, H, D = 1, 256, 2, 64
    q, k, v, do = [torch.randn(B, S, H, D).half() for _ in range(4)]
    o, lse = _both(m.flashattn_fwd, B, H, S, D, causal, 64, 64)(q, k, v)
    delta = _both(m.flashattn_bwd_preprocess, B, H, S, D)(o, do)
    dq = _both(m.flashattn_bwd_dq, B, H, S, D, causal, 64, 64, 256)(q, k, v, do, lse, delta)
    dk, dv = torch.empty_like(q), torch.empty_like(q)
    f = m.flashattn_bwd.get_tir(B, H, S, D, causal, 64, 64, 256, dq_mode="none")
    tilelang.compile(f, target="hip")
    tilelang.compile(f, target="cpu")(q, k, v, do, lse, delta, dk, dv)
    qf, kf, vf = [t.float().requires_grad_() for t in (q, k, v)]
    m.ref_program(qf, kf, vf, causal).backward(do.float())
    for a, r in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(a.float(), r, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash_attention_bwd_dq_fused_delta(causal):
    """dQ kernel computing Delta = rowsum(O * dO) itself (no preprocess kernel): Delta and dQ match
    the separate preprocess + dQ kernels."""
    import example_mha_bwd as m
    B, S, H, D = 1, 256, 2, 64
    q, k, v, do = [torch.randn(B, S, H, D).half() for _ in range(4)]
    o, lse = _both(m.flashattn_fwd, B, H, S, D, causal, 64, 64)(q, k, v)
    delta_ref = _both(m.flashattn_bwd_preprocess, B, H, S, D)(o, do)
    dq_ref = _both(m.flashattn_bwd_dq, B, H, S, D, causal, 64, 64, 256)(q, k, v, do, lse, delta_ref)
    delta = torch.full((B, H, S), float("nan"))
    dq = _both(m.flashattn_bwd_dq, B, H, S, D, causal, 64, 64, 256, fuse_delta=True)(q, k, v, do, lse, delta, o)
    torch.testing.assert_close(delta, delta_ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dq.float(), dq_ref.float(), rtol=1e-2, atol=1e-2)


def test_fused_moe_shared_plus_routed():
    import example_fusedmoe_tilelang as m
    w = m.init_weights(256, 128, 4, 1, device="cpu")
    x = torch.randn(2, 64, 256).half()
    out = m.FusedMoE(w, 2, block_M=64)(x)
    torch.testing.assert_close(out.float(), m.ref_program(x, w, 2).float(), rtol=1e-2, atol=1e-2)


def test_deepseek_v32_sparse_mla_fwd():
    import sparse_mla_fwd as m
    B, S, SKV, H, D, DT, topk = 1, 8, 64, 16, 64, 32, 64
    k = _both(m.sparse_mla_fwd, B, S, SKV, H, D, DT, topk, 1, None, 32, 64, "float16")
    q, kv = torch.randn(B, S, H, D + DT).half(), torch.randn(B, SKV, 1, D + DT).half()
    idx = m.make_indices(B, S, SKV, 1, topk)
    o, _ = k(q, kv, idx)
    torch.testing.assert_close(o.float(), m.ref_program(q, kv, idx, D).float(), rtol=1e-2, atol=1e-2)


def test_deepseek_v32_lightning_indexer():
    import fp8_lighting_indexer as m
    S, SKV, H, D = 8, 128, 16, 128
    k = _both(m.mqa_attn_return_logits, S, SKV, H, D)
    q, kv, sc, w, ks, ke = m.make_inputs(S, SKV, H, D, "cpu")
    out = k(q.view(S * H, D), kv, sc, w, ks, ke)
    ref = m.ref_program(q, kv, sc, w, ks, ke)
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isfinite(out), fin)
    torch.testing.assert_close(out[fin], ref[fin], rtol=1e-4, atol=1e-4)


def test_deepseek_v32_topk_selector():
    import topk_selector as m
    x = torch.randn(4, 1024)
    x[0, :10] = float("-inf")
    x[1, 5:20] = 1.0  # ties at the threshold
    idx = _both(m.topk_selector, 4, 1024, 64)(x)
    m.check(x, idx, 64)


def test_gemm_persistent():
    import example_gemm_persistent as m
    k = _both(m.matmul_persistent, 256, 384, 128, 64, 64, 32, 256, 2, 4)
    a, b = torch.randn(256, 128).half(), torch.randn(128, 384).half()
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float(), rtol=1e-2, atol=2e-2)


def test_gemm_streamk():
    import example_tilelang_gemm_streamk as m
    k = _both(m.matmul_streamk, 128, 256, 256, 64, 64, 32, 5)
    A, B = torch.randn(128, 256).half(), torch.randn(256, 256).half()
    C = torch.zeros(128, 256)
    k(A, B, C)
    torch.testing.assert_close(C, A.float() @ B.float().t(), rtol=1e-3, atol=1e-3)


def test_blocksparse_gemm():
    import example_blocksparse_gemm as m
    k = _both(m.blocksparse_matmul, 256, 256, 256, 64, 64, 32)
    a, b = torch.randn(256, 256).half(), torch.randn(256, 256).half()
    mask = torch.rand(4, 4, 8) > 0.5
    torch.testing.assert_close(k(a, b, mask).float(), m.ref_program(a, b, mask, 64, 64, 32).float(), rtol=1e-2,
                               atol=2e-2)


def _gather_rows_kernel(N, D, R, NT, target):
    import tilelang
    import tilelang.language as T

    @T.prim_func
    def k(X: T.Tensor((2, N, 1, D), "bfloat16"), I: T.Tensor((NT * R, ), "int32"),
          Y: T.Tensor((2, NT * R, D), "bfloat16")):
        with T.Kernel(2, threads=256) as b:
            S = T.alloc_shared((R, D), "bfloat16")
            for t in T.Pipelined(NT, num_stages=2):
                T.gather_rows(X[b, :, 0, 0:D], I[t * R:(t + 1) * R], S)
                T.copy(S, Y[b, t * R, 0])

    return tilelang.compile(k, out_idx=[2], target=target)


def _gather_rows_check(dev, target):
    N, D, R, NT = 300, 256, 64, 4
    k = _gather_rows_kernel(N, D, R, NT, target)
    x = torch.randn(2, N, 1, D).bfloat16().to(dev)
    i = torch.randint(-5, N + 5, (NT * R, ), dtype=torch.int32, generator=torch.Generator().manual_seed(0)).to(dev)
    y = k(x, i)
    ok = (i >= 0) & (i < N)
    ref = torch.where(ok[None, :, None], x[:, i.clamp(0, N - 1).long(), 0], torch.zeros((), dtype=x.dtype, device=dev))
    assert torch.equal(y, ref)
    return k


def test_gather_rows_cpu():
    _gather_rows_check("cpu", "cpu")
    # the HIP lowering is a lane-addressed buffer LDS-DMA inside the pipeline
    src = _gather_rows_kernel(300, 256, 64, 4, "hip").get_kernel_source()
    # invalid indices clamp (unsigned) to the row count: an offset at or past num_records reads zeros
    assert "tl::buffer_lds16" in src and "tl::min_(((uint32_t)(" in src and ", 300u)" in src


def test_nsa_fwd_cpu():
    from example_nsa_fwd import nsa_fwd, make_block_indices, ref_program
    B, SQ, SKV, HQ, H, D, S, BS = 2, 48, 128, 32, 2, 64, 4, 16
    for bt in (16, 8):
        k = nsa_fwd.get_tir(B, HQ, SQ, SKV, D, True, None, BS, HQ // H, S, block_T=bt)
        kc = tilelang.compile(k, out_idx=[-1], target="cpu")
        q, kk, v = (torch.randn(B, n, h, D).bfloat16() for n, h in ((SQ, HQ), (SKV, H), (SKV, H)))
        bi = make_block_indices(B, SQ, SKV, H, S, BS)
        torch.testing.assert_close(kc(q, kk, v, bi).float(), ref_program(q, kk, v, bi, BS).float(), rtol=2e-2,
                                   atol=2e-2)


def test_block_sparse_attn_cpu():
    from example_block_sparse_attn import blocksparse_attn, compact_mask, random_block_mask, ref_program
    B, H, S, D = 1, 2, 256, 64
    for causal in (True, False):
        f = blocksparse_attn.get_tir(B, H, S, D, causal, block=32, threads=128)
        kc = tilelang.compile(f, out_idx=[-1], target="cpu")
        q, k, v = (torch.randn(B, H, S, D).bfloat16() for _ in range(3))
        mask = random_block_mask(B, H, S // 32, 0.4, causal)
        idx, cnt = compact_mask(mask)
        torch.testing.assert_close(kc(q, k, v, idx, cnt).float(), ref_program(q, k, v, mask, 32, causal).float(),
                                   rtol=2e-2, atol=2e-2)


def test_gdn_chunked_matches_recurrence_cpu():
    from example_gdn import chunk_gated_delta_rule, make_inputs, naive_recurrent
    q, k, v, g, beta = make_inputs(1, 128, 2, 64, 32)
    o, hf = chunk_gated_delta_rule(q, k, v, g, beta, C=64, block_DV=16)
    o_ref, h_ref = naive_recurrent(q, k, v, g, beta)
    torch.testing.assert_close(o.float(), o_ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(hf, h_ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("causal,Dv", [(False, 64), (True, 64), (True, 32)])
def test_gqa_attention_fwd_bwd_cpu(causal, Dv):
    """GQA forward + backward; Dv != D is the example_gqa_bwd.py case (QK head dim != V head dim)."""
    import example_mha_bwd as m
    B, S, H, HKV, D = 1, 128, 4, 2, 64
    G = H // HKV
    q, do = torch.randn(B, S, H, D).half(), torch.randn(B, S, H, Dv).half()
    k, v = torch.randn(B, S, HKV, D).half(), torch.randn(B, S, HKV, Dv).half()
    o, lse = _both(m.flashattn_fwd, B, H, S, D, causal, 64, 64, groups=G, dim_v=Dv)(q, k, v)
    qf, kf, vf = [t.float().requires_grad_() for t in (q, k, v)]
    ro = m.ref_program(qf, kf, vf, causal)
    ro.backward(do.float())
    torch.testing.assert_close(o.float(), ro.detach(), rtol=1e-2, atol=1e-2)
    delta = _both(m.flashattn_bwd_preprocess, B, H, S, Dv)(o, do)
    dq = _both(m.flashattn_bwd_dq, B, H, S, D, causal, 64, 64, 256, groups=G, dim_v=Dv)(q, k, v, do, lse, delta)
    dk, dv = torch.empty_like(k), torch.empty_like(v)
    f = m.flashattn_bwd.get_tir(B, H, S, D, causal, 64, 64, 256, dq_mode="none", groups=G, dim_v=Dv)
    tilelang.compile(f, target="hip")
    tilelang.compile(f, target="cpu")(q, k, v, do, lse, delta, dk, dv)
    for a, r in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        torch.testing.assert_close(a.float(), r, rtol=1e-2, atol=1e-2)


def test_mla_decode_paged_cpu():
    from example_mla_decode_paged import make_paged_cache, mla_decode_paged, ref_program
    b, h, S, ps, ns = 3, 16, 200, 32, 3
    q, qpe = torch.randn(b, h, 64).bfloat16(), torch.randn(b, h, 32).bfloat16()
    kv, kpe = torch.randn(b, S, 64).bfloat16(), torch.randn(b, S, 32).bfloat16()
    sl = torch.tensor([200, 37, 129], dtype=torch.int32)
    kvp, pep, tab = make_paged_cache(kv, kpe, sl, ps)
    f = mla_decode_paged.get_tir(b, h, S, kvp.shape[0], ps, 64, 32, 32, 16, ns, 64)
    tilelang.compile(f, out_idx=[8], target="hip")
    o = tilelang.compile(f, out_idx=[8], target="cpu")(q, qpe, kvp, pep, tab, sl, torch.empty(b, h, ns),
                                                       torch.empty(b, h, ns, 64))
    torch.testing.assert_close(o.float(), ref_program(q, qpe, kv, kpe, sl).float(), rtol=2e-2, atol=2e-2)


def test_grouped_gemm_bwd_cpu():
    from example_grouped_gemm_bwd import construct_inputs, grouped_gemm, grouped_gemm_dw
    sizes, K, N = (40, 100, 7), 64, 128
    a, b, bs, bo, bpo = construct_inputs(list(sizes), K, N, False, 64, device="cpu")
    dc = torch.randn(sum(sizes), N).half()
    db = _both(grouped_gemm_dw, sizes, K, N, 64, 64, 32, 2, 128)(a, dc, bs, bo)
    ref = torch.stack([a[s:s + n].float().t() @ dc[s:s + n].float() for s, n in zip(bo.tolist(), sizes)])
    torch.testing.assert_close(db.float(), ref, rtol=1e-2, atol=5e-2)
    da = _both(grouped_gemm, sizes, N, K, 64, 64, 64, 2, 128, "float16", True)(dc, b, bs, bo, bpo)
    ref = torch.cat([dc[s:s + n].float() @ b[i].float().t() for i, (s, n) in enumerate(zip(bo.tolist(), sizes))])
    torch.testing.assert_close(da.float(), ref, rtol=1e-2, atol=5e-2)


def test_dequant_gemm_mxfp4_cpu():
    from example_dequant_gemm_mxfp4 import dequant_gemm_mxfp4, ref_program
    from tilelang.quantize import quantize_mxfp4
    M, N, K = 32, 128, 256
    k = _both(dequant_gemm_mxfp4, M, N, K, 32, 64, 128, 128)
    A = torch.randn(M, K).bfloat16()
    Bq, S = quantize_mxfp4(torch.randn(N, K))
    torch.testing.assert_close(k(A, Bq, S).float(), ref_program(A, Bq, S).float(), rtol=2e-2, atol=0.5)


@pytest.mark.parametrize("M", [1, 3])
def test_mxfp4_gemv_cpu(M):
    from example_dequant_gemm_mxfp4 import mxfp4_gemv, ref_program
    from tilelang.quantize import quantize_mxfp4
    N, K = 100, 512
    k = _both(mxfp4_gemv, M, N, K)
    A = torch.randn(M, K).bfloat16()
    Bq, S = quantize_mxfp4(torch.randn(N, K))
    torch.testing.assert_close(k(A, Bq, S).float(), ref_program(A, Bq, S).float(), rtol=2e-2, atol=0.5)


def test_gemm_with_mesh_tensor_cpu():
    from example_gemm_with_mesh_tensor import matmul
    k = _both(matmul, 128, 128, 128, 64, 64, 32)
    a, b = torch.randn(128, 128).half(), torch.randn(128, 128).half()
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float(), rtol=1e-2, atol=1e-1)
    # a (2, 2) mesh: every core sees its [64, 64] shard
    f = matmul.get_tir(128, 128, 128, 64, 64, 32, (2, 2))
    assert [int(x) for x in f.params[0].shape] == [64, 64]


def test_wide_mla_schedules_cpu():
    """8-wave schedules (S on a 4x2 wave grid, P and the row scales through LDS)."""
    import sparse_mla_fwd as sm
    from example_mla_decode import mla_decode, ref_program as mla_ref
    from example_mla_decode_paged import make_paged_cache, mla_decode_paged, ref_program
    B, S, SKV, H, D, DT, topk = 1, 4, 128, 64, 64, 32, 64
    k = _both(sm.sparse_mla_fwd, B, S, SKV, H, D, DT, topk, 1, None, 32, None, "float16", wide=True)
    q, kv = torch.randn(B, S, H, D + DT).half(), torch.randn(B, SKV, 1, D + DT).half()
    idx = sm.make_indices(B, S, SKV, 1, topk)
    torch.testing.assert_close(k(q, kv, idx)[0].float(), sm.ref_program(q, kv, idx, D).float(), rtol=1e-2, atol=1e-2)
    b, h, S2, ps, ns = 2, 64, 128, 32, 2
    q, qpe = torch.randn(b, h, 64).bfloat16(), torch.randn(b, h, 32).bfloat16()
    kv, kpe = torch.randn(b, S2, 64).bfloat16(), torch.randn(b, S2, 32).bfloat16()
    sl = torch.tensor([128, 45], dtype=torch.int32)
    kvp, pep, tab = make_paged_cache(kv, kpe, sl, ps)
    f = mla_decode_paged.get_tir(b, h, S2, kvp.shape[0], ps, 64, 32, 32, 64, ns, wide=True)
    tilelang.compile(f, out_idx=[8], target="hip")
    o = tilelang.compile(f, out_idx=[8], target="cpu")(q, qpe, kvp, pep, tab, sl, torch.empty(b, h, ns),
                                                       torch.empty(b, h, ns, 64))
    torch.testing.assert_close(o.float(), ref_program(q, qpe, kv, kpe, sl).float(), rtol=2e-2, atol=2e-2)
    kd = _both(mla_decode, b, h, 1, S2, 64, 32, 32, 64, ns, wide=True)
    o = kd(q.half(), qpe.half(), kv.half().unsqueeze(2), kpe.half().unsqueeze(2), torch.empty(b, h, ns),
           torch.empty(b, h, ns, 64))
    torch.testing.assert_close(o.float(), mla_ref(q.half(), qpe.half(), kv.half().unsqueeze(2),
                                                  kpe.half().unsqueeze(2)).float(), rtol=2e-2, atol=2e-2)


def test_sparse_mla_bwd_cpu():
    import sparse_mla_bwd as m
    from sparse_mla_fwd import make_indices
    from tilelang.ops import dsa
    B, S, SKV, H, D, DT, topk = 1, 8, 64, 16, 64, 32, 64
    q, kv = torch.randn(B, S, H, D + DT).bfloat16(), torch.randn(B, SKV, 1, D + DT).bfloat16()
    do = torch.randn(B, S, H, D).bfloat16()
    idx = make_indices(B, S, SKV, 1, topk)
    o, lse = dsa.for_target("sparse_mla_fwd", "cpu", B, S, SKV, H, D, DT, topk)(q, kv, idx)
    dq, dkv = m.sparse_mla_bwd(q, kv, o, do, idx, lse)
    rq, rkv = m.ref_bwd(q, kv, do, idx, D)
    torch.testing.assert_close(dq.float(), rq, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dkv, rkv, rtol=2e-2, atol=2e-2)
    da = m.sparse_mla_bwd(q, kv, o, do, idx, lse, dkv="atomic")[1]
    torch.testing.assert_close(da, rkv, rtol=2e-2, atol=2e-2)
    # past the memory budget the gather path falls back to the atomic one (same fp32 result)
    db = m.sparse_mla_bwd(q, kv, o, do, idx, lse, gather_budget_bytes=0)[1]
    torch.testing.assert_close(db, da, rtol=0, atol=0)
    order, offs = m.inverse_index(idx, SKV, 32)
    assert int(offs[-1]) == B * S * topk and order.numel() == B * S * topk + 32
    for impl, args in ((m.sparse_mla_bwd_dq, (1, 64, 256, 64, 512, 64, 128)),
                       (m.sparse_mla_bwd_dkv, (1, 64, 256, 64, 512, 64, 128)),
                       (m.sparse_mla_bwd_dkv_contrib, (1, 64, 64, 512, 64, 128)),
                       (m.sparse_mla_bwd_dkv_reduce, (1, 256, 64 * 128, 512, 64))):
        tilelang.compile(impl.get_tir(*args), out_idx=impl.out_idx, target="hip", pass_configs=impl.pass_configs)


def test_attention_sink_bwd_cpu():
    import example_gqa_sink_bwd as m
    fa = m.fa
    B, S, H, G, D = 1, 128, 4, 2, 64
    q, do = torch.randn(B, S, H, D).half(), torch.randn(B, S, H, D).half()
    k, v = torch.randn(B, S, H // G, D).half(), torch.randn(B, S, H // G, D).half()
    sinks = torch.randn(H)
    o, lse = _both(fa.flashattn_fwd, B, H, S, D, True, 64, 64, groups=G)(q, k, v)
    o2, lse2 = _both(m.sink_fixup, B, S, H, D, dtype="float16")(o, lse, sinks)
    delta = _both(fa.flashattn_bwd_preprocess, B, H, S, D)(o2, do)
    dq = _both(fa.flashattn_bwd_dq, B, H, S, D, True, 64, 64, 256, groups=G)(q, k, v, do, lse2, delta)
    dk, dv = torch.empty_like(k), torch.empty_like(v)
    f = fa.flashattn_bwd.get_tir(B, H, S, D, True, 64, 64, 256, dq_mode="none", groups=G)
    tilelang.compile(f, target="cpu")(q, k, v, do, lse2, delta, dk, dv)
    ds = _both(m.sink_grad, B, S, H)(lse2, delta, sinks)
    qf, kf, vf, sf = [t.float().requires_grad_() for t in (q, k, v, sinks)]
    ro = m.ref_program(qf, kf, vf, sf)
    ro.backward(do.float())
    for a, r in ((o2, ro.detach()), (dq, qf.grad), (dk, kf.grad), (dv, vf.grad), (ds, sf.grad)):
        torch.testing.assert_close(a.float(), r, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("causal", [True, False])
def test_flash_attention_varlen_cpu(causal):
    from example_mha_fwd_varlen import flashattn_varlen, make_varlen, ref_program
    q, k, v, cq, ck = make_varlen([37, 128, 5], [60, 128, 90], 4, 2, 64)
    f = flashattn_varlen.get_tir(3, 4, q.shape[0], k.shape[0], 128, 64, causal, 2, 64, 32, 256)
    tilelang.compile(f, out_idx=[5], target="hip")
    o = tilelang.compile(f, out_idx=[5], target="cpu")(q, k, v, cq, ck)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, cq, ck, causal).float(), rtol=2e-2, atol=2e-2)


def test_mla_decode_persistent_cpu():
    """One persistent kernel: split-KV tiles, T.sync_grid (host threads on the CPU target), combine."""
    from example_mla_decode_persistent import mla_decode_persistent
    from example_mla_decode import ref_program
    B, H, S, D, P, NS = 2, 64, 256, 128, 32, 2
    k = _both(mla_decode_persistent, B, H, 1, S, D, P, block_N=32, block_H=32, num_split=NS, num_cu=3, threads=256)
    q, qp = torch.randn(B, H, D, dtype=torch.float16), torch.randn(B, H, P, dtype=torch.float16)
    kv, kp = torch.randn(B, S, 1, D, dtype=torch.float16), torch.randn(B, S, 1, P, dtype=torch.float16)
    o = k(q, qp, kv, kp, torch.empty(B, H, NS), torch.empty(B, H, NS, D))
    torch.testing.assert_close(o.float(), ref_program(q, qp, kv, kp).float(), rtol=2e-2, atol=2e-2)


def test_gqa_decode_varlen_logits_contiguous_and_paged():
    import example_gqa_decode_varlen_logits as m
    lens, b, h, kh, d, bn, ns = [150, 256, 37], 3, 8, 2, 64, 32, 3
    q, k, v, cu, s_aux, kp, vp, table = m.make_inputs(lens, h, kh, d, "cpu", torch.float16, True, page_size=64)
    ro, rs = m.ref_program(q, k, v, cu, s_aux, bn)
    kern = _both(m.flashattn, b, h, kh, max(lens), k.shape[0], d, True, block_N=bn, num_split=ns)
    o, s = m.AttnPoolDecode(kern, b, h, d, ns, max(lens), bn, "cpu")(q, k, v, cu, s_aux)
    torch.testing.assert_close(o.float(), ro, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(s.float(), rs, rtol=1e-2, atol=1e-2)
    kern = _both(m.flashattn_paged, b, h, kh, max(lens), kp.shape[0], d, True, 64, block_N=bn, num_split=ns)
    o, s = m.AttnPoolDecode(kern, b, h, d, ns, max(lens), bn, "cpu")(q, kp, vp, cu, s_aux, table)
    torch.testing.assert_close(o.float(), ro, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(s.float(), rs, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_mha_inference_split_kv(causal):
    import example_mha_inference as m
    b, h, sq, sk, d, ns = 1, 2, 80, 300, 64, 3
    k = _both(m.flashattn, b, h, sq, sk, d, causal, 64, 32, ns, 256)
    q, kk, v = torch.randn(b, sq, h, d).half(), torch.randn(b, sk, h, d).half(), torch.randn(b, sk, h, d).half()
    o = k(q, kk, v, torch.empty(b, h, ns, sq), torch.empty(b, sq, h, ns, d))
    torch.testing.assert_close(o.float(), m.ref_program(q, kk, v, causal).float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_mha_fwd_bhsd_seq_q_ne_kv_cpu(causal):
    """bhsd layout, seq_q < seq_kv, bottom-right causal alignment (example_mha_fwd_bhsd.py)."""
    from example_mha_fwd_pipelined import flashattn_pipelined as fa
    from example_mha_fwd_bhsd import ref_program
    f = fa.get_tir(1, 2, 64, 64, causal, 1, 64, 32, 128, 2, "bfloat16", seq_kv=128, layout="bhsd")
    tilelang.compile(f, out_idx=[3], target="hip", pass_configs=fa.pass_configs)
    k = tilelang.compile(f, out_idx=[3], target="cpu", pass_configs=fa.pass_configs)
    q = torch.randn(1, 2, 64, 64).bfloat16()
    kk, v = (torch.randn(1, 2, 128, 64).bfloat16() for _ in range(2))
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, causal).float(), rtol=2e-2, atol=2e-2)


def test_gqa_fwd_bshd_cpu():
    from example_mha_fwd_pipelined import flashattn_pipelined as fa
    from example_mha_fwd import ref_program
    f = fa.get_tir(1, 4, 128, 64, True, 2, 64, 32, 128, 2, "bfloat16")
    k = tilelang.compile(f, out_idx=[3], target="cpu", pass_configs=fa.pass_configs)
    q = torch.randn(1, 128, 4, 64).bfloat16()
    kk, v = (torch.randn(1, 128, 2, 64).bfloat16() for _ in range(2))
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, True, 2).float(), rtol=2e-2, atol=2e-2)


def test_gqa_bwd_kv_split_cpu():
    """GQA dK/dV with the query heads of each KV head split over 2 workgroups (fp32 partials)."""
    import example_mha_bwd as m
    B, S, H, HKV, D = 1, 128, 4, 1, 64
    G = H // HKV
    q, do = torch.randn(B, S, H, D).half(), torch.randn(B, S, H, D).half()
    k, v = torch.randn(B, S, HKV, D).half(), torch.randn(B, S, HKV, D).half()
    o, lse = _both(m.flashattn_fwd, B, H, S, D, True, 64, 64, groups=G)(q, k, v)
    qf, kf, vf = [t.float().requires_grad_() for t in (q, k, v)]
    m.ref_program(qf, kf, vf, True).backward(do.float())
    delta = _both(m.flashattn_bwd_preprocess, B, H, S, D)(o, do)
    dkp = torch.empty(2, B, S, HKV, D)
    dvp = torch.empty(2, B, S, HKV, D)
    f = m.flashattn_bwd.get_tir(B, H, S, D, True, 64, 64, 256, dq_mode="none", groups=G, kv_split=2)
    tilelang.compile(f, target="hip")
    tilelang.compile(f, target="cpu")(q, k, v, do, lse, delta, dkp, dvp)
    torch.testing.assert_close(dkp.sum(0), kf.grad, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dvp.sum(0), vf.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("block_N,stages,qk_fp8,pv_fp8", [(64, 1, True, True), (32, 2, True, True),
                                                         (64, 1, True, False), (32, 2, False, False),
                                                         (128, 1, True, True)])
def test_mla_decode_kv_fp8_cpu(block_N, stages, qk_fp8, pv_fp8):
    """fp8 latent cache: fp8 (or bf16) score GEMM, P V on the fp8 MFMA (e4m3 P, transposed fp8 V
    reads) or on the widened tile, against fp32 over the dequantised cache (with the kernel's fp8 Q
    when ``qk_fp8``)."""
    from example_mla_decode_kv_fp8 import mla_decode_kv_fp8, quantize_kv, ref_program
    b, h, S, D, P, ns = 2, 64, 256, 128, 32, 2
    k = _both(mla_decode_kv_fp8, b, h, S, D, P, block_N, 64, ns, num_stages=stages, qk_fp8=qk_fp8, pv_fp8=pv_fp8)
    q, qpe = torch.randn(b, h, D).bfloat16(), torch.randn(b, h, P).bfloat16()
    kv8, s = quantize_kv(torch.randn(b, S, 1, D) * 2)
    kpe = torch.randn(b, S, 1, P).bfloat16()
    o = k(q, qpe, kv8, kpe, s, torch.empty(b, h, ns), torch.empty(b, h, ns, D))
    rq = ref_program(q, qpe, kv8, s, kpe, qk_fp8)
    if pv_fp8:
        # e4m3 probabilities (3 mantissa bits): ~2 % relative error in the norm, and a few per cent
        # of the row scale on rows dominated by one or two keys (measured: 1.8-1.9 % / 0.135 of 3.9)
        assert (o.float() - rq).norm() / rq.norm() < 3e-2
        assert (o.float() - rq).abs().max() < 0.08 * rq.abs().max()
    else:
        torch.testing.assert_close(o.float(), rq, rtol=2e-2, atol=2e-2)
    r = ref_program(q, qpe, kv8, s, kpe)
    assert (o.float() - r).norm() / r.norm() < 5e-2


def test_group_per_split_token_cast_cpu():
    from example_group_per_split_token_cast_to_fp8 import group_per_split_token_cast_to_fp8, ref_program
    sizes = [10, 0, 25, 6]
    M, N, M_max = sum(sizes), 256, 32
    x = torch.randn(M, N).bfloat16()
    bs = torch.tensor(sizes, dtype=torch.int32)
    q, s = _both(group_per_split_token_cast_to_fp8, M, M_max, N, 4, 8)(x, bs)
    rq, rs = ref_program(x, bs, M_max)
    torch.testing.assert_close(s, rs, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(q.float(), rq.float(), rtol=0.13, atol=0.01)
    assert q[1].float().abs().max() == 0 and q[0, 10:].float().abs().max() == 0
