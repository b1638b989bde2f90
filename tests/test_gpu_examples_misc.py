"""MI355X numerics of the memory-bound / utility example kernels against PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _native():
    from tilelang import _native
    _native.runtime()


def test_elementwise_add():
    import example_elementwise_add as m
    for dt in ("float32", "float16"):
        k = m.elementwise_add(1024, 1024, in_dtype=dt, out_dtype=dt)
        a = torch.randn(1024, 1024, device="cuda", dtype=getattr(torch, dt))
        b = torch.randn(1024, 1024, device="cuda", dtype=getattr(torch, dt))
        torch.testing.assert_close(k(a, b), a + b)


def test_rms_norm():
    import rms_norm as m
    k = m.rms_norm(1024, 4096, 4)
    x = torch.randn(1024, 4096, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-4)
    k = m.rms_norm_splitk(256, 8192, 4, 512)
    x = torch.randn(256, 8192, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-4)


def test_online_softmax():
    import online_softmax as m
    k = m.online_softmax(512, 8192)
    x = torch.randn(512, 8192, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-6)
    k = m.softmax_rows(512, 1024)
    x = torch.randn(512, 1024, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-4, atol=1e-6)


def test_topk():
    import example_topk as m
    k = m.tl_topk(320, 128, 6, 16)
    x = torch.rand(320, 128, device="cuda")
    g, i = k(x)
    rg, ri = m.ref_program(x, 6)
    torch.testing.assert_close(g, rg)
    torch.testing.assert_close(i, ri)


def test_per_token_cast_fp8():
    import example_per_token_cast_to_fp8 as m
    k = m.per_token_cast_to_fp8(1024, 1024, 8)
    x = torch.randn(1024, 1024, device="cuda")
    q, s = k(x)
    rq, rs = m.ref_program(x)
    torch.testing.assert_close(s, rs)
    torch.testing.assert_close(q.float(), rq.float(), rtol=0, atol=0)


def test_gemv():
    import example_gemv as m
    k = m.gemv(4096, 4096)
    A = torch.randn(4096, 4096, device="cuda", dtype=torch.float16)
    x = torch.randn(4096, device="cuda", dtype=torch.float16)
    torch.testing.assert_close(k(A, x).float(), m.ref_program(A, x).float(), rtol=1e-2, atol=1e-1)


@pytest.mark.parametrize("variant", ["tile", "elementwise"])
def test_splitk(variant):
    import example_tilelang_gemm_splitk as m
    fn = m.matmul_splitk if variant == "tile" else m.matmul_splitk_elementwise
    k = fn(512, 512, 4096, split_k=4)
    a = torch.randn(512, 4096, device="cuda", dtype=torch.float16)
    b = torch.randn(4096, 512, device="cuda", dtype=torch.float16)
    c = torch.zeros(512, 512, device="cuda")
    k(a, b, c)
    torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-2, atol=1e-1)


def test_hadamard():
    import example_hadamard as m
    k = m.hadamard(8, 4096)
    x = torch.randn(8, 4096, device="cuda")
    torch.testing.assert_close(k(x), m.ref_program(x), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("dtype", ["float16", "bfloat16"])
def test_flash_attention_bwd(causal, dtype):
    import example_mha_bwd as m
    tdt = getattr(torch, dtype)
    B, S, H, D = 2, 512, 4, 64
    Q = torch.randn(B, S, H, D, dtype=tdt, device="cuda").requires_grad_()
    K = torch.randn_like(Q).requires_grad_()
    V = torch.randn_like(Q).requires_grad_()
    dO = torch.randn_like(Q)
    m.attention(Q, K, V, causal).backward(dO)
    grads = [t.grad.clone() for t in (Q, K, V)]
    for t in (Q, K, V):
        t.grad = None
    m.ref_program(Q, K, V, causal).backward(dO)
    for g, t in zip(grads, (Q, K, V)):
        torch.testing.assert_close(g.float(), t.grad.float(), rtol=3e-2, atol=3e-2)


def test_gqa_decode_contiguous_and_paged():
    import example_gqa_decode as m
    b, h, g, s, d, ns = 4, 32, 8, 2048, 128, 4
    q = torch.randn(b, h, d, device="cuda", dtype=torch.float16)
    k = torch.randn(b, s, g, d, device="cuda", dtype=torch.float16)
    v = torch.randn_like(k)
    lens = torch.tensor([2048, 1500, 700, 1], dtype=torch.int32, device="cuda")
    glse = torch.empty(b, h, ns, device="cuda")
    part = torch.empty(b, h, ns, d, device="cuda")
    o = m.gqa_decode(b, h, g, s, d, num_split=ns)(q, k, v, lens, glse, part)
    torch.testing.assert_close(o, m.ref_program(q, k, v, lens), rtol=2e-2, atol=2e-2)
    ps, mp, npg = 64, 32, 160
    table = torch.randperm(npg, device="cuda")[:b * mp].view(b, mp).int()
    kc = torch.randn(npg, ps, g, d, device="cuda", dtype=torch.float16)
    vc = torch.randn_like(kc)
    o = m.gqa_decode_paged(b, h, g, npg, ps, mp, d, num_split=ns)(q, kc, vc, lens, table, glse, part)
    ref = m.ref_program(q, m.paged_to_contiguous(kc, table, mp, ps), m.paged_to_contiguous(vc, table, mp, ps), lens)
    torch.testing.assert_close(o, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("sq,skv,win", [(1024, 1024, None), (512, 1536, None), (1024, 1024, 256)])
def test_attention_sink(sq, skv, win):
    import example_gqa_sink_fwd_bhsd as m
    k = m.flashattn_sink(2, 16, sq, skv, 128, 8, win)
    q = torch.randn(2, 16, sq, 128, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(2, 2, skv, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(kk)
    s = torch.randn(16, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(k(q, kk, v, s).float(), m.ref_program(q, kk, v, s, win).float(), rtol=2e-2, atol=2e-2)


def test_linear_attention_fwd():
    import example_linear_attn_fwd as m
    B, S, H, D = 2, 1024, 4, 128
    k = m.linear_attn_fwd(B, S, H, D, D)
    q = torch.nn.functional.normalize(torch.randn(B, S, H, D, device="cuda"), dim=-1).half()
    kk = torch.nn.functional.normalize(torch.randn(B, S, H, D, device="cuda"), dim=-1).half()
    v = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16)
    o, h = k(q, kk, v)
    ro, rh = m.ref_program(q, kk, v)
    torch.testing.assert_close(o.float(), ro, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(h, rh, rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize("xcd_group,lean,factored,xscale", [(False, False, False, False), (True, False, False, False),
                                                            (True, True, False, False), (True, False, True, False),
                                                            (False, False, False, True)])
def test_mamba_chunk_scan(xcd_group, lean, factored, xscale):
    import example_mamba_chunk_scan as m
    args = m.make_inputs(2, 4096, 256, 1, 8, 64, 128)
    k = m.chunk_scan_fwd(2, 4096, 256, 1, 8, 64, 128, block_K=64, xcd_group=xcd_group, lean=lean, factored=factored,
                         xscale=xscale)
    torch.testing.assert_close(k(*args).float(), m.ref_program(*args), rtol=2e-2, atol=5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("mask_split,heavy_first", [(True, False), (True, True)])
def test_mamba_chunk_scan_mask_split(mask_split, heavy_first):
    import example_mamba_chunk_scan as m
    args = m.make_inputs(2, 4096, 256, 1, 8, 64, 128)
    k = m.chunk_scan_fwd(2, 4096, 256, 1, 8, 64, 128, block_K=64, mask_split=mask_split, heavy_first=heavy_first)
    torch.testing.assert_close(k(*args).float(), m.ref_program(*args), rtol=2e-2, atol=5e-2)


def test_mamba_chunk_scan_factored_strong_decay():
    import example_mamba_chunk_scan as m
    args = m.make_inputs(1, 1024, 256, 1, 4, 64, 128)
    args[3] = (-torch.rand(1, 4, 4, 256, device="cuda") * 4.0).cumsum(-1).half()
    for kw in (dict(factored=True), dict(xscale=True)):
        k = m.chunk_scan_fwd(1, 1024, 256, 1, 4, 64, 128, block_K=64, **kw)
        out = k(*args).float()
        assert torch.isfinite(out).all()
        torch.testing.assert_close(out, m.ref_program(*args), rtol=2e-2, atol=5e-2)


def test_dequant_gemm_w4a16():
    import example_dequant_gemm_w4a16 as m
    for M in (16, 256):
        k = m.dequant_gemm_w4a16(M, 1024, 2048)
        A = torch.randn(M, 2048, device="cuda", dtype=torch.float16)
        W = torch.randn(1024, 2048, device="cuda", dtype=torch.float16)
        Bq, s = m.quantize_int4(W)
        torch.testing.assert_close(k(A, Bq, s).float(), m.ref_program(A, Bq, s).float(), rtol=1e-2, atol=5e-1)


def test_convolution_im2col():
    import example_convolution as m
    for (n, c, h, w, f, k, s, d, p) in ((8, 64, 32, 32, 128, 3, 1, 1, 1), (4, 64, 33, 33, 128, 3, 2, 1, 1)):
        kern = m.convolution(n, c, h, w, f, k, s, d, p)
        a = torch.randn(n, h, w, c, device="cuda", dtype=torch.float16)
        b = torch.randn(k, k, c, f, device="cuda", dtype=torch.float16)
        torch.testing.assert_close(kern(a, b).float(), m.ref_program(s, p, d)(a, b).float(), rtol=1e-2, atol=1e-1)


def test_fused_moe_shared_plus_routed():
    import example_fusedmoe_tilelang as m
    w = m.init_weights(1024, 512, 8, 1)
    x = torch.randn(1, 512, 1024, device="cuda", dtype=torch.float16)
    out = m.FusedMoE(w, 4)(x)
    torch.testing.assert_close(out.float(), m.ref_program(x, w, 4).float(), rtol=2e-2, atol=2e-2)


def test_deepseek_v32_kernels():
    import fp8_lighting_indexer as li
    import sparse_mla_fwd as sm
    import topk_selector as ts
    S, SKV, H, D = 256, 1024, 64, 128
    q, kv, sc, w, ks, ke = li.make_inputs(S, SKV, H, D)
    logits = li.mqa_attn_return_logits(S, SKV, H, D)(q.view(S * H, D), kv, sc, w, ks, ke)
    ref = li.ref_program(q, kv, sc, w, ks, ke)
    fin = torch.isfinite(ref)
    assert torch.equal(torch.isfinite(logits), fin)
    torch.testing.assert_close(logits[fin], ref[fin], rtol=2e-2, atol=2e-2)
    x = torch.randn(512, 4096, device="cuda")
    ts.check(x, ts.topk_selector(512, 4096, 512)(x), 512)
    B, S2, SKV2, H2, topk = 1, 16, 512, 128, 256
    qq = torch.randn(B, S2, H2, 576, device="cuda", dtype=torch.bfloat16)
    kv2 = torch.randn(B, SKV2, 1, 576, device="cuda", dtype=torch.bfloat16)
    idx = sm.make_indices(B, S2, SKV2, 1, topk, "cuda")
    o, _ = sm.sparse_mla_fwd(B, S2, SKV2, H2, 512, 64, topk)(qq, kv2, idx)
    torch.testing.assert_close(o.float().cpu(), sm.ref_program(qq.cpu(), kv2.cpu(), idx.cpu(), 512).float(),
                               rtol=3e-2, atol=3e-2)


def test_deepseek_v32_model_on_gpu():
    from tilelang.models.deepseek_v32 import ModelArgs, Transformer, generate
    args = ModelArgs.tiny()
    m = Transformer(args, seed=0, device="cuda")
    toks = torch.randint(0, args.vocab_size, (2, 12), generator=torch.Generator().manual_seed(1)).cuda()
    full = m(toks, 0)
    m2 = Transformer(args, seed=0, device="cuda")
    m2(toks[:, :11], 0)
    torch.testing.assert_close(m2(toks[:, 11:12], 11), full, rtol=3e-2, atol=3e-2)
    cpu = Transformer(args, seed=0, device="cpu")(toks.cpu(), 0)
    torch.testing.assert_close(full.cpu(), cpu, rtol=5e-2, atol=5e-2)
    assert len(generate(m, [[1, 2, 3], [4, 5, 6, 7]], 4)[0]) == 4


def test_gemm_persistent_streamk_blocksparse():
    import example_gemm_persistent as gp
    import example_tilelang_gemm_streamk as sk
    import example_blocksparse_gemm as bs
    a = torch.randn(1024, 512, device="cuda", dtype=torch.float16)
    b = torch.randn(512, 768, device="cuda", dtype=torch.float16)
    torch.testing.assert_close(gp.matmul_persistent(1024, 768, 512, 128, 128, 64, 256)(a, b).float(),
                               a.float() @ b.float(), rtol=1e-2, atol=1e-1)
    A = torch.rand(256, 512, device="cuda", dtype=torch.float16) * 2 - 1
    B = torch.rand(1024, 512, device="cuda", dtype=torch.float16) * 2 - 1
    C = torch.zeros(256, 1024, device="cuda")
    sk.matmul_streamk(256, 1024, 512)(A, B, C)
    torch.testing.assert_close(C, A.float() @ B.float().t(), rtol=1e-2, atol=1e-2)
    mask = torch.rand(8, 6, 16, device="cuda") > 0.5
    out = bs.blocksparse_matmul(1024, 768, 512)(a, b, mask)
    torch.testing.assert_close(out.float(), bs.ref_program(a, b, mask, 128, 128, 32).float(), rtol=1e-2, atol=1e-1)


def test_gather_rows_gpu():
    from test_examples_cpu import _gather_rows_check
    _gather_rows_check("cuda", "hip")


def test_nsa_fwd_and_decode_gpu():
    from example_nsa_fwd import nsa_fwd, make_block_indices, ref_program
    B, SKV, HQ, H, D, S, BS = 2, 512, 32, 2, 128, 4, 64
    for SQ in (256, 1):  # prefill and decode (one query at the end of the cache)
        k = nsa_fwd(B, HQ, SQ, SKV, D, True, None, BS, HQ // H, S)
        q = torch.randn(B, SQ, HQ, D, device="cuda", dtype=torch.bfloat16)
        kk = torch.randn(B, SKV, H, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, SKV, H, D, device="cuda", dtype=torch.bfloat16)
        bi = make_block_indices(B, SQ, SKV, H, S, BS, "cuda")
        torch.testing.assert_close(k(q, kk, v, bi).float().cpu(), ref_program(q, kk, v, bi, BS).float(), rtol=2e-2,
                                   atol=2e-2)


def test_block_sparse_attn_gpu():
    from example_block_sparse_attn import blocksparse_attn, compact_mask, random_block_mask, ref_program
    B, H, S, D = 1, 4, 1024, 128
    k_ = blocksparse_attn(B, H, S, D)
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    mask = random_block_mask(B, H, S // 64, 0.3, True, "cuda")
    idx, cnt = compact_mask(mask)
    torch.testing.assert_close(k_(q, k, v, idx, cnt).float(), ref_program(q, k, v, mask).float(), rtol=2e-2, atol=2e-2)


def test_gdn_chunked_gpu():
    from example_gdn import chunk_gated_delta_rule, make_inputs, naive_recurrent
    q, k, v, g, beta = make_inputs(2, 256, 2, 128, 64, "cuda")
    o, hf = chunk_gated_delta_rule(q, k, v, g, beta)
    o_ref, h_ref = naive_recurrent(q, k, v, g, beta)
    torch.testing.assert_close(o.float().cpu(), o_ref, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(hf.cpu(), h_ref, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_gqa_attention_bwd_gpu(causal):
    import example_mha_bwd as m
    B, S, H, HKV, D = 2, 512, 8, 2, 64
    Q = torch.randn(B, S, H, D, dtype=torch.bfloat16, device="cuda").requires_grad_()
    K = torch.randn(B, S, HKV, D, dtype=torch.bfloat16, device="cuda").requires_grad_()
    V = torch.randn(B, S, HKV, D, dtype=torch.bfloat16, device="cuda").requires_grad_()
    dO = torch.randn_like(Q)
    m.attention(Q, K, V, causal).backward(dO)
    grads = [t.grad.clone() for t in (Q, K, V)]
    for t in (Q, K, V):
        t.grad = None
    m.ref_program(Q, K, V, causal).backward(dO)
    for g, t in zip(grads, (Q, K, V)):
        torch.testing.assert_close(g.float(), t.grad.float(), rtol=3e-2, atol=5e-2)


def test_mla_decode_paged_gpu():
    from example_mla_decode_paged import make_paged_cache, mla_decode_paged, ref_program
    b, h, S, ps, ns = 4, 128, 1024, 64, 4
    q = torch.randn(b, h, 512, device="cuda", dtype=torch.bfloat16)
    qpe = torch.randn(b, h, 64, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(b, S, 512, device="cuda", dtype=torch.bfloat16)
    kpe = torch.randn(b, S, 64, device="cuda", dtype=torch.bfloat16)
    sl = torch.tensor([1024, 77, 640, 300], dtype=torch.int32, device="cuda")
    kvp, pep, tab = make_paged_cache(kv, kpe, sl, ps)
    k = mla_decode_paged(b, h, S, kvp.shape[0], ps, num_split=ns)
    o = k(q, qpe, kvp, pep, tab, sl, torch.empty(b, h, ns, device="cuda"), torch.empty(b, h, ns, 512, device="cuda"))
    torch.testing.assert_close(o.float(), ref_program(q, qpe, kv, kpe, sl).float(), rtol=2e-2, atol=2e-2)


def test_grouped_gemm_autograd_gpu():
    import example_grouped_gemm_bwd as m
    m.main((64, 300, 1024, 17), 512, 1024)


def test_dequant_gemm_mxfp4_gpu():
    from example_dequant_gemm_mxfp4 import dequant_gemm_mxfp4, ref_program
    from tilelang.quantize import quantize_mxfp4
    M, N, K = 64, 1024, 2048
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
    torch.testing.assert_close(dequant_gemm_mxfp4(M, N, K)(A, Bq, S).float(), ref_program(A, Bq, S).float(),
                               rtol=2e-2, atol=1.0)


@pytest.mark.parametrize("M,N,K", [(1, 8192, 8192), (4, 1000, 4096), (8, 512, 1024)])
def test_mxfp4_gemv_gpu(M, N, K):
    """Decode GEMV over MXFP4 weights (tl/gemv.h: hardware fp4 -> bf16 conversion + dot2)."""
    from example_dequant_gemm_mxfp4 import mxfp4_gemv, ref_program
    from tilelang.quantize import quantize_mxfp4
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
    k = mxfp4_gemv(M, N, K)
    assert "mxfp4_gemv<" in k.get_kernel_source()
    torch.testing.assert_close(k(A, Bq, S).float(), ref_program(A, Bq, S).float(), rtol=2e-2, atol=1.0)


@pytest.mark.parametrize("dkv", ["gather", "atomic"])
def test_sparse_mla_bwd_gpu(dkv):
    import sparse_mla_bwd as m
    from tilelang.ops.dsa import sparse_mla_fwd
    B, S, SKV, H, topk = 1, 64, 256, 64, 128
    q = (torch.randn(B, S, H, 576, device="cuda") / 4).bfloat16()
    kv = (torch.randn(B, SKV, 1, 576, device="cuda") / 4).bfloat16()
    do = torch.randn(B, S, H, 512, device="cuda", dtype=torch.bfloat16)
    r = torch.rand(S, SKV, device="cuda")
    pos = torch.arange(S, device="cuda")[:, None] + SKV - S
    r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
    idx = r.topk(topk, -1).indices.int()
    idx = torch.where(torch.gather(r, 1, idx.long()) >= 0, idx, torch.full_like(idx, SKV)).view(B, S, 1, topk)
    o, lse = sparse_mla_fwd(B, S, SKV, H, 512, 64, topk)(q, kv, idx)
    dq, dkv_ = m.sparse_mla_bwd(q, kv, o, do, idx, lse, dkv=dkv)
    rq, rkv = m.ref_bwd(q, kv, do, idx)
    torch.testing.assert_close(dq.float().cpu(), rq, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(dkv_.cpu(), rkv, rtol=3e-2, atol=3e-2)


def test_attention_sink_autograd_gpu():
    import example_gqa_sink_bwd as m
    B, S, H, G, D = 2, 512, 8, 4, 64
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    k = torch.randn(B, S, H // G, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    v = torch.randn(B, S, H // G, D, device="cuda", dtype=torch.bfloat16).requires_grad_()
    sinks = torch.randn(H, device="cuda").requires_grad_()
    do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    m.attention_sink(q, k, v, sinks).backward(do)
    grads = [t.grad.clone() for t in (q, k, v, sinks)]
    for t in (q, k, v, sinks):
        t.grad = None
    m.ref_program(q, k, v, sinks).backward(do)
    for g, t in zip(grads, (q, k, v, sinks)):
        torch.testing.assert_close(g.float(), t.grad.float(), rtol=3e-2, atol=5e-2)


def test_flash_attention_varlen_gpu():
    from example_mha_fwd_varlen import flashattn_varlen, make_varlen, ref_program
    q, k, v, cq, ck = make_varlen([300, 1024, 77, 513], [300, 1100, 200, 513], 8, 2, 128, "cuda")
    o = flashattn_varlen(4, 8, q.shape[0], k.shape[0], 1024, 128, True, 4)(q, k, v, cq, ck)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, cq, ck).float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("paged", [False, True])
def test_gqa_decode_varlen_logits(paged):
    import example_gqa_decode_varlen_logits as m
    lens, b, h, kh, d = [1500, 4096, 377, 2900], 4, 32, 8, 128
    q, k, v, cu, s_aux, kp, vp, table = m.make_inputs(lens, h, kh, d, "cuda", torch.float16, True, page_size=128)
    ro, rs = m.ref_program(q, k, v, cu, s_aux, 64)
    if paged:
        kern = m.flashattn_paged(b, h, kh, max(lens), kp.shape[0], d, True, 128)
        o, s = m.AttnPoolDecode(kern, b, h, d, 8, max(lens), 64, "cuda")(q, kp, vp, cu, s_aux, table)
    else:
        kern = m.flashattn(b, h, kh, max(lens), k.shape[0], d, True)
        o, s = m.AttnPoolDecode(kern, b, h, d, 8, max(lens), 64, "cuda")(q, k, v, cu, s_aux)
    torch.testing.assert_close(o.float(), ro, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(s.float(), rs, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_mha_inference_split_kv(causal):
    import example_mha_inference as m
    b, h, sq, sk, d, ns = 2, 8, 128, 2048, 128, 8
    k = m.flashattn(b, h, sq, sk, d, causal, num_split=ns)
    q = torch.randn(b, sq, h, d, device="cuda", dtype=torch.float16)
    kk, v = torch.randn(b, sk, h, d, device="cuda", dtype=torch.float16), torch.randn(b, sk, h, d, device="cuda",
                                                                                       dtype=torch.float16)
    o = k(q, kk, v, torch.empty(b, h, ns, sq, device="cuda"), torch.empty(b, sq, h, ns, d, device="cuda"))
    torch.testing.assert_close(o.float(), m.ref_program(q, kk, v, causal).float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_flash_attention_varlen_reference_entry_gpu(causal):
    """The reference-named flashattn(batch, UQ, UKV, heads, dim, causal) entry; non-causal is its default."""
    from example_mha_fwd_varlen import flashattn, make_varlen, ref_program
    lens = [300, 1024, 77, 513]
    q, k, v, cq, ck = make_varlen(lens, lens, 8, 8, 128, "cuda", torch.float16)
    kern = flashattn(4, q.shape[0], k.shape[0], 8, 128, causal)
    o = kern(q, k, v, cq, ck, max(lens))
    torch.testing.assert_close(o.float(), ref_program(q, k, v, cq, ck, causal).float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("causal", [False, True])
def test_mha_fwd_bhsd(causal):
    import example_mha_fwd_bhsd as m
    m.main(2, 8, 256, 1024, 128, causal)


def test_gqa_fwd_bshd():
    import example_gqa_fwd_bshd as m
    m.main(1, 32, 1024, 128, True, 8)


@pytest.mark.parametrize("causal", [False, True])
def test_gqa_bwd_qk192_v128(causal):
    import example_gqa_bwd as m
    m.main(1, 16, 512, 192, 128, 8, causal)


def test_mha_sink_fwd_bhsd():
    import example_mha_sink_fwd_bhsd as m
    m.main(1, 8, 512, 512, 128, None)
    m.main(1, 8, 512, 512, 128, 128)
