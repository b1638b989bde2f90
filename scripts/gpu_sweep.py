"""Config sweeps of example kernels on one MI355X.

    python scripts/gpu_sweep.py <workload> '<json cfg>' ['<json cfg>' ...]
workloads: sink, mamba, fa_bwd, linear_attn, decode.  Each config is checked against the
PyTorch reference where cheap, then timed with do_bench; one JSON line per config.
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT] + sorted(d for d in glob.glob(os.path.join(ROOT, "examples", "*")) if os.path.isdir(d))
import torch  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402


def w_sink(c):
    import example_gqa_sink_fwd_bhsd as m
    B, H, S, D, G = 1, 64, 4096, 128, 8
    q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(B, H // G, S, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(kk)
    s = torch.randn(H, device="cuda", dtype=torch.bfloat16)
    k = m.flashattn_sink(B, H, S, S, D, G, **c)
    o = k(q, kk, v, s)
    if c.get("causal", True):
        ref = m.ref_program(q[:, :8], kk[:, :1], v[:, :1], s[:8]).float()
        torch.testing.assert_close(o[:, :8].float(), ref, rtol=2e-2, atol=2e-2)
    ms = do_bench(lambda: k(q, kk, v, s))
    return ms, m.flops(B, H, S, S, D) * (1 if c.get("causal", True) else 2)


def w_mamba(c):
    import example_mamba_chunk_scan as m
    small = m.make_inputs(1, 512, 256, 1, 4, 64, 128)
    ks = m.chunk_scan_fwd(1, 512, 256, 1, 4, 64, 128, **c)
    torch.testing.assert_close(ks(*small).float(), m.ref_program(*small), rtol=2e-2, atol=5e-2)
    args = m.make_inputs(8, 4096, 256, 1, 80, 64, 128)
    k = m.chunk_scan_fwd(8, 4096, 256, 1, 80, 64, 128, **c)
    ms = do_bench(lambda: k(*args))
    return ms, m.flops(8, 4096, 256, 80, 64, 128)


def w_fa_bwd(c):
    import example_mha_bwd as m
    B, S, H, D = 8, 1024, 32, 64
    q, k_, v, do = [torch.randn(B, S, H, D, dtype=torch.half, device="cuda") for _ in range(4)]
    o, lse = m.flashattn_fwd(B, H, S, D, False)(q, k_, v)
    delta = m.flashattn_bwd_preprocess(B, H, S, D)(o, do)
    kern = m.flashattn_bwd(B, H, S, D, False, **c)
    dq = torch.zeros(B, S, H, D, dtype=torch.float32, device="cuda")
    dk, dv = torch.empty_like(q), torch.empty_like(q)

    def run():
        kern(q, k_, v, do, lse, delta, dq, dk, dv)

    run()
    qf, kf, vf = [t[:1].float().requires_grad_() for t in (q, k_, v)]
    m.ref_program(qf, kf, vf, False).float().backward(do[:1].float())
    torch.testing.assert_close(dk[:1].float(), kf.grad, rtol=3e-2, atol=3e-2)
    ms = do_bench(run)
    return ms, 4 * 2.0 * B * H * S * S * D  # this kernel runs 4 of the 5 backward GEMMs


def w_linear_attn(c):
    import example_linear_attn_fwd as m
    B, S, H, D = 1, 8192, 32, 128
    k = m.linear_attn_fwd(B, S, H, D, D, **c)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) * 0.1
    kk = torch.randn_like(q) * 0.1
    v = torch.randn_like(q)
    ms = do_bench(lambda: k(q, kk, v))
    return ms, B * H * (S // 64) * (2 * 64 * 64 * D * 2 + 2 * 64 * D * D * 2)


def w_decode(c):
    import example_gqa_decode as m
    b, h, g, s, d = 32, 32, 8, 8192, 128
    ns = c.pop("num_split", 8)
    k = m.gqa_decode(b, h, g, s, d, num_split=ns, **c)
    q = torch.randn(b, h, d, device="cuda", dtype=torch.float16)
    kk = torch.randn(b, s, g, d, device="cuda", dtype=torch.float16)
    v = torch.randn_like(kk)
    lens = torch.full((b, ), s, dtype=torch.int32, device="cuda")
    glse = torch.empty(b, h, ns, device="cuda")
    part = torch.empty(b, h, ns, d, device="cuda")
    ms = do_bench(lambda: k(q, kk, v, lens, glse, part))
    return ms, None, 2 * b * s * g * d * 2


def w_fa_fwd(c):
    import example_mha_fwd as m
    B, H, S, D = 1, 64, 4096, 128
    causal = c.pop("causal", False)
    q, k_, v = [torch.randn(B, S, H, D, dtype=torch.bfloat16, device="cuda") for _ in range(3)]
    k = m.flashattn(B, H, S, D, causal, 1, **c)
    o = k(q, k_, v)
    torch.testing.assert_close(o[:, :, :2].float(), m.ref_program(q[:, :, :2], k_[:, :, :2], v[:, :, :2], causal).float(),
                               rtol=2e-2, atol=2e-2)
    return do_bench(lambda: k(q, k_, v)), 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)


def w_fa_fwd_lse(c):
    import example_mha_bwd as m
    B, H, S, D, G = 1, 64, 4096, 128, 8
    q = torch.randn(B, S, H, D, dtype=torch.bfloat16, device="cuda")
    k_, v = [torch.randn(B, S, H // G, D, dtype=torch.bfloat16, device="cuda") for _ in range(2)]
    k = m.flashattn_fwd(B, H, S, D, True, dtype="bfloat16", groups=G, **c)
    o, _ = k(q, k_, v)
    torch.testing.assert_close(o[:, :256].float(), m.ref_program(q[:, :256], k_[:, :256], v[:, :256], True).float(),
                               rtol=2e-2, atol=2e-2)
    return do_bench(lambda: k(q, k_, v)), 4.0 * B * H * S * S * D * 0.5


def w_varlen(c):
    import example_mha_fwd_varlen as m
    B, L, H, G, D = 8, 4096, 32, 4, 128
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(L // 4, L + 1, (B, ), generator=g).tolist()
    q, k_, v, cq, ck = m.make_varlen(lens, lens, H, H // G, D, "cuda")
    k = m.flashattn_varlen(B, H, q.shape[0], k_.shape[0], max(lens), D, True, G, **c)
    k(q, k_, v, cq, ck)
    return do_bench(lambda: k(q, k_, v, cq, ck)), sum(2 * 2.0 * H * x * x * D * 0.5 for x in lens)


def w_sink_lazy(c):
    return w_sink(c)


if __name__ == "__main__":
    fn = globals()["w_" + sys.argv[1]]
    for a in sys.argv[2:]:
        c = json.loads(a)
        try:
            r = fn(dict(c))
            ms, fl = r[0], r[1]
            out = dict(cfg=c, ms=round(ms, 4))
            if fl:
                out["TFLOPS"] = round(fl / ms * 1e-9, 1)
            if len(r) > 2:
                out["GBs"] = round(r[2] / ms * 1e-6, 1)
            print(json.dumps(out), flush=True)
        except Exception as e:  # noqa: BLE001 - report and continue
            print(json.dumps(dict(cfg=c, error=f"{type(e).__name__}: {str(e)[:300]}")), flush=True)
