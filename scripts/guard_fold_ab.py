"""A/B of the gemm wave-guard folding (tl/gemm.h TL_GEMM_FOLD_DEFAULT_GUARD) on the kernels that
call T.gemm with per-tile cleared / initialised accumulators: the bench FA forward, the FA backward
dK/dV and dQ kernels, the GQA+sink forward.  Both builds of every kernel are compiled in ONE
process (the old behaviour via -DTL_GEMM_FOLD_DEFAULT_GUARD=0), checked against each other, then
timed round-robin after a pre-warm (median of 5 rounds of 20 launches).

    python scripts/guard_fold_ab.py
"""
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT] + sorted(d for d in glob.glob(os.path.join(ROOT, "examples", "*")) if os.path.isdir(d))
import torch  # noqa: E402

import tilelang  # noqa: E402

OLD = ["-DTL_GEMM_FOLD_DEFAULT_GUARD=0"]


def build(impl, args, kwargs=None, flags=None):
    pc = dict(getattr(impl, "pass_configs", None) or {})
    pc.pop("tl.gemm_fold_default_guard", None)  # the A/B sets the macro itself
    pc.pop(tilelang.PassConfigKey.TL_GEMM_FOLD_DEFAULT_GUARD, None)
    return tilelang.compile(impl.get_tir(*args, **(kwargs or {})), out_idx=impl.out_idx, target="hip",
                            pass_configs=pc, compile_flags=flags)


def cases():
    out = []
    import example_mha_fwd_pipelined as fa
    a = dict(q_in_regs=True, sum_mfma=True, fold_max=True, young_prio=True, xcd_heads=True)
    args = (1, 64, 4096, 128, False, 1, 256, 64, 512, 2, "bfloat16", True)
    q, k, v = (torch.randn(1, 4096, 64, 128, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    out.append(("FA fwd bench", 4.0 * 64 * 4096 * 4096 * 128, [build(fa.flashattn_pipelined, args, a, f)
                                                               for f in (None, OLD)], (q, k, v)))
    import example_mha_bwd as m
    B, S, H, D = 8, 1024, 32, 64
    qq, kk, vv, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
    o, lse = m.flashattn_fwd(B, H, S, D, False, dtype="float16")(qq, kk, vv) if hasattr(m, "flashattn_fwd") else (
        None, None)
    if lse is None:
        raise SystemExit("example_mha_bwd has no flashattn_fwd")
    delta = m.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
    dk, dv = torch.empty_like(kk), torch.empty_like(vv)
    flops_kv = 4 * 2.0 * B * H * S * S * D
    bw = m._tiles(D, D, "bwd", False)
    out.append(("FA bwd dK/dV", flops_kv, [build(m.flashattn_bwd, (B, H, S, D, False), dict(dtype="float16",
                                                                                       dq_mode="none", **bw), f)
                                           for f in (None, OLD)], (qq, kk, vv, do, lse, delta, dk, dv)))
    dqt = m._tiles(D, D, "dq", False)
    out.append(("FA bwd dQ", 3 * 2.0 * B * H * S * S * D, [build(m.flashattn_bwd_dq, (B, H, S, D, False),
                                                                 dict(dtype="float16", **dqt), f)
                                                           for f in (None, OLD)], (qq, kk, vv, do, lse, delta)))
    import example_mla_decode as md
    bb, hh, ctx, dd, pe = 64, 128, 8192, 512, 64
    mq = torch.randn(bb, hh, dd, device="cuda", dtype=torch.float16)
    mqp = torch.randn(bb, hh, pe, device="cuda", dtype=torch.float16)
    mkv = torch.randn(bb, ctx, 1, dd, device="cuda", dtype=torch.float16)
    mkp = torch.randn(bb, ctx, 1, pe, device="cuda", dtype=torch.float16)
    glse = torch.empty(bb, hh, 4, device="cuda")
    part = torch.empty(bb, hh, 4, dd, device="cuda")
    out.append(("MLA decode b64 h128 kv8192", md.flops(bb, hh, ctx, dd, pe),
                [build(md.mla_decode, (bb, hh, 1, ctx, dd, pe), dict(num_split=4), f) for f in (None, OLD)],
                (mq, mqp, mkv, mkp, glse, part)))
    from tilelang.ops import dsa
    Bs, Ss, SKV, Hs, topk = 1, 2048, 8192, 128, 2048
    sq = torch.randn(Bs, Ss, Hs, 576, device="cuda", dtype=torch.bfloat16)
    skv = torch.randn(Bs, SKV, 1, 576, device="cuda", dtype=torch.bfloat16)
    r = torch.rand(Ss, SKV, device="cuda")
    pos = torch.arange(Ss, device="cuda")[:, None] + SKV - Ss
    r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
    idx = r.topk(topk, dim=-1).indices.int().view(Bs, Ss, 1, topk)
    out.append(("sparse MLA fwd s2048 h128 topk2048", 2.0 * Bs * Ss * Hs * topk * (576 + 512),
                [build(dsa.sparse_mla_fwd, (Bs, Ss, SKV, Hs, 512, 64, topk), None, f) for f in (None, OLD)],
                (sq, skv, idx)))
    import example_gqa_sink_fwd_bhsd as sk
    gq = torch.randn(1, 64, 4096, 128, device="cuda", dtype=torch.bfloat16)
    gk = torch.randn(1, 8, 4096, 128, device="cuda", dtype=torch.bfloat16)
    gv = torch.randn_like(gk)
    gs = torch.randn(64, device="cuda", dtype=torch.bfloat16)
    out.append(("GQA+sink fwd causal s4096", sk.flops(1, 64, 4096, 4096, 128),
                [build(sk.flashattn_sink, (1, 64, 4096, 4096, 128, 8), None, f) for f in (None, OLD)],
                (gq, gk, gv, gs)))
    return out


def main():
    cs = cases()
    for name, _, (new, old), args in cs:
        r1, r2 = new(*args), old(*args)
        r1 = r1 if isinstance(r1, (tuple, list)) else [r1]
        r2 = r2 if isinstance(r2, (tuple, list)) else [r2]
        same = all(torch.allclose(x.float(), y.float(), rtol=1e-3, atol=1e-3) for x, y in zip(r1, r2) if x is not None)
        print(f"{name}: new == old: {same}", flush=True)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _, _, ks, args in cs:
            for kk in ks:
                kk(*args)
        torch.cuda.synchronize()
    res = {}
    for rnd in range(5):
        for name, _, ks, args in cs:
            for tag, kk in zip(("new", "old"), ks):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    kk(*args)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((name, tag), []).append(e0.elapsed_time(e1) / 20)
    for name, flops, _, _ in cs:
        n = sorted(res[(name, "new")])[2]
        o = sorted(res[(name, "old")])[2]
        print(f"{name}: folded guard {n:.4f} ms ({flops / n * 1e-9:.0f} TF) | unconditional guard {o:.4f} ms "
              f"({flops / o * 1e-9:.0f} TF) | {o / n:.3f}x", flush=True)


if __name__ == "__main__":
    main()
