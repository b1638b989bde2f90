"""A/B of ``tl.pipeline_unroll`` (lowered pipelined main loops emitted under #pragma unroll N, so the
LDS ring slot of each copy is a constant) on the secondary kernels, one process, round-robin after a
pre-warm; outputs compared bitwise between the builds (the unroll changes no arithmetic).

    python scripts/unroll_ab.py [--unroll 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT] + [os.path.join(ROOT, "examples", d) for d in ("flash_attention", "linear_attention")]

import torch  # noqa: E402

import tilelang  # noqa: E402


def build(jitfn, args, kwargs, extra):
    pc = dict(getattr(jitfn, "pass_configs", None) or {})
    pc.update(extra)
    f = jitfn.get_tir(*args, **kwargs)
    return tilelang.compile(f, out_idx=getattr(jitfn, "out_idx", None), target="hip", pass_configs=pc)


def _base(tiles):
    """A tile config without its own unroll (the A/B sets it through the pass config)."""
    return {k: v for k, v in tiles.items() if k != "unroll"}


def cases(only=None):
    out = []
    if only in (None, "fa_bwd"):
        import example_mha_bwd as E
        B, H, S, D = 8, 32, 1024, 64
        q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
        for causal in (False, True):
            o, lse = E.flashattn_fwd(B, H, S, D, causal, dtype="float16")(q, k, v)
            delta = E.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
            fl = 2.0 * B * H * S * S * D * (0.5 if causal else 1.0)
            dk = torch.empty(B, S, H, D, device="cuda", dtype=torch.float16)
            dv = torch.empty(B, S, H, D, device="cuda", dtype=torch.float16)
            tag = "causal" if causal else "non-causal"
            # the autograd path's tiles (example_mha_bwd._tiles); outputs written in place: compared
            # through the (-2, -1) argument slots
            out.append((f"FA bwd dK/dV {tag} fp16 b8 h32 s1024 d64", E.flashattn_bwd, (B, H, S, D, causal),
                        dict(dq_mode="none", **_base(E._tiles(D, D, "bwd", causal))), (q, k, v, do, lse, delta, dk, dv),
                        4 * fl, (-2, -1)))
            out.append((f"FA bwd dQ {tag} fp16 b8 h32 s1024 d64", E.flashattn_bwd_dq, (B, H, S, D, causal),
                        _base(E._tiles(D, D, "dq", causal)), (q, k, v, do, lse, delta), 3 * fl, None))
    if only in (None, "smla"):
        from tilelang.ops.dsa import sparse_mla_fwd
        Bs, Ss, SKV, Hs, topk = 1, 4096, 8192, 128, 2048
        qs = torch.randn(Bs, Ss, Hs, 576, device="cuda", dtype=torch.bfloat16)
        kvs = torch.randn(Bs, SKV, 1, 576, device="cuda", dtype=torch.bfloat16)
        r = torch.rand(Ss, SKV, device="cuda")
        pos = torch.arange(Ss, device="cuda")[:, None] + SKV - Ss
        r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
        idx = r.topk(topk, dim=-1).indices.int().view(Bs, Ss, 1, topk)
        out.append(("sparse MLA fwd b1 s4096 h128 topk2048", sparse_mla_fwd, (Bs, Ss, SKV, Hs, 512, 64, topk), {},
                    (qs, kvs, idx), 2.0 * Bs * Ss * Hs * topk * (576 + 512), None))
    if only in (None, "mamba"):
        from example_mamba_chunk_scan import chunk_scan_fwd, make_inputs
        L = 4096
        margs = make_inputs(8, L, 256, 1, 80, 64, 128)
        out.append(("Mamba-2 chunk scan 4K", chunk_scan_fwd, (8, L, 256, 1, 80, 64, 128),
                    dict(block_M=128, block_N=64, block_K=32, threads=256), margs, None, None))
    return out


def _outs(res, inputs, slots):
    if slots is not None:
        return [inputs[i].clone() for i in slots]
    return list(res) if isinstance(res, (list, tuple)) else [res]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--unroll", type=int, default=2)
    ap.add_argument("--only", choices=["fa_bwd", "smla", "mamba"], default=None)
    ap.add_argument("--pc", default=None, help='B variant pass configs instead of the unroll, e.g. \'{"tl.enable_fast_math": true}\'')
    a = ap.parse_args()
    torch.manual_seed(0)
    runs = []
    for name, fn, args, kw, inputs, flops, slots in cases(a.only):
        ks = []
        bvar = ("pc", json.loads(a.pc)) if a.pc else (f"unroll{a.unroll}", {"tl.pipeline_unroll": a.unroll})
        for tag, extra in (("base", {}), bvar):
            try:
                kern = build(fn, args, kw, extra)
                ks.append((tag, kern, _outs(kern(*inputs), inputs, slots)))
            except Exception as e:  # noqa: BLE001
                print(f"{name} {tag}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
        if len(ks) == 2:
            r0, r1 = ks[0][2], ks[1][2]
            same = all(torch.equal(x, y) for x, y in zip(r0, r1))
            print(f"{name}: outputs identical: {same}", flush=True)
            if not same:
                d = max((x.float() - y.float()).abs().max().item() for x, y in zip(r0, r1))
                print(f"{name}: max abs diff {d:.3g} (fp contraction under the unrolled body)", flush=True)
        for tag, kern, _ in ks:
            runs.append((name, tag, kern, inputs, flops))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _, _, kern, inputs, _ in runs:
            kern(*inputs)
        torch.cuda.synchronize()
    res = {(n, t): [] for n, t, _, _, _ in runs}
    for _ in range(5):
        for n, t, kern, inputs, _ in runs:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                kern(*inputs)
            e1.record()
            torch.cuda.synchronize()
            res[(n, t)].append(e0.elapsed_time(e1) / 10)
    for n, t, _, _, fl in runs:
        ms = sorted(res[(n, t)])[2]
        extra = f", {fl / ms * 1e-9:.1f} TF" if fl else ""
        print(f"{n} [{t}]: {ms:.4f} ms{extra}", flush=True)


if __name__ == "__main__":
    main()
