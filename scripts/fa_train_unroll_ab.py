"""A/B of the main-loop unroll (T.Pipelined(unroll=2)) on the training FA kernels of
examples/flash_attention/example_mha_bwd.py -- forward with LSE, dK/dV, dQ -- at the head sizes the
autograd path serves (d64, d128, d_qk 192 / d_v 128 with GQA), with the tiles example_mha_bwd._tiles
picks; outputs compared bitwise, times round-robin in one process.

    python scripts/fa_train_unroll_ab.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "flash_attention")]

import torch  # noqa: E402

import example_mha_bwd as E  # noqa: E402

SHAPES = [  # B, H, S, D, Dv, G, causal
    (8, 32, 1024, 64, 64, 1, False), (1, 8, 2048, 128, 128, 1, False), (4, 32, 2048, 128, 128, 1, False),
    (4, 32, 2048, 128, 128, 1, True), (1, 32, 4096, 192, 128, 16, False),
]


def strip(t):
    return {k: v for k, v in t.items() if k != "unroll"}


def main():
    torch.manual_seed(0)
    rows = []
    for B, H, S, D, Dv, G, causal in SHAPES:
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16)
        k = torch.randn(B, S, H // G, D, device="cuda", dtype=torch.float16)
        v = torch.randn(B, S, H // G, Dv, device="cuda", dtype=torch.float16)
        do = torch.randn(B, S, H, Dv, device="cuda", dtype=torch.float16)
        tag = f"B{B} H{H} S{S} D{D}/{Dv} G{G}{' causal' if causal else ''}"
        fl = 2.0 * B * H * S * S * (0.5 if causal else 1.0)
        base_f = strip(E._tiles(D, Dv, "fwd"))
        kf = {u: E.flashattn_fwd(B, H, S, D, causal, dtype="float16", groups=G, dim_v=Dv, unroll=u, **base_f)
              for u in (None, 2)}
        outs = {u: kf[u](q, k, v) for u in kf}
        o, lse = outs[None]
        same = all(torch.equal(a, b) for a, b in zip(outs[None], outs[2]))
        delta = E.flashattn_bwd_preprocess(B, H, S, Dv, dtype="float16")(o, do)
        base_b = strip(E._tiles(D, Dv, "bwd", causal))
        base_q = strip(E._tiles(D, Dv, "dq", causal))
        dk = torch.empty_like(k)
        dv = torch.empty_like(v)
        kb = {u: E.flashattn_bwd(B, H, S, D, causal, dtype="float16", dq_mode="none", groups=G, dim_v=Dv, unroll=u,
                                 **base_b) for u in (None, 2)}
        kq = {u: E.flashattn_bwd_dq(B, H, S, D, causal, dtype="float16", groups=G, dim_v=Dv, unroll=u, **base_q)
              for u in (None, 2)}
        res_b = {}
        for u in (None, 2):
            kb[u](q, k, v, do, lse, delta, dk, dv)
            res_b[u] = (dk.clone(), dv.clone(), kq[u](q, k, v, do, lse, delta))
        same_b = all(torch.equal(a, b) for a, b in zip(res_b[None], res_b[2]))
        print(f"{tag}: outputs identical fwd {same} bwd {same_b}", flush=True)
        for name, ks, args, f in (("fwd", kf, (q, k, v), fl * (D + Dv)),
                                  ("dK/dV", kb, (q, k, v, do, lse, delta, dk, dv), fl * (2 * D + 2 * Dv)),
                                  ("dQ", kq, (q, k, v, do, lse, delta), fl * (2 * D + Dv))):
            rows.append((tag, name, ks, args, f))
    for _ in range(3):  # warm
        for _, _, ks, args, _ in rows:
            for u in ks:
                ks[u](*args)
    torch.cuda.synchronize()
    res = {}
    for _ in range(5):
        for tag, name, ks, args, _ in rows:
            for u in ks:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    ks[u](*args)
                e1.record()
                torch.cuda.synchronize()
                res.setdefault((tag, name, u), []).append(e0.elapsed_time(e1) / 10)
    for tag, name, ks, _, f in rows:
        t0, t2 = sorted(res[(tag, name, None)])[2], sorted(res[(tag, name, 2)])[2]
        print(f"{tag} {name}: base {t0:.4f} ms ({f / t0 * 1e-9:.0f} TF), unroll2 {t2:.4f} ms ({f / t2 * 1e-9:.0f} TF), "
              f"{(t0 / t2 - 1) * 100:+.1f} %", flush=True)


if __name__ == "__main__":
    main()
