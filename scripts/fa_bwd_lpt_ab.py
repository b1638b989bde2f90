"""Causal FA training kernels (examples/flash_attention/example_mha_bwd.py): grid order A/B.

``lpt=False``: the tile axis is the middle grid axis (heaviest tiles first within one batch only);
``lpt=True``: the tile axis is the slowest axis, so the longest walks of EVERY (batch, head) are
dispatched before any shorter one.  Each config is checked against fp32 autograd gradients and
timed in the same process, round-robin over the variants.

    python scripts/fa_bwd_lpt_ab.py [--s 1024] [--d 64]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_mha_bwd as E  # noqa: E402

DKV = [(64, 32, 256, 2), (64, 64, 256, 2), (128, 32, 256, 2), (128, 64, 256, 2), (128, 64, 512, 2),
       (256, 64, 512, 4), (128, 32, 512, 2)]
DQ = [(64, 64, 256, 2), (64, 32, 256, 2), (128, 64, 256, 2), (128, 64, 512, 4), (128, 32, 512, 2),
      (64, 64, 256, None)]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--b", type=int, default=8)
    p.add_argument("--h", type=int, default=32)
    p.add_argument("--s", type=int, default=1024)
    p.add_argument("--d", type=int, default=64)
    a = p.parse_args()
    B, H, S, D = a.b, a.h, a.s, a.d
    torch.manual_seed(0)
    q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref = E.ref_program(qr, kr, vr, True).float()
    ref.backward(do.float())
    gq, gk, gv = qr.grad, kr.grad, vr.grad
    unit = 2.0 * B * H * S * S * D * 0.5  # one causal S x S x D GEMM
    print(f"causal b{B} h{H} s{S} d{D} fp16", flush=True)
    # forward (writes the LSE the backward kernels read)
    fw = {lpt: E.flashattn_fwd(B, H, S, D, True, dtype="float16", lpt=lpt) for lpt in (False, True)}
    for lpt, kern in fw.items():
        o, lse = kern(q, k, v)
        err = (o.float() - ref).abs().max().item()
        ms = [do_bench(lambda: kern(q, k, v), warmup=10, rep=50) for _ in range(2)]
        print(f"fwd lpt={int(lpt)}: {min(ms) * 1e3:.1f} us {2 * unit / min(ms) * 1e-9:.0f} TF err {err:.4f}",
              flush=True)
    o, lse = fw[False](q, k, v)
    delta = E.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
    dk, dv = torch.empty_like(k), torch.empty_like(v)
    for bm, bn, th, un in DKV:
        ks = {lpt: E.flashattn_bwd(B, H, S, D, True, bm, bn, th, 2, "float16", dq_mode="none", unroll=un, lpt=lpt)
              for lpt in (False, True)}
        res = {}
        for _ in range(2):
            for lpt, kern in ks.items():
                kern(q, k, v, do, lse, delta, dk, dv)
                err = max((dk.float() - gk).abs().max().item(), (dv.float() - gv).abs().max().item())
                ms = do_bench(lambda: kern(q, k, v, do, lse, delta, dk, dv), warmup=10, rep=50)
                res[lpt] = (min(ms, res.get(lpt, (1e9, ))[0]), err)
        print("dkv bm%d bn%d t%d u%s: " % (bm, bn, th, un) + "  ".join(
            f"lpt={int(l)} {m * 1e3:.1f} us {4 * unit / m * 1e-9:.0f} TF err {e:.3f}" for l, (m, e) in res.items()),
            flush=True)
    for bm, bn, th, un in DQ:
        ks = {lpt: E.flashattn_bwd_dq(B, H, S, D, True, bm, bn, th, 2, "float16", unroll=un, lpt=lpt)
              for lpt in (False, True)}
        res = {}
        for _ in range(2):
            for lpt, kern in ks.items():
                dq = kern(q, k, v, do, lse, delta)
                err = (dq.float() - gq).abs().max().item()
                ms = do_bench(lambda: kern(q, k, v, do, lse, delta), warmup=10, rep=50)
                res[lpt] = (min(ms, res.get(lpt, (1e9, ))[0]), err)
        print("dq bm%d bn%d t%d u%s: " % (bm, bn, th, un) + "  ".join(
            f"lpt={int(l)} {m * 1e3:.1f} us {3 * unit / m * 1e-9:.0f} TF err {e:.3f}" for l, (m, e) in res.items()),
            flush=True)


if __name__ == "__main__":
    main()
