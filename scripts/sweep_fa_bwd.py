"""Tile sweep of the FA backward kernels (examples/flash_attention/example_mha_bwd.py): the dK/dV
kernel (dq_mode="none") and the atomic-free dQ kernel, fp16 b8 h32 s1024 d64 (the verdict's shape),
each config checked against fp32 autograd gradients, timed cold.

    python scripts/sweep_fa_bwd.py [--causal]
"""
import argparse
import itertools
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_mha_bwd as E  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--causal", action="store_true")
    p.add_argument("--b", type=int, default=8)
    p.add_argument("--h", type=int, default=32)
    p.add_argument("--s", type=int, default=1024)
    p.add_argument("--d", type=int, default=64)
    a = p.parse_args()
    B, H, S, D, causal = a.b, a.h, a.s, a.d, a.causal
    torch.manual_seed(0)
    q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
    o, lse = E.flashattn_fwd(B, H, S, D, causal, dtype="float16")(q, k, v)
    delta = E.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    E.ref_program(qr, kr, vr, causal).float().backward(do.float())
    gq, gk, gv = qr.grad, kr.grad, vr.grad
    unit = 2.0 * B * H * S * S * D * (0.5 if causal else 1.0)  # one S x S x D GEMM
    res = []
    for bm, bn, th in itertools.product((64, 128, 256), (32, 64, 128), (256, 512)):
        if bm // (th // 64) < 16:
            continue
        try:
            kern = E.flashattn_bwd(B, H, S, D, causal, bm, bn, th, 2, "float16", dq_mode="none")
        except Exception as e:  # noqa: BLE001
            print(f"dkv bm{bm} bn{bn} t{th}: compile failed: {str(e)[:80]}", flush=True)
            continue
        dk, dv = torch.empty_like(k), torch.empty_like(v)
        kern(q, k, v, do, lse, delta, dk, dv)
        err = max((dk.float() - gk).abs().max().item(), (dv.float() - gv).abs().max().item())
        ms = do_bench(lambda: kern(q, k, v, do, lse, delta, dk, dv), warmup=10, rep=50)
        tf = 4 * unit / ms * 1e-9
        res.append(("dkv", bm, bn, th, ms, tf, err))
        print(f"dkv bm{bm} bn{bn} t{th}: {ms * 1e3:.1f} us {tf:.0f} TF err {err:.3f}", flush=True)
    for bm, bn, th in itertools.product((64, 128, 256), (32, 64, 128), (256, 512)):
        if bm // (th // 64) < 16:
            continue
        try:
            kern = E.flashattn_bwd_dq(B, H, S, D, causal, bm, bn, th, 2, "float16")
        except Exception as e:  # noqa: BLE001
            print(f"dq bm{bm} bn{bn} t{th}: compile failed: {str(e)[:80]}", flush=True)
            continue
        dq = kern(q, k, v, do, lse, delta)
        err = (dq.float() - gq).abs().max().item()
        ms = do_bench(lambda: kern(q, k, v, do, lse, delta), warmup=10, rep=50)
        tf = 3 * unit / ms * 1e-9
        res.append(("dq", bm, bn, th, ms, tf, err))
        print(f"dq bm{bm} bn{bn} t{th}: {ms * 1e3:.1f} us {tf:.0f} TF err {err:.3f}", flush=True)
    for kind in ("dkv", "dq"):
        ok = [r for r in res if r[0] == kind and r[6] < 0.05]
        if ok:
            best = min(ok, key=lambda r: r[4])
            print(f"best {kind}: bm{best[1]} bn{best[2]} t{best[3]} {best[4] * 1e3:.1f} us {best[5]:.0f} TF")


if __name__ == "__main__":
    main()
