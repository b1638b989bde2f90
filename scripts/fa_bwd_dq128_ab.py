"""Causal d128 dQ kernel tiles (examples/flash_attention/example_mha_bwd.py), same process,
round-robin, checked against fp32 autograd: the default 128x64 / 8 waves (unroll 2) vs 256x32 / 8
waves (the best of scripts/sweep_fa_bwd.py --causal --d 128 --b 4 --s 2048).

    python scripts/fa_bwd_dq128_ab.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_mha_bwd as E  # noqa: E402

CFGS = {"128x64 u2": dict(block_M=128, block_N=64, threads=512, unroll=2),
        "256x32": dict(block_M=256, block_N=32, threads=512),
        "256x32 u2": dict(block_M=256, block_N=32, threads=512, unroll=2)}


def main():
    torch.manual_seed(0)
    for B, H, S, D in ((4, 32, 2048, 128), (1, 32, 8192, 128), (8, 16, 1024, 128)):
        q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
        qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
        E.ref_program(qr, kr, vr, True).float().backward(do.float())
        o, lse = E.flashattn_fwd(B, H, S, D, True, dtype="float16")(q, k, v)
        delta = E.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
        ks = {n: E.flashattn_bwd_dq(B, H, S, D, True, dtype="float16", **c) for n, c in CFGS.items()}
        res = {n: [1e9, (kk(q, k, v, do, lse, delta).float() - qr.grad).abs().max().item()] for n, kk in ks.items()}
        for _ in range(3):
            for n, kk in ks.items():
                res[n][0] = min(res[n][0], do_bench(lambda: kk(q, k, v, do, lse, delta), warmup=10, rep=50))
        fl = 3 * 2.0 * B * H * S * S * D * 0.5
        print(f"causal dq b{B} h{H} s{S} d{D}: " + "  ".join(
            f"{n} {m * 1e3:.1f} us {fl / m * 1e-9:.0f} TF err {e:.3f}" for n, (m, e) in res.items()), flush=True)


if __name__ == "__main__":
    main()
