"""A/B of the FlashAttention forward (examples/flash_attention/example_mha_fwd_pipelined.py) with
16x16x32 vs 32x32x16 MFMA tiles, plus tile / stage variants of the 32x32 form; one process, one box.

    python scripts/fa_mfma_ab.py [--seq 4096] [--causal]
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_mha_fwd import ref_program  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined as fa  # noqa: E402

VARIANTS = {
    "m16_n64_s2": dict(block_N=64, num_stages=2, mfma="16x16"),
    "m32_n64_s2": dict(block_N=64, num_stages=2, mfma="32x32"),
    "m32_n64_s3": dict(block_N=64, num_stages=3, mfma="32x32"),
    "m32_n128_s2": dict(block_N=128, num_stages=2, mfma="32x32"),
    "m16_sum": dict(block_N=64, num_stages=2, mfma="16x16", sum_mfma=True),
    "m32_sum": dict(block_N=64, num_stages=2, mfma="32x32", sum_mfma=True),
    "m16_sum_s3": dict(block_N=64, num_stages=3, mfma="16x16", sum_mfma=True),
    "m16_sum_n128": dict(block_N=128, num_stages=2, mfma="16x16", sum_mfma=True),
    "m16_sum_n32": dict(block_N=32, num_stages=3, mfma="16x16", sum_mfma=True),
}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seq", type=int, default=4096)
    p.add_argument("--heads", type=int, default=64)
    p.add_argument("--causal", action="store_true")
    p.add_argument("--variants", nargs="*", default=list(VARIANTS))
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    torch.manual_seed(0)
    b, h, s, d = 1, a.heads, a.seq, 128
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    ref = ref_program(q, k, v, a.causal).float()
    flops = 4.0 * b * h * s * s * d * (0.5 if a.causal else 1.0)
    kern = {}
    for name in a.variants:
        cfg = VARIANTS[name]
        kk = fa(b, h, s, d, a.causal, 1, 256, cfg["block_N"], 512, cfg["num_stages"], "bfloat16", True, True,
                mfma=cfg["mfma"], sum_mfma=cfg.get("sum_mfma", False))
        err = (kk(q, k, v).float() - ref).abs().max().item()
        print(f"{name}: max err {err:.4f}{'  WRONG' if err > 0.05 else ''}", flush=True)
        if err <= 0.05:
            kern[name] = kk
    best = {n: 0.0 for n in kern}
    for _ in range(a.rounds):
        for n, kk in kern.items():
            ms = do_bench(lambda: kk(q, k, v), warmup=25, rep=100)
            best[n] = max(best[n], flops / ms * 1e-9)
    print(f"FA fwd b{b} h{h} s{s} d{d} causal={a.causal}: " +
          ", ".join(f"{n} {t:.0f}" for n, t in best.items()) + " TF (cold, best of rounds)", flush=True)


if __name__ == "__main__":
    main()
