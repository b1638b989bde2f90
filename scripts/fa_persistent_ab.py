"""Persistent FA (examples/amd/example_amd_flash_attn_fwd.py) vs the one-tile-per-workgroup staged
kernel (examples/flash_attention/example_mha_fwd_pipelined.py), 16x16 and 32x32 MFMA, causal and
not; fp16 b1 h64 s4096 d128 (the round-2 persistent measurement's shape).  One process, cold cache.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "amd"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_amd_flash_attn_fwd import fast_flashattn, ref_program  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined  # noqa: E402


def main():
    torch.manual_seed(0)
    b, h, s, d = 1, 64, 4096, 128
    q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.float16) for _ in range(3))
    for causal in (False, True):
        ref = ref_program(q, k, v, causal).float()
        flops = 4.0 * b * h * s * s * d * (0.5 if causal else 1.0)
        kerns = {}
        for mfma in ("16x16", "32x32"):
            kerns[f"persistent_{mfma}"] = fast_flashattn(b, h, s, d, causal, 1, mfma=mfma)
            kerns[f"staged_{mfma}"] = flashattn_pipelined(b, h, s, d, causal, 1, 256, 64, 512, 2, "float16",
                                                          mfma=mfma)
        best = {}
        for name, kern in kerns.items():
            err = (kern(q, k, v).float() - ref).abs().max().item()
            print(f"causal={causal} {name}: max err {err:.4f}{'  WRONG' if err > 0.05 else ''}", flush=True)
            if err <= 0.05:
                best[name] = 0.0
        for _ in range(3):
            for name in best:
                ms = do_bench(lambda: kerns[name](q, k, v), warmup=25, rep=100)
                best[name] = max(best[name], flops / ms * 1e-9)
        print(f"FA fwd fp16 b{b} h{h} s{s} d{d} causal={causal}: " +
              ", ".join(f"{n} {t:.0f}" for n, t in best.items()) + " TF (cold, best of 3)", flush=True)


if __name__ == "__main__":
    main()
