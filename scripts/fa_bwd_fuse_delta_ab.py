"""FA backward through autograd (examples/flash_attention/example_mha_bwd.py): Delta from the
preprocess kernel (BWD_FUSE_DELTA=False) vs computed inside the dQ kernel, which then runs before
dK/dV (True).  Same process, round-robin; gradients checked against each other.

    python scripts/fa_bwd_fuse_delta_ab.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_mha_bwd as E  # noqa: E402


def main():
    torch.manual_seed(0)
    for B, H, S, D, causal in ((8, 32, 1024, 64, False), (8, 32, 1024, 64, True), (4, 32, 2048, 128, False),
                               (4, 32, 2048, 128, True)):
        q, k, v = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16).requires_grad_() for _ in range(3))
        do = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16)
        o = E.attention(q, k, v, causal)
        fl = 5 * 2.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        grads, best = {}, {}
        for mode in (False, True):
            E.BWD_FUSE_DELTA = mode
            grads[mode] = torch.autograd.grad(o, (q, k, v), do, retain_graph=True)
        err = max((a.float() - b.float()).abs().max().item() for a, b in zip(grads[False], grads[True]))
        for _ in range(3):
            for mode in (False, True):
                E.BWD_FUSE_DELTA = mode
                ms = do_bench(lambda: torch.autograd.grad(o, (q, k, v), do, retain_graph=True), warmup=10, rep=50)
                best[mode] = min(ms, best.get(mode, 1e9))
        print(f"b{B} h{H} s{S} d{D} causal={int(causal)}: preprocess {best[False] * 1e3:.1f} us "
              f"{fl / best[False] * 1e-9:.1f} TF  fused {best[True] * 1e3:.1f} us {fl / best[True] * 1e-9:.1f} TF  "
              f"max |grad diff| {err:.4f}", flush=True)
    E.BWD_FUSE_DELTA = True


if __name__ == "__main__":
    main()
