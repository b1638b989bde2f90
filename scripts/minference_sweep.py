"""Tile / pipeline-depth sweep of the vertical-slash attention kernel at the reference's shape (B1 H1 D64)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "minference")]

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_vertical_slash_sparse_attn import vertical_slash_sparse_attention, ref_program  # noqa: E402

CFGS = [(64, 64, 256, 2), (64, 128, 256, 2), (128, 64, 512, 2), (128, 128, 512, 2), (128, 32, 512, 3),
        (128, 64, 512, 3), (64, 32, 256, 3), (64, 64, 128, 2), (128, 128, 256, 2)]
for S, nv, ns in ((8192, 1000, 200), (32768, 1000, 600), (65536, 1000, 600)):
    g = torch.Generator(device="cuda").manual_seed(0)
    q, k, v = (torch.randn(1, 1, S, 64, device="cuda", dtype=torch.float16) for _ in range(3))
    v_idx = torch.randperm(S, device="cuda", generator=g)[:nv].view(1, 1, -1)
    s_idx = torch.randperm(S, device="cuda", generator=g)[:ns].view(1, 1, -1)
    s_idx[..., 0] = 0
    for bm, bn, th, st in CFGS:
        try:
            o = vertical_slash_sparse_attention(q, k, v, v_idx, s_idx, bm, bn, th, st)
            if S <= 8192:
                sub = slice(S - 128, S)
                r = ref_program(q, k, v, v_idx, s_idx, bm, bn)
                err = (o[:, :, sub].float() - r[:, :, sub]).abs().max().item()
            else:
                err = float("nan")
            t = do_bench(lambda: vertical_slash_sparse_attention(q, k, v, v_idx, s_idx, bm, bn, th, st))
            print(f"S{S} [{nv},{ns}] bm{bm} bn{bn} t{th} st{st}: {t:.3f} ms (err {err:.2g})", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"S{S} bm{bm} bn{bn} t{th} st{st}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
