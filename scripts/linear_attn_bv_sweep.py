"""Value-tile sweep of the chunked linear attention forward (examples/linear_attention): a smaller BV
means more workgroups (DV / BV x B*H) for the sequential chunk walk."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "linear_attention")]

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_linear_attn_fwd import linear_attn_fwd, ref_program  # noqa: E402

for B, S, H, D in ((1, 4096, 16, 128), (1, 8192, 32, 128), (8, 4096, 32, 128)):
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) * 0.1
    k = torch.randn_like(q) * 0.1
    v = torch.randn_like(q)
    ro, rh = ref_program(q, k, v)
    for bv, th in ((64, 256), (32, 256), (32, 128), (16, 128), (16, 64)):
        try:
            kern = linear_attn_fwd(B, S, H, D, D, BV=bv, threads=th)
            o, h = kern(q, k, v)
            err = (o.float() - ro).abs().max().item()
            t = do_bench(lambda: kern(q, k, v))
            print(f"B{B} S{S} H{H} D{D} BV{bv} t{th}: {t:.4f} ms (max err {err:.3g})", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"B{B} S{S} H{H} BV{bv} t{th}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
