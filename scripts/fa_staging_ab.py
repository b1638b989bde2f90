"""FA forward (bench kernel): K/V tiles by LDS-DMA (glds, default) vs register staging with the
split issue-early / write-late copy (tl.disable_glds), 2 and 3 stages.  One process, cold.
    python scripts/fa_staging_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "flash_attention")]
import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_mha_fwd import ref_program  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined as fa  # noqa: E402

b, h, s, d = 1, 64, 4096, 128
torch.manual_seed(0)
q, k, v = (torch.randn(b, s, h, d, device="cuda", dtype=torch.bfloat16) for _ in range(3))
ref = ref_program(q, k, v, False).float()
flops = 4.0 * b * h * s * s * d
res = {}
for name, st, glds_off in (("glds_s2", 2, False), ("staged_s2", 2, True), ("staged_s3", 3, True)):
    f = fa.get_tir(b, h, s, d, False, 1, 256, 64, 512, st, "bfloat16", True, True, sum_mfma=True)
    cfg = dict(fa.pass_configs)
    if glds_off:
        cfg["tl.disable_glds"] = True
    try:
        kern = tilelang.compile(f, out_idx=[3], target="hip", pass_configs=cfg)
    except Exception as e:  # noqa: BLE001
        print(name, "failed", str(e)[:200], flush=True)
        continue
    err = (kern(q, k, v).float() - ref).abs().max().item()
    best = 0.0
    for _ in range(3):
        best = max(best, flops / do_bench(lambda: kern(q, k, v), warmup=25, rep=100) * 1e-9)
    res[name] = best
    print(f"{name}: {best:.0f} TF (err {err:.4f})", flush=True)
