"""Config sweep of the GQA+sink causal attention kernel at the reference headline shape."""
import glob
import itertools
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT] + sorted(d for d in glob.glob(os.path.join(ROOT, "examples", "*")) if os.path.isdir(d))
import torch  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
import example_gqa_sink_fwd_bhsd as m  # noqa: E402

B, H, S, D, G = 1, 64, 4096, 128, 8
q = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)
kk = torch.randn(B, H // G, S, D, device="cuda", dtype=torch.bfloat16)
v = torch.randn_like(kk)
s = torch.randn(H, device="cuda", dtype=torch.bfloat16)
ref = None
cfgs = sys.argv[1:] and [json.loads(a) for a in sys.argv[1:]] or [
    dict(block_M=bm, block_N=bn, threads=t, num_stages=st)
    for bm, bn, t, st in itertools.product([128, 256], [64, 128], [256, 512], [1, 2])]
for c in cfgs:
    try:
        k = m.flashattn_sink(B, H, S, S, D, G, None, None, c["block_M"], c["block_N"], c["num_stages"], c["threads"],
                             causal=c.get("causal", True))
        o = k(q, kk, v, s)
        err = -1.0
        if c.get("causal", True):
            if ref is None:
                ref = m.ref_program(q[:, :8], kk[:, :1], v[:, :1], s[:8]).float()
            err = (o[:, :8].float() - ref).abs().max().item()
        ms = do_bench(lambda: k(q, kk, v, s))
        fl = m.flops(B, H, S, S, D) * (1 if c.get("causal", True) else 2)
        print(json.dumps(dict(cfg=c, ms=round(ms, 4), TFLOPS=round(fl / ms * 1e-9, 1),
                              err=round(err, 4))), flush=True)
    except Exception as e:  # noqa: BLE001
        print(json.dumps(dict(cfg=c, error=f"{type(e).__name__}: {str(e)[:200]}")), flush=True)
