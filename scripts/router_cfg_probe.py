"""Fused MoE router kernel (x [2048, 4096] bf16, 8 experts, top-2) across (block_K, num_stages):
bytes in flight per wave vs the counted-vmcnt limit; same process, results checked against the
default config.

    python scripts/router_cfg_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tilelang.ops import moe as K  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

torch.manual_seed(0)
T_, H, E, TOP = 2048, 4096, 8, 2
x = torch.randn(T_, H, device="cuda", dtype=torch.bfloat16)
g = K._padded_gate((torch.randn(E, H, device="cuda") * 0.05).to(torch.bfloat16))
ref = None
for bk, st in ((256, 3), (128, 3), (128, 5), (128, 7), (64, 8), (256, 2), (256, 3)):
    ids = torch.empty(T_, TOP, dtype=torch.int32, device="cuda")
    w = torch.empty(T_, TOP, dtype=torch.float32, device="cuda")
    try:
        k = K.router_fused_kernel(T_, H, E, TOP, "bfloat16", "hip", block_K=bk, num_stages=st)
        k(x, g, ids, w)
        if ref is None:
            ref = (ids.clone(), w.clone())
        same = bool(torch.equal(ids, ref[0])) and bool(torch.allclose(w, ref[1]))
        t = do_bench(lambda: k(x, g, ids, w), warmup=10, rep=100)
        print(f"block_K={bk} stages={st}: {t * 1e3:.2f} us same={same}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"block_K={bk} stages={st}: FAILED {type(e).__name__}: {str(e)[:160]}", flush=True)
