"""MoE router: the fused one-wave-per-16-tokens kernel vs router_wide_kernel (K chunks side by side
in one tile GEMM) on the bench layer's shape; ids must agree except on bf16 logit ties, weights
to fp32 rounding.

    python scripts/router_wide_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tilelang.ops import moe as K  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

T_, H, E, TOP = 2048, 4096, 8, 2
torch.manual_seed(0)
x = torch.randn(T_, H, device="cuda", dtype=torch.bfloat16)
g = (torch.randn(E, H, device="cuda") * 0.02).to(torch.bfloat16)
gp = K._padded_gate(g)
ids0 = torch.empty(T_, TOP, dtype=torch.int32, device="cuda")
w0 = torch.empty(T_, TOP, dtype=torch.float32, device="cuda")
kf = K.router_fused_kernel(T_, H, E, TOP, "bfloat16", "hip")
kf(x, gp, ids0, w0)
t = do_bench(lambda: kf(x, gp, ids0, w0), warmup=20, rep=200)
print(f"fused: {t * 1e3:.2f} us", flush=True)
for bt, kc, bk, st in ((8, 8, 64, 2), (8, 8, 64, 4), (8, 8, 64, 6), (8, 8, 128, 3), (8, 4, 128, 4), (8, 4, 64, 6),
                       (16, 4, 64, 4), (8, 16, 32, 4)):
    ids = torch.empty_like(ids0)
    w = torch.empty_like(w0)
    try:
        k = K.router_wide_kernel(T_, H, E, TOP, "bfloat16", "hip", block_T=bt, kc=kc, block_K=bk, num_stages=st)
    except Exception as ex:  # noqa: BLE001
        print(bt, kc, bk, st, "failed", str(ex)[:200], flush=True)
        continue
    xv, gv = x.view(T_ * kc, H // kc), gp.view(gp.shape[0] * kc, H // kc)
    k(xv, gv, ids, w)
    torch.cuda.synchronize()
    mism = (ids != ids0).any(1).sum().item()
    werr = (w - w0).abs().max().item()
    t = do_bench(lambda: k(xv, gv, ids, w), warmup=20, rep=200)
    print(f"wide block_T={bt} kc={kc} block_K={bk} stages={st}: {t * 1e3:.2f} us, id rows differing {mism} / {T_}, max |dw| {werr:.2e}",
          flush=True)
