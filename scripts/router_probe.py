"""The bench MoE layer's router (x [2048, 4096] bf16, 8 experts, top-2): the fused one-pass kernel
vs the K-split logits kernel + summing top-k kernel (ops/moe.py ROUTER_SPLITS), same process.

    python scripts/router_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tilelang.ops import moe as K  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

torch.manual_seed(0)
x = torch.randn(2048, 4096, device="cuda", dtype=torch.bfloat16)
g = (torch.randn(8, 4096, device="cuda") * 0.05).to(torch.bfloat16)
ref = None
for sp in (0, 2, 4, 8, 0, 4):
    K.ROUTER_SPLITS = sp
    ids, w = K.route(x, g, 2)
    if ref is None:
        ref = (ids.clone(), w.clone())
    same = bool(torch.equal(ids, ref[0])) and bool(torch.allclose(w, ref[1]))
    t = do_bench(lambda: K.route(x, g, 2), warmup=10, rep=100)
    print(f"router splits={sp}: {t * 1e3:.2f} us (incl. host launch), same={same}", flush=True)
# whole bench layer (GPU runs ahead of the host as in the bench step)
from tilelang.models.moe import MoEConfig, MoELayer  # noqa: E402
cfg = MoEConfig(hidden=4096, ffn=2048, n_experts=8, topk=2, dtype=torch.bfloat16, block_M=256,
                gemm_cfg=dict(block_N=256, block_K=64, num_stages=2, threads=512, ext_M=32))
layer = MoELayer(cfg, "local", device="cuda")
for sp in (0, 4, 0, 4):
    K.ROUTER_SPLITS = sp
    t = do_bench(lambda: layer(x), warmup=10, rep=50)
    print(f"MoE layer router splits={sp}: {t * 1e3:.1f} us", flush=True)
