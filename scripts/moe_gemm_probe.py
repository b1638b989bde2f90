"""Expert GEMMs of the bench MoE layer in isolation: balanced routing (every expert exactly
tokens*topk/E rows: whole tiles only, no tail) vs random routing, against the plain GEMM with the
same FLOPs.  Separates "the expert GEMM kernel is slow" from "the routing tail is slow".

    python scripts/moe_gemm_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm")]
import torch  # noqa: E402

from tilelang.ops import moe as K  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

T_, H, F, E, TOP = 2048, 4096, 2048, 8, 2
BM = 256
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(T_, H, device=dev, dtype=torch.bfloat16)
w1 = (torch.randn(E, 2 * F, H, device=dev) * 0.02).to(torch.bfloat16)
w2 = (torch.randn(E, H, F, device=dev) * 0.02).to(torch.bfloat16)
n = T_ * TOP


def run(ids, tag, BM=256, **kw):
    ext = kw.get("ext_M", 0)
    max_rows = K.max_padded_rows(K._bucket(n), E, BM + ext)
    dest, row_src, te, counts, trows = K.dispatch_plan(ids, E, BM + ext, max_rows, TOP, even=ext > 0)
    act = torch.empty(max_rows, F, dtype=x.dtype, device=dev)
    y = torch.empty(max_rows, H, dtype=x.dtype, device=dev)
    k1 = K.expert_gemm_sk_kernel(max_rows, H, 2 * F, E, "bfloat16", "hip", BM, n_src=T_, swiglu=True, **kw)
    k2 = K.expert_gemm_sk_kernel(max_rows, F, H, E, "bfloat16", "hip", BM, **kw)
    ws = K._tail_workspace(dev, 256, kw["tail_ksplit"], BM, 256) if kw.get("tail_ksplit") else ()
    t1 = do_bench(lambda: k1(x, w1, te, row_src, trows, act, *ws), warmup=10, rep=50)
    t2 = do_bench(lambda: k2(act, w2, te, row_src, trows, y, *ws), warmup=10, rep=50)
    f1, f2 = 2.0 * n * H * 2 * F, 2.0 * n * F * H
    nt = int((te >= 0).sum())
    print(f"{tag} BM{BM} {kw}: tiles {nt}  GEMM1 {t1 * 1e3:.1f} us {f1 / t1 * 1e-9:.0f} TF  GEMM2 {t2 * 1e3:.1f} us "
          f"{f2 / t2 * 1e-9:.0f} TF", flush=True)


bal = torch.arange(n, device=dev, dtype=torch.int32) % E  # exactly n/E rows per expert
rnd = torch.randint(0, E, (n, ), device=dev, dtype=torch.int32)
VARIANTS = eval(sys.argv[1]) if len(sys.argv) > 1 else ({}, dict(BM=128), dict(BM=128, threads=256), {})
for kw in VARIANTS:
    try:
        run(bal, "balanced", **kw)
        run(rnd, "random  ", **kw)
    except Exception as e:  # noqa: BLE001
        print(kw, "failed", str(e)[:200], flush=True)
# the whole bench layer (router, dispatch, both GEMMs, combine) per gemm_cfg
from tilelang.models.moe import MoEConfig, MoELayer  # noqa: E402
LAYERS = eval(sys.argv[2]) if len(sys.argv) > 2 else ((0, True), (32, True), (0, True), (32, True))
for ext, quad in LAYERS:
    cfg = MoEConfig(hidden=H, ffn=F, n_experts=E, topk=TOP, dtype=torch.bfloat16, block_M=BM,
                    gemm_cfg=dict(block_N=256, block_K=64, num_stages=2, threads=512, ext_M=ext, quad=quad))
    layer = MoELayer(cfg, "local", device=dev)
    xs = torch.randn(T_, H, device=dev, dtype=torch.bfloat16)
    t = do_bench(lambda: layer(xs), warmup=10, rep=50)
    print(f"MoE layer ext_M={ext} quad={quad}: {t * 1e3:.1f} us {6.0 * n * H * F / t * 1e-9:.0f} TF", flush=True)
from example_gemm import matmul  # noqa: E402
g = matmul(4096, 4096, 4096, 256, 256, 64, 512, 2, staged_epilogue=True)
a, b = torch.randn(4096, 4096, device=dev).half(), torch.randn(4096, 4096, device=dev).half()
t = do_bench(lambda: g(a, b), warmup=10, rep=50)
print(f"plain GEMM 4096^3 (= GEMM1 FLOPs): {t * 1e3:.1f} us {2 * 4096**3 / t * 1e-9:.0f} TF")
