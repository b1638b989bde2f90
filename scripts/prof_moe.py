"""Time the bench.py MoE layer (local, 1 GPU); optional sweep of the expert GEMM tile.

    python scripts/prof_moe.py [reps] [--sweep]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402

import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 10
m = bench.MOE_CFG
fl = 6.0 * m["tokens"] * m["topk"] * m["hidden"] * m["ffn"]


def run(layer, x, tag):
    for _ in range(3):
        layer(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        layer(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"{tag}: moe layer {ms * 1e3:.1f} us = {fl / ms * 1e-9:.1f} TF", flush=True)


layer, x = bench.build_moe(None, "cuda")
from tilelang.models.moe import moe_reference, init_moe_weights  # noqa: E402

run(layer, x, "default " + str(layer.cfg.gemm_cfg))
if "--check" in sys.argv:
    out = layer(x).float()
    g, w1, w2 = (t.to("cuda") for t in init_moe_weights(layer.cfg))
    ref = moe_reference(x, g, w1, w2, layer.cfg.topk)
    print("max abs err", (out - ref).abs().max().item(), "ref max", ref.abs().max().item(), flush=True)
if "--skip-ab" in sys.argv:  # T.gemm(valid_m=) on the padded tail tiles vs full-tile MFMAs
    base = dict(layer.cfg.gemm_cfg or {})
    for skip in (False, True, False, True):
        layer.cfg.gemm_cfg = dict(base, skip_padding=skip)
        run(layer, x, f"skip_padding={skip}")
    layer.cfg.gemm_cfg = base
    out = layer(x).float()
    g, w1, w2 = (t.to("cuda") for t in init_moe_weights(layer.cfg))
    ref = moe_reference(x, g, w1, w2, layer.cfg.topk)
    print("max abs err", (out - ref).abs().max().item(), "ref max", ref.abs().max().item(), flush=True)
if "--sk-ab" in sys.argv:  # stream-K hybrid expert GEMMs vs the plain tile grid
    base = dict(layer.cfg.gemm_cfg or {})
    for sk in (False, True, False, True):
        layer.cfg.gemm_cfg = dict(base, stream_k=sk)
        run(layer, x, f"stream_k={sk}")
    layer.cfg.gemm_cfg = base
    out = layer(x).float()
    g, w1, w2 = (t.to("cuda") for t in init_moe_weights(layer.cfg))
    ref = moe_reference(x, g, w1, w2, layer.cfg.topk)
    print("max abs err", (out - ref).abs().max().item(), "ref max", ref.abs().max().item(), flush=True)
if "--tail-sweep" in sys.argv:  # narrow-tail width of the tail-balanced expert GEMMs
    base = dict(layer.cfg.gemm_cfg or {})
    for ts, ph in ((4, False), (2, False), (4, False), (2, False)):
        layer.cfg.gemm_cfg = dict(base, stream_k=True, tail_split=ts, phased=ph)
        run(layer, x, f"tail_split={ts} phased={ph}")
    layer.cfg.gemm_cfg = base
if "--prefetch-ab" in sys.argv:  # phased K-half (+register prefetch when nothing is skipped) vs whole-K loop
    base = dict(layer.cfg.gemm_cfg or {})
    for ph, sk in ((False, True), (True, False), (True, True), (False, False), (False, True), (True, False)):
        layer.cfg.gemm_cfg = dict(base, phased=ph, skip_padding=sk)
        run(layer, x, f"phased={ph} skip_padding={sk}")
    layer.cfg.gemm_cfg = dict(base, phased=True, skip_padding=False)
    out = layer(x).float()
    g, w1, w2 = (t.to("cuda") for t in init_moe_weights(layer.cfg))
    ref = moe_reference(x, g, w1, w2, layer.cfg.topk)
    print("phased/prefetch max abs err", (out - ref).abs().max().item(), "ref max", ref.abs().max().item(), flush=True)
    layer.cfg.gemm_cfg = base
if "--sweep" in sys.argv:
    for bm in (128, 256):
        for cfg in (dict(block_N=128, block_K=64, num_stages=2, threads=256),
                    dict(block_N=256, block_K=64, num_stages=2, threads=512),
                    dict(block_N=256, block_K=64, num_stages=3, threads=512),
                    dict(block_N=128, block_K=64, num_stages=3, threads=256),
                    dict(block_N=256, block_K=32, num_stages=4, threads=512)):
            try:
                layer.cfg.block_M = bm
                layer.cfg.gemm_cfg = cfg
                run(layer, x, f"bm{bm} {cfg}")
            except Exception as e:  # noqa: BLE001
                print(f"bm{bm} {cfg}: failed {type(e).__name__}: {str(e)[:200]}", flush=True)
