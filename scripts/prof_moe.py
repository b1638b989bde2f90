"""Run the bench.py MoE layer (local, 1 GPU) N times for rocprofv3 --kernel-trace --stats."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import torch  # noqa: E402

import bench  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
layer, x = bench.build_moe(None, "cuda")
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
m = bench.MOE_CFG
fl = 6.0 * m["tokens"] * m["topk"] * m["hidden"] * m["ffn"]
print(f"moe layer {ms * 1e3:.1f} us = {fl / ms * 1e-9:.1f} TF", flush=True)
