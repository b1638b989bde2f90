"""Run the Mamba-2 chunk scan kernel for rocprofv3 (--kernel-trace --stats / --pmc).

    python scripts/prof_mamba.py [seq_len] [reps] [json config]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "linear_attention")]
import torch  # noqa: E402

from example_mamba_chunk_scan import chunk_scan_fwd, make_inputs  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
cfg = json.loads(sys.argv[3]) if len(sys.argv) > 3 else dict(block_M=128, block_N=64, block_K=32, threads=256)
args = make_inputs(8, L, 256, 1, 80, 64, 128)
k = chunk_scan_fwd(8, L, 256, 1, 80, 64, 128, **cfg)
for _ in range(reps):
    k(*args)
torch.cuda.synchronize()
print("done")
