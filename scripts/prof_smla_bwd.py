"""Sparse MLA bwd kernels at the reference shape, a few iterations (for rocprofv3 --stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "examples", "deepseek_v32"))
from sparse_mla_bwd import sparse_mla_bwd  # noqa: E402
from tilelang.ops.dsa import sparse_mla_fwd  # noqa: E402

B, S, SKV, H, topk = 1, 4096, 8192, 64, 2048
q = (torch.randn(B, S, H, 576, device="cuda") / 10).to(torch.bfloat16)
kv = (torch.randn(B, SKV, 1, 576, device="cuda") / 10).to(torch.bfloat16)
do = torch.randn(B, S, H, 512, device="cuda", dtype=torch.bfloat16)
r = torch.rand(S, SKV, device="cuda")
pos = torch.arange(S, device="cuda")[:, None] + SKV - S
r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
idx = r.topk(topk, dim=-1).indices.int().view(B, S, 1, topk)
o, lse = sparse_mla_fwd(B, S, SKV, H, 512, 64, topk)(q, kv, idx)
for _ in range(3):
    sparse_mla_bwd(q, kv, o, do, idx, lse)
torch.cuda.synchronize()
print("done")
