"""Run the sparse MLA fwd kernel a few times (for rocprofv3 counter passes)."""
import torch

from tilelang.ops.dsa import sparse_mla_fwd

B, S, SKV, H, topk = 1, 4096, 8192, 128, 2048
q = torch.randn(B, S, H, 576, device="cuda", dtype=torch.bfloat16)
kv = torch.randn(B, SKV, 1, 576, device="cuda", dtype=torch.bfloat16)
r = torch.rand(S, SKV, device="cuda")
pos = torch.arange(S, device="cuda")[:, None] + SKV - S
r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
idx = r.topk(topk, dim=-1).indices.int().view(B, S, 1, topk)
k = sparse_mla_fwd(B, S, SKV, H, 512, 64, topk)
for _ in range(3):
    k(q, kv, idx)
torch.cuda.synchronize()
print("done")
