"""A/B of sparse MLA fwd's MFMA row sums (tilelang/ops/dsa.py sparse_mla_fwd(sum_mfma=)) at the
reference benchmark shape (B1 S4096 SKV8192 H128 topk2048), one process, round-robin.

    python scripts/smla_sum_ab.py
"""
import torch

from tilelang.ops.dsa import sparse_mla_fwd

B, S, SKV, H, topk = 1, 4096, 8192, 128, 2048
torch.manual_seed(0)
q = torch.randn(B, S, H, 576, device="cuda", dtype=torch.bfloat16)
kv = torch.randn(B, SKV, 1, 576, device="cuda", dtype=torch.bfloat16)
r = torch.rand(S, SKV, device="cuda")
pos = torch.arange(S, device="cuda")[:, None] + SKV - S
r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
idx = r.topk(topk, dim=-1).indices.int().view(B, S, 1, topk)
ks = {sm: sparse_mla_fwd(B, S, SKV, H, 512, 64, topk, sum_mfma=sm) for sm in (False, True)}
outs = {sm: ks[sm](q, kv, idx) for sm in ks}
o0, l0 = outs[False]
o1, l1 = outs[True]
print(f"max |dO| {(o0.float() - o1.float()).abs().max().item():.3g}, max |dLSE| {(l0 - l1).abs().max().item():.3g}",
      flush=True)
fl = 2.0 * B * S * H * topk * (576 + 512)
res = {sm: [] for sm in ks}
for _ in range(3):
    for sm in ks:
        ks[sm](q, kv, idx)
torch.cuda.synchronize()
for _ in range(5):
    for sm, k in ks.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            k(q, kv, idx)
        e1.record()
        torch.cuda.synchronize()
        res[sm].append(e0.elapsed_time(e1) / 5)
for sm in ks:
    ms = sorted(res[sm])[2]
    print(f"sum_mfma={sm}: {ms:.4f} ms, {fl / ms * 1e-9:.1f} TF", flush=True)
