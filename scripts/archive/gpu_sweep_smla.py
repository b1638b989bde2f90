"""Sparse MLA fwd sweep at the reference's benchmark shape (B1 S4096 SKV8192 H128 topk2048)."""
import sys
import time

import torch

sys.path.insert(0, "examples/deepseek_v32")
from sparse_mla_fwd import make_indices, ref_program  # noqa: E402
from tilelang.ops.dsa import sparse_mla_fwd  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

B, S, SKV, H, DQK, DV, topk = 1, 4096, 8192, 128, 576, 512, 2048
q = torch.randn(B, S, H, DQK, device="cuda", dtype=torch.bfloat16)
kv = torch.randn(B, SKV, 1, DQK, device="cuda", dtype=torch.bfloat16)
t0 = time.time()
g = torch.Generator(device="cuda").manual_seed(0)
# per-token random subsets of the visible prefix (vectorised: random keys, top-k of a random permutation)
past = SKV - S
pos = torch.arange(S, device="cuda")[:, None] + past
r = torch.rand(S, SKV, device="cuda", generator=g)
r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
idx = r.topk(topk, dim=-1).indices.int()
idx = torch.where(torch.gather(r, 1, idx.long()) >= 0, idx, torch.full_like(idx, SKV)).view(B, S, 1, topk)
print(f"indices in {time.time() - t0:.1f}s", flush=True)
flops = B * S * (DQK + DV) * topk * 2 * H
configs = eval(sys.argv[1]) if len(sys.argv) > 1 else [dict(), dict(wide=True), dict(wide=True, lazy_rescale=False)]
for cfg in configs:
    try:
        k = sparse_mla_fwd(B, S, SKV, H, DV, DQK - DV, topk, **cfg)
        o, _ = k(q, kv, idx)
        sub = slice(S - 2, S)
        ref = ref_program(q[:, sub].cpu(), kv.cpu(), idx[:, sub].cpu(), DV)
        err = (o[:, sub].float().cpu() - ref.float()).abs().max().item()
        lat = do_bench(lambda: k(q, kv, idx))
        print(f"{cfg}: {lat:.3f} ms {flops / lat * 1e-9:.1f} TFLOPS maxerr {err:.3g}", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{cfg}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
