"""MoE combine kernel (out[t] = sum_k w[t,k] Y[dest[t*k]]) at the bench layer's shape across tile
configs: checked against torch, timed cold; prints us and effective TB/s (Y rows read + out written).

    python scripts/moe_combine_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tilelang.ops import moe as K  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

T_, H, TOP, ROWS = 2048, 4096, 2, 4608
torch.manual_seed(0)
y = torch.randn(ROWS, H, device="cuda", dtype=torch.bfloat16)
dest = torch.randperm(ROWS, device="cuda")[:T_ * TOP].to(torch.int32)
w = torch.rand(T_, TOP, device="cuda")
ref = (y[dest.long()].float().view(T_, TOP, H) * w.unsqueeze(-1)).sum(1)
nbytes = (T_ * TOP * H + T_ * H) * 2
for bh, th in ((1024, 128), (1024, 256), (2048, 256), (4096, 256), (4096, 512), (1024, 128)):
    k = K.combine_kernel(T_, H, TOP, ROWS, "bfloat16", "hip", block_H=bh, threads=th)
    out = torch.empty(T_, H, device="cuda", dtype=torch.bfloat16)
    k(y, dest, w, out)
    err = (out.float() - ref).abs().max().item()
    t = do_bench(lambda: k(y, dest, w, out), warmup=10, rep=100)
    print(f"combine block_H={bh} threads={th}: {t * 1e3:.2f} us {nbytes / t * 1e-9:.2f} TB/s err {err:.3g}", flush=True)
