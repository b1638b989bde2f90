"""Locate the fp8-score MLA decode mismatch: per-row errors under input variations."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "examples", "deepseek_mla"))
import torch  # noqa: E402

from example_mla_decode_kv_fp8 import mla_decode_kv_fp8, quantize_kv, ref_program  # noqa: E402

torch.manual_seed(0)
B, H, S = 4, 128, 1024
k = mla_decode_kv_fp8(B, H, S, 512, 64, block_N=64, num_split=2, num_stages=1, qk_fp8=True)
for kvmul, pe0, qconst in ((1.0, False, False), (3.0, False, False), (3.0, True, False), (3.0, True, True)):
    q = torch.randn(B, H, 512, device="cuda", dtype=torch.bfloat16)
    if qconst:
        q = torch.ones_like(q) * 0.5
    qpe = torch.randn(B, H, 64, device="cuda", dtype=torch.bfloat16) * (0 if pe0 else 1)
    kv8, s = quantize_kv(torch.randn(B, S, 1, 512, device="cuda") * kvmul)
    kpe = torch.randn(B, S, 1, 64, device="cuda", dtype=torch.bfloat16)
    glse = torch.empty(B, H, 2, device="cuda")
    part = torch.empty(B, H, 2, 512, device="cuda")
    out = k(q, qpe, kv8, kpe, s, glse, part).float()
    rq = ref_program(q, qpe, kv8, s, kpe, True)
    rn = ref_program(q, qpe, kv8, s, kpe, False)
    e = (out - rq).abs().amax(-1)  # [B, H]
    bad = (e > 0.02).nonzero().tolist()
    print(f"kv x{kvmul} pe0={pe0} qconst={qconst}: max err vs quant-ref {e.max():.4f}, vs fp32 ref "
          f"{(out - rn).abs().max():.4f}; bad rows {len(bad)} e.g. {bad[:8]}", flush=True)
    if bad:
        b, h = bad[0]
        d = (out[b, h] - rq[b, h]).abs()
        print("   worst cols", d.topk(5).indices.tolist(), "rel-norm", float((out[b, h] - rq[b, h]).norm() / rq[b, h].norm()))
        heads = sorted({hh for _, hh in bad})
        print("   heads with errors:", heads[:40])
