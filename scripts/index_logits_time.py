"""Sparse fine-tune indexer logits (examples/dsa_sparse_finetune/indexer_topk_reducesum.py
``index_logits``), S tokens in 2 sequences, H64 D128 bf16: time + check against the fp32 definition
on a few tokens.

    python scripts/index_logits_time.py [S]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "dsa_sparse_finetune")]
import torch  # noqa: E402

from index import prepare_token_indices  # noqa: E402
from indexer_topk_reducesum import index_logits  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
H, D = 64, 128
torch.manual_seed(0)
q = torch.randn(S, H, D, device="cuda", dtype=torch.bfloat16)
k = torch.randn(S, D, device="cuda", dtype=torch.bfloat16)
w = torch.randn(S, H, device="cuda", dtype=torch.bfloat16)
offsets = torch.tensor([0, S // 2, S], dtype=torch.int32, device="cuda")
tok = prepare_token_indices(offsets)
offs = torch.zeros(S + 1, dtype=torch.int32, device="cuda")
offs[:3] = offsets
kern = index_logits(S, H, D)
fn = lambda: kern(q.reshape(S * H, D).contiguous(), k, w, offs, tok)  # noqa: E731
out = fn()
rows = [5, S // 2 + 7, S - 1]
for t in rows:
    lo = 0 if t < S // 2 else S // 2
    sc = (q[t].float() @ k[lo:t + 1].float().T).relu() * (w[t].float()[:, None] * D**-0.5)
    ref = sc.sum(0)
    torch.testing.assert_close(out[t, lo:t + 1], ref, rtol=2e-2, atol=2e-2)
    assert torch.isinf(out[t, t + 1:]).all() if t + 1 < S else True
ms = do_bench(fn, warmup=5, rep=30)
flops = 2.0 * H * D * (S // 2) * (S // 2 + 1)  # causal within each of the 2 sequences (x2 seqs / 2)
print(f"index_logits S={S} H{H} D{D}: {ms:.4f} ms, {flops / ms * 1e-9:.1f} TFLOPS (causal useful work)")
