"""Block-sparse attention forward on one MI355X (reference: benchmark/blocksparse_attention/
benchmark_tilelang_block_sparse_fmha.py with benchmark_configs.py [4, 2, 256, 64, topk 2, block 64],
against a dense library FMHA).  The reference publishes no numbers for this benchmark ("parity
unpinned"): the table reports the tilelang block-sparse kernel (examples/blocksparse_attention/
example_block_sparse_attn.py, top-k key blocks per query block, causal), the dense tilelang FA
on the same shape and torch's SDPA (the library dense FMHA), all in one process.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import bench, out_dir_arg, table, tune  # noqa: E402

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from example_block_sparse_attn import blocksparse_attn, compact_mask, ref_program  # noqa: E402

# BATCH, N_HEADS, SEQ_LEN, D_HEAD, TOPK, BLOCK: the reference's config, then production-sized ones
CONFIGS = [(4, 2, 256, 64, 2, 64), (1, 32, 4096, 128, 16, 64), (1, 32, 8192, 128, 32, 64), (4, 32, 8192, 128, 64, 64)]


def topk_mask(B, H, S, topk, block, seed):
    """Per query block: the diagonal block plus the top-k scored earlier blocks (causal)."""
    nb = S // block
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.rand(B, H, nb, nb, device="cuda", generator=g)
    causal = torch.ones(nb, nb, device="cuda", dtype=torch.bool).tril()
    x = x.masked_fill(~causal, -1.0)
    k = min(topk, nb)
    idx = x.topk(k, -1).indices
    mask = torch.zeros(B, H, nb, nb, device="cuda", dtype=torch.bool).scatter_(-1, idx, True)
    mask &= causal
    mask |= torch.eye(nb, device="cuda", dtype=torch.bool)
    return mask


def main():
    a = out_dir_arg()
    rows, extra = [], {}
    for (Bz, Hh, S, D, topk, blk) in CONFIGS:
        torch.manual_seed(S)
        q, k, v = (torch.randn(Bz, Hh, S, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
        mask = topk_mask(Bz, Hh, S, topk, blk, S)
        idx, cnt = compact_mask(mask)
        ref = ref_program(q[:1, :1], k[:1, :1], v[:1, :1], mask[:1, :1], blk)

        def build(cfg):
            kern = blocksparse_attn(Bz, Hh, S, D, True, blk, **cfg)
            return lambda: kern(q, k, v, idx, cnt)

        def check(fn):
            o = fn()
            torch.testing.assert_close(o[:1, :1].float(), ref.float(), rtol=2e-2, atol=2e-2)

        cfgs = [dict(threads=256, num_stages=2), dict(threads=256, num_stages=3), dict(threads=128, num_stages=2)]
        best = tune(f"bsa {Bz}x{Hh}x{S}x{D} top{topk}", cfgs[:1] if a.quick else cfgs, build, check)
        active = int(cnt.sum())
        flops = 4 * D * blk * blk * active
        sdpa = bench(lambda: F.scaled_dot_product_attention(q, k, v, is_causal=True))
        dense_flops = 4 * Bz * Hh * S * S * D * 0.5
        rows.append([f"{Bz}x{Hh}x{S}x{D}", topk, f"{active / mask.numel():.3f}", f"{best['ms']:.4f}",
                     f"{flops / best['ms'] * 1e-9:.1f}", f"{sdpa:.4f}", f"{dense_flops / sdpa * 1e-9:.1f}",
                     f"{sdpa / best['ms']:.2f}x"])
        extra[f"{Bz}x{Hh}x{S}x{D}"] = best
    table("Block-sparse attention fwd bf16 causal (MI355X): tilelang block-sparse vs torch SDPA (dense)",
          ["B x H x S x D", "topk", "density", "ms", "TFLOPS (active blocks)", "SDPA dense ms",
           "SDPA TFLOPS (causal)", "speedup vs dense"], rows, a.out, "blocksparse_attention", extra)


if __name__ == "__main__":
    main()
