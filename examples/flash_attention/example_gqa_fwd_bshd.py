"""Grouped-query FlashAttention forward, [batch, seq, heads, dim] layout
(reference: examples/flash_attention/example_gqa_fwd_bshd.py).

``flashattn_pipelined`` with ``groups`` query heads per K/V head: each workgroup (256 query rows
of one head) streams the K/V tiles of head ``h // groups`` through the LDS-DMA ring.  Workgroups
of the same KV group run back to back in launch order (head is grid.y), so a K/V tile read by one
is usually still in the XCD's L2 for the next.
"""
import argparse

import tilelang  # noqa: F401

from example_mha_fwd import ref_program
from example_mha_fwd_pipelined import flashattn_pipelined


def flashattn(batch, heads, seq_len, dim, is_causal=False, groups=16, block_M=256, block_N=64, threads=512,
              num_stages=2, dtype="bfloat16"):
    return flashattn_pipelined(batch, heads, seq_len, dim, is_causal, groups, block_M, block_N, threads, num_stages,
                               dtype)


def main(batch=1, heads=64, seq_len=4096, dim=128, is_causal=False, groups=16):
    import torch
    kernel = flashattn(batch, heads, seq_len, dim, is_causal, groups)
    q = torch.randn(batch, seq_len, heads, dim, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(kernel(q, k, v).float(), ref_program(q, k, v, is_causal, groups).float(), rtol=2e-2,
                               atol=2e-2)
    print("All checks pass.")
    flops = 4.0 * batch * heads * seq_len * seq_len * dim * (0.5 if is_causal else 1.0)
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v))
    print(f"gqa fwd b{batch} h{heads} kvh{heads // groups} s{seq_len} d{dim}: {lat:.3f} ms, "
          f"{flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=64)
    p.add_argument("--seq_len", type=int, default=4096)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--is_causal", action="store_true")
    p.add_argument("--groups", type=int, default=16)
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_len, a.dim, a.is_causal, a.groups)
