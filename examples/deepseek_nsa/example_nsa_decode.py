"""NSA decode: one new token per sequence attends to its selected KV blocks
(reference: examples/deepseek_nsa/example_tilelang_nsa_decode.py:18-135).

The decode token is the last position of the cache, so decode is ``example_nsa_fwd.nsa_fwd`` with
one query row: one workgroup per (sequence, kv head), the G >= 16 query heads of the kv head as
the MFMA M dimension, selected blocks streamed through an LDS-DMA ring.  Padding entries of
``BlockIndices`` (negative, or past the token — the reference pads with ``seq_len``) are skipped.
"""
import argparse

import tilelang

from example_nsa_fwd import nsa_fwd, ref_program


def native_sparse_attention(batch, heads, seq_len, dim, scale=None, block_size=64, groups=16, selected_blocks=16,
                            dtype="float16"):
    """Reference-named entry: kernel(Q [B,1,HQ,D], K/V [B,seq_len,H,D], BlockIndices [B,1,H,S]) -> O."""
    return nsa_fwd(batch, heads, 1, seq_len, dim, False, scale, block_size, groups, selected_blocks, dtype=dtype)


def main(B=64, SEQ_LEN=8192, H=4, HQ=64, D=128, S=16, block_size=64):
    import torch
    kernel = native_sparse_attention(B, HQ, SEQ_LEN, D, block_size=block_size, groups=HQ // H, selected_blocks=S)
    q = torch.randn(B, 1, HQ, D, device="cuda", dtype=torch.float16)
    k = torch.randn(B, SEQ_LEN, H, D, device="cuda", dtype=torch.float16)
    v = torch.randn_like(k)
    nblk = SEQ_LEN // block_size
    idx = torch.stack([torch.randperm(nblk)[:S].sort()[0] for _ in range(B * H)]).view(B, 1, H, S)
    idx = idx.int().cuda()
    o = kernel(q, k, v, idx)
    ref = ref_program(q[:2], k[:2], v[:2], idx[:2], block_size, is_causal=False)
    torch.testing.assert_close(o[:2].float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = tilelang.profiler.do_bench(lambda: kernel(q, k, v, idx))
    kv_bytes = 2 * B * H * S * block_size * D * 2
    print(f"NSA decode B{B} HQ{HQ} H{H} S{S}x{block_size}: {lat * 1e3:.1f} us, {kv_bytes / lat * 1e-6:.0f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--seq_len", type=int, default=8192)
    a = p.parse_args()
    main(a.batch, a.seq_len)
