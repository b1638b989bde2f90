"""FlashAttention forward, [batch, heads, seq, dim] layout, seq_q != seq_kv
(reference: examples/flash_attention/example_mha_fwd_bhsd.py).

The kernel is ``flashattn_pipelined`` with ``layout="bhsd"``: the same LDS-DMA K/V ring and
``T.Pipelined(order, stage)`` schedule as the bshd bench kernel, only the tile copies index
[b, h, s, d].  Causal masking is bottom-right aligned (query i of seq_q sees keys
<= i + seq_kv - seq_q), the convention of decoding with a KV cache.
"""
import argparse

import tilelang  # noqa: F401

from example_mha_fwd_pipelined import flashattn_pipelined


def flashattn(batch, heads, seq_q, seq_kv, dim, is_causal=False, block_M=256, block_N=64, threads=512,
              num_stages=2, dtype="bfloat16"):
    return flashattn_pipelined(batch, heads, seq_q, dim, is_causal, 1, block_M, block_N, threads, num_stages, dtype,
                               seq_kv=seq_kv, layout="bhsd")


def ref_program(Q, K, V, is_causal):
    import torch
    dim = Q.size(-1)
    scores = torch.einsum("bhqd,bhkd->bhqk", Q.float(), K.float()) / dim**0.5
    if is_causal:
        sq, sk = Q.size(2), K.size(2)
        mask = torch.ones(sq, sk, device=Q.device).tril(sk - sq).bool()
        scores = scores.masked_fill(~mask, float("-inf"))
    return torch.einsum("bhqk,bhkd->bhqd", torch.softmax(scores, -1), V.float()).to(Q.dtype)


def main(batch=1, heads=1, seq_q=256, seq_kv=256, dim=64, is_causal=False, block_M=256, block_N=64, threads=512):
    import torch
    kernel = flashattn(batch, heads, seq_q, seq_kv, dim, is_causal, block_M, block_N, threads)
    q = torch.randn(batch, heads, seq_q, dim, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(batch, heads, seq_kv, dim, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(batch, heads, seq_kv, dim, device="cuda", dtype=torch.bfloat16)
    torch.testing.assert_close(kernel(q, k, v).float(), ref_program(q, k, v, is_causal).float(), rtol=2e-2,
                               atol=2e-2)
    print("All checks pass.")
    pairs = seq_q * seq_kv - (seq_q * (seq_q - 1) // 2 if is_causal else 0)
    flops = 4.0 * batch * heads * pairs * dim
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v))
    print(f"mha fwd bhsd b{batch} h{heads} q{seq_q} kv{seq_kv} d{dim}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=1)
    p.add_argument("--seq_q", type=int, default=256)
    p.add_argument("--seq_kv", type=int, default=256)
    p.add_argument("--dim", type=int, default=64)
    p.add_argument("--is_causal", action="store_true")
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_q, a.seq_kv, a.dim, a.is_causal)
