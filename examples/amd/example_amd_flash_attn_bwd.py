"""FlashAttention backward on MI355X (reference: examples/amd/example_amd_flash_attn_bwd.py).

The AMD backward of the reference is the FA-2 split: a forward that keeps the log-sum-exp, a
Delta = rowsum(O * dO) pre-pass, one kernel for dK/dV per KV tile and one for dQ per query tile.
This example drives the gfx950 kernels of examples/flash_attention/example_mha_bwd.py (K/V
resident in LDS, Q/dO streamed by LDS-DMA, GQA groups accumulated in registers, atomic-free dQ)
through ``torch.autograd`` and checks every gradient against PyTorch."""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flash_attention"))

from example_mha_bwd import attention, ref_program  # noqa: E402


def main(batch=1, heads=8, seq_len=2048, dim=128, is_causal=False, groups=1):
    import torch
    q = torch.randn(batch, seq_len, heads, dim, device="cuda", dtype=torch.float16, requires_grad=True)
    k = torch.randn(batch, seq_len, heads // groups, dim, device="cuda", dtype=torch.float16, requires_grad=True)
    v = torch.randn_like(k, requires_grad=True)
    do = torch.randn_like(q)
    o = attention(q, k, v, is_causal)
    o.backward(do)
    grads = [x.grad.clone() for x in (q, k, v)]
    for x in (q, k, v):
        x.grad = None
    ref = ref_program(q, k, v, is_causal)
    ref.backward(do)
    torch.testing.assert_close(o.float(), ref.float(), rtol=2e-2, atol=2e-2)
    for name, g, x in zip(("dq", "dk", "dv"), grads, (q, k, v)):
        torch.testing.assert_close(g.float(), x.grad.float(), rtol=5e-2, atol=5e-2, msg=name)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    lat = do_bench(lambda: attention(q, k, v, is_causal).backward(do))
    flops = 3.5 * 4.0 * batch * heads * seq_len * seq_len * dim * (0.5 if is_causal else 1.0)
    print(f"flash attention fwd+bwd: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=8)
    p.add_argument("--seq_len", type=int, default=2048)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--is_causal", action="store_true")
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_len, a.dim, a.is_causal)
