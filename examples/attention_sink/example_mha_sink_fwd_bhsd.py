"""MHA attention with a learned per-head sink (bhsd layout)
(reference: examples/attention_sink/example_mha_sink_fwd_bhsd.py).

The GQA sink kernel with one query head per K/V head (``groups=1``): same LDS-DMA K/V ring,
unmasked main loop + masked diagonal tail, longest-first query tiles.  Optional sliding window.
"""
import argparse

from example_gqa_sink_fwd_bhsd import flashattn_sink, flops, ref_program


def main(batch=1, heads=32, seq_q=4096, seq_kv=4096, dim=128, window_size=None, dtype="bfloat16"):
    import torch
    kernel = flashattn_sink(batch, heads, seq_q, seq_kv, dim, 1, window_size, dtype=dtype)
    tdt = getattr(torch, dtype)
    q = torch.randn(batch, heads, seq_q, dim, device="cuda", dtype=tdt)
    k = torch.randn(batch, heads, seq_kv, dim, device="cuda", dtype=tdt)
    v = torch.randn(batch, heads, seq_kv, dim, device="cuda", dtype=tdt)
    sinks = torch.randn(heads, device="cuda", dtype=tdt)
    o = kernel(q, k, v, sinks)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, sinks, window_size).float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v, sinks))
    print(f"mha+sink fwd b{batch} h{heads} s{seq_q} d{dim}: {lat:.3f} ms, "
          f"{flops(batch, heads, seq_q, seq_kv, dim, window_size) / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=32)
    p.add_argument("--seq_q", type=int, default=4096)
    p.add_argument("--seq_kv", type=int, default=4096)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--window_size", type=int, default=None)
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_q, a.seq_kv, a.dim, a.window_size)
