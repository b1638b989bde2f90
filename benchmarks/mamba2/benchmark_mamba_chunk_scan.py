"""Mamba-2 SSD chunk scan forward, b8 h80 g1 chunk 256 headdim 64 dstate 128, seq 1K ... 32K on one
MI355X (reference: benchmark/mamba2/benchmark_mamba_chunk_scan.py and README.md:41-46, H800 SXM,
same FLOP count).  Candidate tilings of examples/linear_attention/example_mamba_chunk_scan.py (the row-tiled
``chunk_scan_fwd`` and the whole-chunk ``chunk_scan_fwd_fused``),
checked against the fp32 einsum definition on the smallest row, fastest per row.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import out_dir_arg, table, tune  # noqa: E402

import torch  # noqa: E402

from example_mamba_chunk_scan import chunk_scan_fwd, chunk_scan_fwd_fused, flops, make_inputs, ref_program  # noqa

B, H, G, CH, P, N = 8, 80, 1, 256, 64, 128
H800 = {1024: 126.477, 2048: 130.195, 4096: 133.054, 8192: 134.362, 16384: 135.711, 32768: 135.379}


def configs():
    return [dict(kernel="fused", block_K=64, threads=512, num_stages=2),
            dict(kernel="fused", block_K=32, threads=512, num_stages=2),
            dict(kernel="fused", block_K=64, threads=256, num_stages=2),
            dict(kernel="fused", block_K=64, threads=512, num_stages=1),
            dict(block_M=256, block_N=64, block_K=64, threads=256, num_stages=2),
            dict(block_M=256, block_N=64, block_K=64, threads=512, num_stages=2),
            dict(block_M=256, block_N=64, block_K=32, threads=256, num_stages=2),
            dict(block_M=128, block_N=64, block_K=64, threads=256, num_stages=2),
            dict(block_M=128, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True),
            dict(block_M=128, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True, lean=True),
            dict(block_M=128, block_N=64, block_K=32, threads=256, num_stages=2, xcd_group=True, lean=True),
            dict(block_M=64, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True, lean=True),
            dict(block_M=64, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True),
            dict(block_M=128, block_N=64, block_K=32, threads=256, num_stages=2),
            dict(block_M=64, block_N=64, block_K=64, threads=256, num_stages=2),
            dict(block_M=128, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True, factored=True),
            dict(block_M=128, block_N=64, block_K=32, threads=256, num_stages=2, xcd_group=True, factored=True),
            dict(block_M=64, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True, factored=True),
            dict(block_M=256, block_N=64, block_K=64, threads=256, num_stages=2, xcd_group=True, factored=True),
            # r5: the interior / diagonal split without the XCD grouping (which cost 15 % alone)
            dict(block_M=128, block_N=64, block_K=64, threads=256, num_stages=2, lean=True),
            dict(block_M=128, block_N=64, block_K=32, threads=256, num_stages=2, lean=True),
            dict(block_M=64, block_N=64, block_K=64, threads=256, num_stages=2, lean=True),
            dict(block_M=128, block_N=64, block_K=64, threads=256, num_stages=2, factored=True)]


def selected():
    """``TL_MAMBA_CFGS="8,15,16"``: only those configs (indices into ``configs()``)."""
    sel = os.environ.get("TL_MAMBA_CFGS")
    cfgs = configs()
    return [cfgs[int(i)] for i in sel.split(",")] if sel else cfgs


def main():
    a = out_dir_arg()
    Ls = [int(x) for x in a.rows.split(",")] if a.rows else list(H800)
    rows, extra = [], {}
    for L in Ls:
        torch.manual_seed(L)
        args = make_inputs(B, L, CH, G, H, P, N)
        ref = ref_program(*[t[:1] if t.dim() > 1 and t.shape[0] == B else t for t in args]) if L <= 2048 else None

        def build(cfg, L=L):
            cfg = dict(cfg)
            fac = chunk_scan_fwd_fused if cfg.pop("kernel", None) == "fused" else chunk_scan_fwd
            k = fac(B, L, CH, G, H, P, N, **cfg)
            return lambda: k(*args)

        def check(fn):
            out = fn()
            if ref is not None:
                torch.testing.assert_close(out[:1].float(), ref, rtol=2e-2, atol=5e-2)
            assert torch.isfinite(out).all()

        cfgs = configs()[:1] if a.quick else selected()
        best = tune(f"mamba2 L={L}", cfgs, build, check)
        tf = flops(B, L, CH, H, P, N) / best["ms"] * 1e-9
        rows.append([L, f"{best['ms']:.4f}", f"{tf:.1f}", H800[L], f"{tf / H800[L]:.2f}x"])
        extra[L] = best
        del args
        torch.cuda.empty_cache()
    table("Mamba-2 chunk scan b8 h80 chunk256 d64 dstate128 (MI355X, tilelang) vs the reference's H800 table",
          ["seq_len", "ms", "TFLOPS", "H800 TFLOPS", "vs H800"], rows, a.out, "mamba2_chunk_scan", extra)


if __name__ == "__main__":
    main()
