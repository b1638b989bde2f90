"""MX (e8m0 block-scaled) GEMM tile sweep at 8192^3 on one MI355X.
    python scripts/sweep_mx.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_fp8")]
import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_tilelang_gemm_mx import mx_matmul, quantize, ref_program  # noqa: E402

M = N = K = 8192
CFGS = [  # fmt, bm, bn, bk, threads, stages
    ("e4m3", 256, 128, 128, 512, 3), ("e4m3", 256, 256, 128, 512, 2), ("e4m3", 128, 256, 128, 256, 3),
    ("e4m3", 256, 128, 128, 512, 2), ("e4m3", 256, 128, 256, 512, 2), ("e4m3", 128, 128, 128, 256, 3),
    ("e2m1", 256, 128, 256, 512, 3), ("e2m1", 256, 256, 256, 512, 2), ("e2m1", 256, 256, 128, 512, 3),
    ("e2m1", 256, 128, 256, 512, 2), ("e2m1", 128, 256, 256, 256, 3),
]
data = {}
for f, bm, bn, bk, th, st in CFGS:
    if f not in data:
        a, sa = quantize(torch.randn(M, K, device="cuda") * 3, f)
        b, sb = quantize(torch.randn(N, K, device="cuda") * 0.2, f)
        data[f] = (a, b, sa, sb, ref_program(a[:128], b, sa[:128], sb, f, f))
    a, b, sa, sb, ref = data[f]
    tag = f"{f} {bm}x{bn}x{bk} t{th} st{st}"
    try:
        k = mx_matmul(M, N, K, bm, bn, bk, th, st, f, f)
        c = k(a, b, sa, sb)
        err = ((c[:128].float() - ref).norm() / ref.norm()).item()
        lat = do_bench(lambda: k(a, b, sa, sb), warmup=5, rep=30)
        print(f"{tag}: {2 * M * N * K / lat * 1e-9:.0f} TF (err {err:.1e})", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{tag}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
