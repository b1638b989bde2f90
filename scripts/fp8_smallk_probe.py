"""fp8 quad GEMM M=N=8192 around K=1024 (the benchmark table's 0.60x row): time vs K, cold (read
flush) and warm, against hipBLASLt _scaled_mm, to see whether the K=1024 point is an outlier of
the kernel or of the memory system.  python scripts/fp8_smallk_probe.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "gemm_fp8")]

import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_tilelang_gemm_fp8 import matmul  # noqa: E402

M = N = 8192
one = torch.ones((), device="cuda")
for K in [512, 768, 896, 1024, 1152, 1280, 1536, 2048]:
    A = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
    B = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
    k = matmul(M, N, K, staged_epilogue=True)
    row = []
    for flush in (True, False):
        t = do_bench(lambda: k(A, B), warmup=20, rep=100, flush_l2=flush)
        v = do_bench(lambda: torch._scaled_mm(A, B.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16),
                     warmup=20, rep=100, flush_l2=flush)
        row.append(f"{'cold' if flush else 'warm'} {t * 1e3:.1f} us ({2 * M * N * K / t * 1e-9:.0f} TF) "
                   f"vendor {v * 1e3:.1f} us")
    print(f"K={K}: " + " | ".join(row), flush=True)
