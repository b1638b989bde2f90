"""bf16 x MXFP4 decode GEMV (tl/gemv.h) block shape sweep, M = 1 / 4, N = K = 8192 and 16384.
    python scripts/sweep_gemv_fp4.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "dequantize_gemm")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from tilelang.quantize import quantize_mxfp4  # noqa: E402
from example_dequant_gemm_mxfp4 import mxfp4_gemv, ref_program  # noqa: E402

for N, K in ((8192, 8192), (16384, 16384)):
    Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
    for M in (1, 4):
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        ref = ref_program(A, Bq, S).float()
        for bn, th in ((16, 256), (8, 256), (4, 256), (16, 512), (8, 512), (4, 128), (2, 256), (32, 256)):
            if bn * M > th:
                continue
            try:
                k = mxfp4_gemv(M, N, K, block_N=bn, threads=th)
                c = k(A, Bq, S)
                rel = ((c.float() - ref).norm() / ref.norm()).item()
                lat = do_bench(lambda: k(A, Bq, S), warmup=10, rep=100)
                gbs = (N * K // 2 + N * K // 32) / lat * 1e-6
                print(f"M{M} N{N} K{K} block_N {bn} threads {th}: {lat * 1e3:.1f} us {gbs:.0f} GB/s (rel {rel:.0e})",
                      flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"M{M} bn{bn} t{th}: FAILED {str(e)[:120]}", flush=True)
