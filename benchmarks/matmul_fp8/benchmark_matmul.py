"""FP8 (e4m3, OCP) GEMM, M = N = 8192, K = 256 ... 16384 on one MI355X (reference:
benchmark/matmul_fp8/benchmark_matmul.py and its README table, H800 SXM).  B is [N, K]; fp32
accumulation, bf16 output.  Candidate tilings of examples/gemm_fp8/example_tilelang_gemm_fp8.py
(block_K % 128 == 0: the f8f6f4 MFMA at twice the bf16 rate), fastest per row, next to
hipBLASLt's ``torch._scaled_mm`` (unit scales, bf16 out) in the same process.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import bench, out_dir_arg, table, tune  # noqa: E402

import torch  # noqa: E402

from example_tilelang_gemm_fp8 import matmul  # noqa: E402

M = N = 8192
H800 = {256: 569, 512: 858, 1024: 1129, 2048: 1343, 4096: 1467, 8192: 1507, 16384: 1541}  # README.md:30-36


def configs(K):
    return [dict(block_M=256, block_N=256, block_K=128, threads=512, num_stages=2),
            dict(block_M=256, block_N=256, block_K=128, threads=512, num_stages=2, staged_epilogue=True),
            dict(block_M=256, block_N=256, block_K=256, threads=512, num_stages=1, staged_epilogue=True),
            dict(block_M=256, block_N=128, block_K=128, threads=256, num_stages=2, staged_epilogue=True),
            dict(block_M=128, block_N=128, block_K=128, threads=256, num_stages=3, staged_epilogue=True)]


def main():
    a = out_dir_arg()
    Ks = [int(x) for x in a.rows.split(",")] if a.rows else list(H800)
    rows, extra = [], {}
    one = torch.ones((), device="cuda")
    for K in Ks:
        torch.manual_seed(K)
        A = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
        B = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
        sel = torch.randint(0, M, (48, ), device="cuda")
        ref = A[sel].float() @ B.float().T

        def build(cfg, K=K):
            k = matmul(M, N, K, **cfg)
            return lambda: k(A, B)

        def check(fn):
            C = fn()
            torch.testing.assert_close(C[sel].float(), ref, rtol=2e-2, atol=2e-2 * K**0.5)

        cfgs = configs(K)[:1] if a.quick else configs(K)
        best = tune(f"fp8 K={K}", cfgs, build, check)
        vend = None
        try:
            f = lambda: torch._scaled_mm(A, B.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)  # noqa: E731
            for _ in range(3):
                f()
            vend = bench(f)
        except Exception as e:  # noqa: BLE001
            print(f"_scaled_mm unavailable: {e}")
        tf = 2 * M * N * K / best["ms"] * 1e-9
        vtf = 2 * M * N * K / vend * 1e-9 if vend else float("nan")
        rows.append([K, f"{best['ms']:.4f}", f"{tf:.0f}", H800[K], f"{tf / H800[K]:.2f}x", f"{vtf:.0f}",
                     f"{tf / vtf:.2f}"])
        extra[K] = best
    table("FP8 e4m3 GEMM M=N=8192 (MI355X, tilelang) vs the reference's H800 table", ["K", "ms", "TFLOPS",
          "H800 TFLOPS", "vs H800", "hipBLASLt _scaled_mm TFLOPS", "vs hipBLASLt"], rows, a.out, "matmul_fp8", extra)


if __name__ == "__main__":
    main()
