"""FP16 GEMM, M = N = 8192, K = 256 ... 16384 on one MI355X (reference: benchmark/matmul/
benchmark_matmul.py and its README table, H800 SXM).  B is given [N, K] (``transpose_B``), as the
reference's kernel takes it.  Per row: every candidate tiling of examples/gemm/example_gemm.py is
compiled, checked against fp32 on sampled rows and timed cold; the fastest is reported next to
hipBLASLt (``torch.matmul``, same process) and the reference's H800 number.

    python benchmarks/matmul/benchmark_matmul.py [--out DIR] [--rows 256,4096]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import bench, out_dir_arg, table, tune  # noqa: E402

import torch  # noqa: E402

from example_gemm import matmul  # noqa: E402

M = N = 8192
H800 = {256: 386, 512: 520, 1024: 628, 2048: 705, 4096: 736, 8192: 758, 16384: 766}  # README.md:30-36


def configs(K):
    base = [dict(block_M=256, block_N=256, block_K=64, threads=512, num_stages=2, staged_epilogue=True),
            dict(block_M=256, block_N=256, block_K=64, threads=512, num_stages=2, staged_epilogue=False),
            dict(block_M=256, block_N=256, block_K=32, threads=512, num_stages=3, staged_epilogue=True),
            dict(block_M=256, block_N=128, block_K=64, threads=256, num_stages=2, staged_epilogue=True),
            dict(block_M=128, block_N=256, block_K=64, threads=256, num_stages=2, staged_epilogue=True),
            dict(block_M=128, block_N=128, block_K=64, threads=256, num_stages=2, staged_epilogue=True)]
    return base


def main():
    a = out_dir_arg()
    Ks = [int(x) for x in a.rows.split(",")] if a.rows else list(H800)
    rows, extra = [], {}
    for K in Ks:
        torch.manual_seed(K)
        A = torch.randn(M, K, device="cuda").half()
        B = torch.randn(N, K, device="cuda").half()
        sel = torch.randint(0, M, (48, ), device="cuda")
        ref = A[sel].float() @ B.float().T

        def build(cfg, K=K):
            k = matmul(M, N, K, trans_B=True, **cfg)
            return lambda: k(A, B)

        def check(fn):
            C = fn()
            torch.testing.assert_close(C[sel].float(), ref, rtol=1e-2, atol=2e-2 * K**0.5)

        cfgs = configs(K)[:1] if a.quick else configs(K)
        best = tune(f"fp16 K={K}", cfgs, build, check)
        for _ in range(3):
            torch.matmul(A, B.T)
        vend = bench(lambda: torch.matmul(A, B.T))
        tf = 2 * M * N * K / best["ms"] * 1e-9
        vtf = 2 * M * N * K / vend * 1e-9
        rows.append([K, f"{best['ms']:.4f}", f"{tf:.0f}", H800[K], f"{tf / H800[K]:.2f}x", f"{vtf:.0f}",
                     f"{tf / vtf:.2f}"])
        extra[K] = best
    table("FP16 GEMM M=N=8192 (MI355X, tilelang) vs the reference's H800 table", ["K", "ms", "TFLOPS", "H800 TFLOPS",
          "vs H800", "hipBLASLt TFLOPS", "vs hipBLASLt"], rows, a.out, "matmul_fp16", extra)


if __name__ == "__main__":
    main()
