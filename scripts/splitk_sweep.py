"""Tile / split sweep of the split-K example (examples/gemm_splitk) at 1024x1024x16384 fp16, B [K, N],
fp32 atomics into C (the scripts/gpu_bench_examples.py workload), against torch's GEMM.

    python scripts/splitk_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_splitk")]

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_tilelang_gemm_splitk import matmul_splitk  # noqa: E402

M, N, K = 1024, 1024, 16384
CFGS = [  # block_M, block_N, block_K, threads, split_k, num_stages
    (128, 128, 32, 256, 8, 2), (128, 128, 64, 256, 8, 2), (128, 128, 64, 256, 4, 2), (128, 128, 64, 256, 16, 2),
    (256, 128, 64, 512, 8, 2), (256, 128, 64, 512, 16, 2), (128, 256, 64, 512, 8, 2), (256, 256, 64, 512, 16, 2),
    (256, 256, 64, 512, 8, 2), (128, 128, 64, 256, 8, 3), (64, 128, 64, 256, 8, 2), (128, 64, 64, 256, 16, 2),
]


def main():
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    ref = a.float() @ b.float()
    c = torch.zeros(M, N, device="cuda")
    print(f"torch {do_bench(lambda: a @ b):.4f} ms", flush=True)
    for bm, bn, bk, th, sk, st in CFGS:
        try:
            k = matmul_splitk(M, N, K, block_M=bm, block_N=bn, block_K=bk, split_k=sk, threads=th, num_stages=st)
            c.zero_()
            k(a, b, c)
            err = (c - ref).abs().max().item()

            def run():
                c.zero_()
                k(a, b, c)

            ms = do_bench(run)
            print(f"{bm}x{bn}x{bk} t{th} split{sk} st{st}: {ms:.4f} ms, {2 * M * N * K / ms * 1e-9:.1f} TF "
                  f"(max err {err:.3g})", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{bm}x{bn}x{bk} t{th} split{sk} st{st}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)


if __name__ == "__main__":
    main()
