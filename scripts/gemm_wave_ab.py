"""fp16 GEMM (B transposed, K-contiguous) A/B of wave layouts for the 256x256 tile in ONE process:
8 waves (2 per SIMD, 64x128 per wave) vs 4 waves (1 per SIMD, 128x128 per wave, AGPR accumulators),
next to hipBLASLt (torch.matmul) on the same data.

    python scripts/gemm_wave_ab.py [M,N,K ...]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm")]
import torch  # noqa: E402

from example_gemm import matmul  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

import json  # noqa: E402
CFGS = [dict(block_M=256, block_N=256, block_K=64, threads=512, num_stages=2, staged_epilogue=True),
        dict(block_M=256, block_N=256, block_K=64, threads=256, num_stages=2, staged_epilogue=True),
        dict(block_M=256, block_N=256, block_K=32, threads=256, num_stages=3, staged_epilogue=True)]
if os.environ.get("TL_GEMM_CFGS"):  # JSON list of extra matmul() kwargs merged into the first config
    CFGS = [dict(CFGS[0], **c) for c in json.loads(os.environ["TL_GEMM_CFGS"])]
shapes = [tuple(int(v) for v in s.split(",")) for s in sys.argv[1:]] or [(8192, 8192, 8192), (4096, 4096, 4096)]
NN = os.environ.get("TL_GEMM_NN") == "1"  # B as [K, N] (the bench's layout) instead of [N, K]
for M, N, K in shapes:
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda").half()
    B = torch.randn(K, N, device="cuda").half() if NN else torch.randn(N, K, device="cuda").half()
    Bt = B if NN else B.T
    ref = (A[:64].float() @ Bt.float())
    fl = 2.0 * M * N * K
    t = do_bench(lambda: A @ Bt, warmup=10, rep=50)
    print(f"{M}x{N}x{K} hipBLASLt: {t:.4f} ms {fl / t * 1e-9:.0f} TF", flush=True)
    for cfg in CFGS + CFGS[:1]:
        try:
            k = matmul(M, N, K, trans_B=not NN, **cfg)
            c = k(A, B)
            err = (c[:64].float() - ref).abs().max().item()
            t = do_bench(lambda: k(A, B), warmup=10, rep=50)
            print(f"{M}x{N}x{K} {cfg}: {t:.4f} ms {fl / t * 1e-9:.0f} TF err {err:.3g}", flush=True)
        except Exception as e:  # noqa: BLE001
            print(f"{cfg}: FAILED {type(e).__name__}: {str(e)[:200]}", flush=True)
