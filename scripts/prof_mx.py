"""Run the MX GEMM (8192^3) a few times for rocprofv3 (--pmc / --kernel-trace).
    python scripts/prof_mx.py e4m3 e4m3 [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_fp8")]
import torch  # noqa: E402

from example_tilelang_gemm_mx import mx_matmul, quantize  # noqa: E402

fa, fb = sys.argv[1], sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
M = N = K = 8192
a, sa = quantize(torch.randn(M, K, device="cuda") * 3, fa)
b, sb = quantize(torch.randn(N, K, device="cuda") * 0.2, fb)
k = mx_matmul(M, N, K, a_fmt=fa, b_fmt=fb)
for _ in range(reps):
    k(a, b, sa, sb)
torch.cuda.synchronize()
print("done")
