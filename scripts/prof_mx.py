"""Run the MX GEMM (8192^3) a few times for rocprofv3 (--pmc / --kernel-trace).
    python scripts/prof_mx.py e4m3 e4m3 [reps]
    python scripts/prof_mx.py pt8 pt8 [reps]   # per-tensor fp8 GEMM of the same tile, for comparison"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_fp8")]
import torch  # noqa: E402

from example_tilelang_gemm_mx import mx_matmul, quantize  # noqa: E402

fa, fb = sys.argv[1], sys.argv[2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
M = N = K = 8192
if fa == "pt8":
    from example_tilelang_gemm_fp8 import matmul
    a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
    b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
    k = matmul(M, N, K, 256, 256, 128, 512, 2)
    args = (a, b)
else:
    a, sa = quantize(torch.randn(M, K, device="cuda") * 3, fa)
    b, sb = quantize(torch.randn(N, K, device="cuda") * 0.2, fb)
    k = mx_matmul(M, N, K, a_fmt=fa, b_fmt=fb)
    args = (a, b, sa, sb)
for _ in range(reps):
    k(*args)
torch.cuda.synchronize()
print("done")
