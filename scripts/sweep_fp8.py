"""Per-tensor fp8 (e4m3) GEMM tile sweep at 8192^3 (examples/gemm_fp8/example_tilelang_gemm_fp8.py)
next to hipBLASLt's _scaled_mm in the same process.

    python scripts/sweep_fp8.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_fp8")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_tilelang_gemm_fp8 import matmul  # noqa: E402

M = N = K = 8192
a = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
b = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
ref = a[:256].float() @ b.float().t()
one = torch.ones((), device="cuda")
lat = do_bench(lambda: torch._scaled_mm(a, b.t(), one, one, out_dtype=torch.bfloat16), warmup=10, rep=50)
print(f"hipBLASLt _scaled_mm: {2 * M * N * K / lat * 1e-9:.0f} TF", flush=True)
CFGS = [(256, 256, 128, 512, 2), (256, 128, 128, 512, 3), (128, 256, 128, 512, 3), (256, 128, 256, 512, 2),
        (256, 256, 128, 256, 2), (128, 128, 256, 256, 3), (256, 256, 256, 512, 1)]
for bm, bn, bk, th, st in CFGS:
    tag = f"{bm}x{bn}x{bk} t{th} st{st}"
    try:
        k = matmul(M, N, K, bm, bn, bk, th, st)
        c = k(a, b)
        err = ((c[:256].float() - ref).norm() / ref.norm()).item()
        lat = do_bench(lambda: k(a, b), warmup=10, rep=50)
        print(f"{tag}: {2 * M * N * K / lat * 1e-9:.0f} TF (err {err:.1e})", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{tag}: FAILED {type(e).__name__}: {str(e)[:150]}", flush=True)
