"""MX (e8m0 block-scaled) GEMMs at 8192^3 next to the per-tensor fp8 GEMM of the same tile, one
process (examples/gemm_fp8/): fp8 x fp8, fp4 x fp4, fp8 x fp4, each with row-major and pre-shuffled scales, cold do_bench, best of 3 rounds.
    python scripts/mx_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_fp8")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_tilelang_gemm_mx import mx_matmul, quantize, ref_program  # noqa: E402
from example_tilelang_gemm_fp8 import matmul  # noqa: E402
from tilelang.quantize import preshuffle_mx_scales  # noqa: E402

M = N = K = 8192
runs = {}
for fa, fb in (("e4m3", "e4m3"), ("e2m1", "e2m1"), ("e4m3", "e2m1")):
    a, sa = quantize(torch.randn(M, K, device="cuda") * 3, fa)
    b, sb = quantize(torch.randn(N, K, device="cuda") * 0.2, fb)
    ref = ref_program(a[:128], b, sa[:128], sb, fa, fb)
    k = mx_matmul(M, N, K, a_fmt=fa, b_fmt=fb)
    err = ((k(a, b, sa, sb)[:128].float() - ref).norm() / ref.norm()).item()
    print(f"MX {fa} x {fb}: err {err:.1e}", flush=True)
    runs[f"MX {fa}x{fb}"] = (lambda k=k, a=a, b=b, sa=sa, sb=sb: k(a, b, sa, sb))
    bk = 256 if fa == fb == "e2m1" else 128
    kp = mx_matmul(M, N, K, a_fmt=fa, b_fmt=fb, preshuffle_scales=True)
    pa, pb = preshuffle_mx_scales(sa, 256, bk), preshuffle_mx_scales(sb, 256, bk)
    err = ((kp(a, b, pa, pb)[:128].float() - ref).norm() / ref.norm()).item()
    print(f"MX {fa} x {fb} pre-shuffled scales: err {err:.1e}", flush=True)
    runs[f"MX {fa}x{fb} ps"] = (lambda k=kp, a=a, b=b, sa=pa, sb=pb: k(a, b, sa, sb))
a8 = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
b8 = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
k8 = matmul(M, N, K, 256, 256, 128, 512, 2)
runs["per-tensor fp8"] = lambda: k8(a8, b8)
best = {n: 0.0 for n in runs}
for _ in range(3):
    for n, fn in runs.items():
        best[n] = max(best[n], 2 * M * N * K / do_bench(fn, warmup=5, rep=30) * 1e-9)
print("8192^3 cold, best of 3: " + ", ".join(f"{n} {t:.0f} TF" for n, t in best.items()), flush=True)
