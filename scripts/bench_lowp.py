"""Low-precision GEMM numbers on one MI355X: MX-scaled fp4/fp8 at 8192^3 vs
the dense fp4 (10 PF) / fp8 (5 PF) matrix-core roofline, the native bf16 x MXFP4 prefill path and
the dequant decode path.

    python scripts/bench_lowp.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm_fp8"), os.path.join(ROOT, "examples", "dequantize_gemm")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from tilelang.quantize import quantize_mxfp4  # noqa: E402
from example_tilelang_gemm_mx import mx_matmul, quantize, ref_program  # noqa: E402
from example_dequant_gemm_mxfp4 import dequant_gemm_mxfp4, mxfp4_gemm_native, mxfp4_gemv, ref_program as mxfp4_ref  # noqa: E402,E501

PEAK = {"e2m1": 10.0, "e4m3": 5.0}
M = N = K = 8192
for fa, fb, lds in (("e2m1", "e2m1", True), ("e4m3", "e4m3", True), ("e4m3", "e2m1", True)):
    a, sa = quantize(torch.randn(M, K, device="cuda") * 3, fa)
    b, sb = quantize(torch.randn(N, K, device="cuda") * 0.2, fb)
    k = mx_matmul(M, N, K, a_fmt=fa, b_fmt=fb, scales_in_lds=lds)
    c = k(a, b, sa, sb)
    ref = ref_program(a[:256], b, sa[:256], sb, fa, fb)
    err = ((c[:256].float() - ref).norm() / ref.norm()).item()
    lat = do_bench(lambda: k(a, b, sa, sb), warmup=10, rep=50)
    tf = 2 * M * N * K / lat * 1e-9
    peak = min(PEAK[fa], PEAK[fb]) * 1000
    print(f"MX {fa} x {fb} {M}x{N}x{K} scales_in_lds={lds}: {lat:.3f} ms = {tf:.0f} TFLOPS ({100 * tf / peak:.1f}% of the "
          f"{peak / 1000:.0f} PF dense roofline), rel err {err:.2e}", flush=True)

A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
Bq, S = quantize_mxfp4(torch.randn(N, K, device="cuda"))
mxfp4_gemm_native(A, Bq, S)
lat = do_bench(lambda: mxfp4_gemm_native(A, Bq, S), warmup=10, rep=50)
print(f"bf16(->MXFP8) x MXFP4 {M}x{N}x{K} native (quant + scaled MFMA): {lat:.3f} ms = "
      f"{2 * M * N * K / lat * 1e-9:.0f} TFLOPS", flush=True)
kd = dequant_gemm_mxfp4(M, N, K)
lat = do_bench(lambda: kd(A, Bq, S), warmup=10, rep=50)
print(f"bf16 x MXFP4 {M}x{N}x{K} dequant-to-bf16 path: {lat:.3f} ms = {2 * M * N * K / lat * 1e-9:.0f} TFLOPS",
      flush=True)
for m in (1, 16):
    Am = torch.randn(m, K, device="cuda", dtype=torch.bfloat16)
    kd = dequant_gemm_mxfp4(m, N, K)
    lat = do_bench(lambda: kd(Am, Bq, S), warmup=10, rep=100)
    gbs = (N * K // 2 + N * K // 32 + m * K * 2) / lat * 1e-6
    print(f"decode bf16 x MXFP4 {m}x{N}x{K}: {lat * 1e3:.1f} us, {gbs:.0f} GB/s of weights", flush=True)
for m in (1, 4, 8):  # the weight-streaming GEMV (tl/gemv.h: hardware fp4 -> bf16 with the scale folded in)
    Am = torch.randn(m, K, device="cuda", dtype=torch.bfloat16)
    kg = mxfp4_gemv(m, N, K)
    cg = kg(Am, Bq, S)
    rel = ((cg.float() - mxfp4_ref(Am, Bq, S).float()).norm() / mxfp4_ref(Am, Bq, S).float().norm()).item()
    lat = do_bench(lambda: kg(Am, Bq, S), warmup=10, rep=100)
    gbs = (N * K // 2 + N * K // 32 + m * K * 2) / lat * 1e-6
    print(f"decode GEMV bf16 x MXFP4 {m}x{N}x{K}: {lat * 1e3:.1f} us, {gbs:.0f} GB/s of weights, rel err {rel:.1e}",
          flush=True)
a8 = torch.randn(M, K, device="cuda").to(torch.float8_e4m3fn)
b8 = torch.randn(N, K, device="cuda").to(torch.float8_e4m3fn)
one = torch.ones((), device="cuda")
lat = do_bench(lambda: torch._scaled_mm(a8, b8.t(), one, one, out_dtype=torch.bfloat16), warmup=10, rep=50)
print(f"torch._scaled_mm (hipBLASLt) fp8 {M}x{N}x{K}: {2 * M * N * K / lat * 1e-9:.0f} TFLOPS", flush=True)
from example_tilelang_gemm_fp8 import matmul as fp8_matmul  # noqa: E402
kf = fp8_matmul(M, N, K)
c8 = kf(a8, b8)
ref8 = a8[:256].float() @ b8.float().t()
rel = ((c8[:256].float() - ref8).norm() / ref8.norm()).item()
lat = do_bench(lambda: kf(a8, b8), warmup=10, rep=50)
print(f"per-tensor fp8 e4m3 GEMM {M}x{N}x{K} (tilelang, same process): {2 * M * N * K / lat * 1e-9:.0f} TFLOPS, "
      f"rel err {rel:.1e}", flush=True)
