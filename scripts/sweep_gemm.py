"""fp16 GEMM config sweep (bench shape 4096^3 and 8192x8192x4096): warm back-to-back and cold
(do_bench) TFLOPS per config in one process (guide rule 24); correctness spot-checked.

    python scripts/sweep_gemm.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm")]
import torch  # noqa: E402

import tilelang  # noqa: E402
from example_gemm import matmul  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

CFGS = [
    # M, N, K, bm, bn, bk, threads, stages, mfma_shape, phased (None = default: phased + prefetch)
    (4096, 4096, 4096, 256, 256, 64, 512, 2, "16x16", None),
    (4096, 4096, 4096, 256, 128, 64, 512, 2, "16x16", None),
    (4096, 4096, 4096, 128, 256, 64, 512, 2, "16x16", None),
    (4096, 4096, 4096, 256, 128, 64, 256, 2, "16x16", None),
    (4096, 4096, 4096, 256, 128, 128, 512, 2, "16x16", None),
    (8192, 8192, 4096, 256, 256, 64, 512, 2, "16x16", None),
    (8192, 8192, 4096, 256, 128, 64, 512, 2, "16x16", None),
]
if len(sys.argv) > 1 and sys.argv[1] == "--quick":
    CFGS = [c for c in CFGS if c[0] == 4096 and c[5] == 64 and c[8] == "16x16"]
for M, N, K, bm, bn, bk, th, st, sh, ph in CFGS:
    tag = f"{M}x{N}x{K} {bm}x{bn}x{bk} t{th} st{st} {sh}{(' phased=' + str(ph)) if ph else ''}"
    try:
        f = matmul.get_tir(M, N, K, bm, bn, bk, th, st, "float16")
        k = tilelang.compile(f, out_idx=[-1], target="hip",
                             pass_configs={"tl.mfma_shape": sh, **({} if ph is None else {"tl.gemm_phased": ph})})
        a = torch.randn(M, K, device="cuda", dtype=torch.float16)
        b = torch.randn(K, N, device="cuda", dtype=torch.float16)
        c = k(a, b)
        err = max((c[:128].float() - a[:128].float() @ b.float()).abs().max().item(),
                  (c[-128:].float() - a[-128:].float() @ b.float()).abs().max().item())
        fn = lambda: k(a, b)  # noqa: E731
        cold = do_bench(fn, warmup=5, rep=30)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            fn()
        e1.record()
        torch.cuda.synchronize()
        warm = e0.elapsed_time(e1) / 30
        fl = 2.0 * M * N * K
        print(f"{tag}: err {err:.3g} | cold {fl / cold * 1e-9:.1f} TF | warm {fl / warm * 1e-9:.1f} TF", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{tag}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
ref = torch.randn(4096, 4096, device="cuda", dtype=torch.float16)
t = do_bench(lambda: ref @ ref, warmup=5, rep=30)
print(f"torch (hipBLASLt) 4096^3: cold {2 * 4096**3 / t * 1e-9:.1f} TF", flush=True)
