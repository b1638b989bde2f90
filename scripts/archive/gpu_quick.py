"""Quick on-GPU sanity + timing for the GEMM path (used during development)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "examples", "gemm"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import torch
from example_gemm import matmul


def bench(fn, iters=50, warmup=10):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


torch.manual_seed(0)
print("device:", torch.cuda.get_device_name(0), flush=True)
# correctness
for (M, N, K, bm, bn, bk, th, st, tb) in [(1024, 1024, 1024, 128, 128, 32, 256, 3, False),
                                          (512, 512, 256, 64, 64, 32, 256, 2, False),
                                          (1024, 1024, 1024, 128, 128, 64, 256, 2, True)]:
    k = matmul(M, N, K, bm, bn, bk, th, st, trans_B=tb)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn((N, K) if tb else (K, N), device="cuda", dtype=torch.float16)
    c = k(a, b)
    ref = a @ (b.t() if tb else b)
    err = (c.float() - ref.float()).abs().max().item()
    print(f"gemm {M}x{N}x{K} tile {bm}x{bn}x{bk} th{th} st{st} tB{tb}: max err {err:.4f}", flush=True)
M = N = K = 4096
a = torch.randn(M, K, device="cuda", dtype=torch.float16)
b = torch.randn(K, N, device="cuda", dtype=torch.float16)
ref = a @ b
t = bench(lambda: a @ b)
print(f"torch/hipBLASLt 4096^3: {t:.3f} ms {2*M*N*K/t*1e-9:.1f} TF", flush=True)
for cfg in [(128, 128, 32, 256, 3), (128, 128, 64, 256, 2), (128, 128, 64, 256, 3), (256, 128, 64, 256, 2),
            (256, 256, 64, 512, 2), (256, 256, 32, 512, 3), (128, 256, 64, 256, 2)]:
    try:
        k = matmul(M, N, K, *cfg)
        c = k(a, b)
        err = (c.float() - ref.float()).abs().max().item()
        t = bench(lambda: k(a, b))
        print(f"cfg {cfg}: {t:.3f} ms {2*M*N*K/t*1e-9:.1f} TF  err {err:.3f}", flush=True)
    except Exception as ex:
        print(f"cfg {cfg}: FAILED {type(ex).__name__}: {str(ex)[:300]}", flush=True)
