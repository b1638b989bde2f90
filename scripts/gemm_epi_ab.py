"""A/B of the GEMM epilogue: direct MFMA-fragment stores vs LDS-staged row-contiguous 16-byte
stores (example_gemm.matmul(staged_epilogue=True)), same process, interleaved, cold-cache do_bench."""
import sys

import torch

import tilelang
from tilelang.profiler import do_bench

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", "examples", "gemm"))
from example_gemm import matmul  # noqa: E402

for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 4096), (8192, 8192, 8192)]:
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    ref = a @ b
    ks = {}
    for staged in (False, True):
        f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, "float16", staged_epilogue=staged)
        ks[staged] = tilelang.compile(f, out_idx=[-1], target="hip")
        torch.testing.assert_close(ks[staged](a, b), ref, rtol=1e-2, atol=1e-1)
    res = {False: [], True: []}
    for _ in range(3):
        for staged in (False, True):
            res[staged].append(do_bench(lambda: ks[staged](a, b), warmup=20, rep=100))
    lat_blas = do_bench(lambda: a @ b, warmup=20, rep=100)
    fl = 2.0 * M * N * K
    line = f"{M}x{N}x{K}: " + ", ".join(
        f"{'staged' if s else 'direct'} {min(v):.4f} ms {fl / min(v) * 1e-9:.0f} TF" for s, v in res.items())
    print(line + f", torch(hipBLASLt) {lat_blas:.4f} ms {fl / lat_blas * 1e-9:.0f} TF", flush=True)
