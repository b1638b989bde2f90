"""Persistent GEMM (examples/gemm/example_gemm_persistent.py, NT, quad loop) with direct vs staged
(iteration-local LDS) epilogue against the one-tile-per-workgroup GEMM and hipBLASLt; same process,
cold.   python scripts/gemm_persistent_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "gemm")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_gemm import matmul  # noqa: E402
from example_gemm_persistent import matmul_persistent  # noqa: E402

for M, N, K in ((8192, 8192, 1024), (8192, 8192, 4096)):
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(N, K, device="cuda", dtype=torch.float16)
    ref = a[:128].float() @ b.float().T
    ks = {"persistent": matmul_persistent(M, N, K, trans_B=True),
          "persistent_staged": matmul_persistent(M, N, K, trans_B=True, staged_epilogue=True),
          "tile_per_wg_staged": matmul(M, N, K, 256, 256, 64, 512, 2, "float16", trans_B=True, staged_epilogue=True)}
    for n, k in ks.items():
        torch.testing.assert_close(k(a, b)[:128].float(), ref, rtol=2e-2, atol=2e-1)
    res = {n: [] for n in ks}
    res["hipblaslt"] = []
    bt = b.T
    for _ in range(3):
        for n, k in ks.items():
            res[n].append(do_bench(lambda: k(a, b), warmup=20, rep=100))
        res["hipblaslt"].append(do_bench(lambda: a @ bt, warmup=20, rep=100))
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K}: " + ", ".join(f"{n} {fl / min(v) * 1e-9:.0f}" for n, v in res.items()) + " TF", flush=True)
