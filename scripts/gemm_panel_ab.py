"""Bench GEMM (4096^3 fp16 NT, quad loop) with different rasterisation panels / no swizzle,
same process, round-robin, cold.   python scripts/gemm_panel_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "gemm")]
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_gemm import matmul  # noqa: E402

M = N = K = 4096
a = torch.randn(M, K, device="cuda", dtype=torch.float16)
b = torch.randn(N, K, device="cuda", dtype=torch.float16)
ref = a[:64].float() @ b.float().T
ks = {}
for name, kw in (("panel8", dict(panel=8)), ("panel4", dict(panel=4)), ("panel16", dict(panel=16)),
                 ("panel2", dict(panel=2)), ("noswizzle", dict(swizzle=False))):
    k = matmul(M, N, K, 256, 256, 64, 512, 2, "float16", trans_B=True, staged_epilogue=True, **kw)
    torch.testing.assert_close(k(a, b)[:64].float(), ref, rtol=2e-2, atol=2e-1)
    ks[name] = k
res = {n: [] for n in ks}
res["hipblaslt"] = []
bt = b.T
for _ in range(4):
    for n, k in ks.items():
        res[n].append(do_bench(lambda: k(a, b), warmup=20, rep=100))
    res["hipblaslt"].append(do_bench(lambda: a @ bt, warmup=20, rep=100))
fl = 2.0 * M * N * K
print(", ".join(f"{n} {fl / min(v) * 1e-9:.0f}" for n, v in res.items()) + " TF (cold, best of 4)")
