"""Staged (LDS, 16-byte row stores) vs direct fragment-store epilogue of the quad-loop NT GEMM at the
bench MoE expert-GEMM shapes (dense stand-ins: GEMM2 4608x4096x2048, GEMM1 4608x4096x4096) and
4096^3; same process, round-robin, cold.   python scripts/gemm_epi_shape_ab.py"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "examples", "gemm")]
import torch  # noqa: E402

import tilelang  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402
from example_gemm import matmul  # noqa: E402

for M, N, K in ((4608, 4096, 2048), (4608, 4096, 4096), (4096, 4096, 4096)):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    ks = {}
    for st in (False, True):
        f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, "bfloat16", trans_B=True, staged_epilogue=st)
        ks[st] = tilelang.compile(f, out_idx=[-1], target="hip")
        assert "gemm_quad_nt" in ks[st].get_kernel_source()
        ref = a[:64].float() @ b.float().T
        torch.testing.assert_close(ks[st](a, b)[:64].float(), ref, rtol=2e-2, atol=2e-2 * K ** 0.5)
    res = {False: [], True: []}
    for _ in range(4):
        for st in (False, True):
            res[st].append(do_bench(lambda: ks[st](a, b), warmup=20, rep=100))
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K} bf16 NT: direct {fl / min(res[False]) * 1e-9:.0f} TF, staged {fl / min(res[True]) * 1e-9:.0f} TF",
          flush=True)
