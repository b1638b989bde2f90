"""2:4 structured-sparse GEMM (reference: benchmark/matmul/benchmark_matmul_sp.py).

A (M x K) is 2:4 sparse, stored compressed (M x K/2 values + int16 metadata, one 4-bit group
index pair per 4 columns: tilelang.utils.sparse.compress); the kernel is
examples/gemm_sp/example_gemm_sp.py, ``T.gemm_sp`` lowered to gfx950 ``v_smfmac_f32_16x16x64``
(the sparse matrix core: K=64 per instruction at the dense instruction's cost).  Candidate tilings
are compiled, checked against the dense fp32 product and timed cold; reported next to the dense
``T.gemm`` kernel and hipBLASLt on the decompressed A.  FLOPs are counted dense (2 M N K), as the
reference does, so the sparse kernel's TFLOPS can exceed the dense peak.

    python benchmarks/matmul/benchmark_matmul_sp.py [--m 16384 --n 16384 --k 16384]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import bench, table, tune  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm_sp"))

import torch  # noqa: E402

from example_gemm_sp import matmul_sp  # noqa: E402
from tilelang.utils.sparse import compress, randn_semi_sparse  # noqa: E402


def configs(quick):
    out = [dict(block_M=256, block_N=256, block_K=64, num_stages=2, threads=512),
           dict(block_M=256, block_N=128, block_K=64, num_stages=2, threads=256),
           dict(block_M=128, block_N=256, block_K=64, num_stages=2, threads=256),
           dict(block_M=128, block_N=128, block_K=128, num_stages=2, threads=256)]
    return out[:1] if quick else out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--k", type=int, default=16384)
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    M, N, K = a.m, a.n, a.k
    torch.manual_seed(0)
    A = randn_semi_sparse(M, K, device="cuda", dtype=torch.float16)
    B = torch.randn(K, N, device="cuda").half()
    As, E = compress(A)
    sel = torch.randint(0, M, (32, ), device="cuda")
    ref = A[sel].float() @ B.float()

    def build(cfg):
        k = matmul_sp(M, N, K, out_dtype="float16", **cfg)
        return lambda: k(As, E, B)

    def check(fn):
        C = fn()
        torch.testing.assert_close(C[sel].float(), ref, rtol=1e-2, atol=2e-2 * (K / 2)**0.5)

    best = tune(f"gemm_sp {M}x{N}x{K}", configs(a.quick), build, check)
    flops = 2.0 * M * N * K
    from example_gemm import matmul
    kd = matmul(M, N, K, 256, 256, 64, 512, 2, staged_epilogue=True)
    dense_ms = bench(lambda: kd(A, B))
    for _ in range(3):
        torch.matmul(A, B)
    vend_ms = bench(lambda: torch.matmul(A, B))
    rows = [["2:4 sparse T.gemm_sp (v_smfmac)", f"{best['ms']:.4f}", f"{flops / best['ms'] * 1e-9:.0f}", "1.00"],
            ["dense T.gemm", f"{dense_ms:.4f}", f"{flops / dense_ms * 1e-9:.0f}", f"{dense_ms / best['ms']:.2f}"],
            ["dense hipBLASLt", f"{vend_ms:.4f}", f"{flops / vend_ms * 1e-9:.0f}", f"{vend_ms / best['ms']:.2f}"]]
    table(f"2:4 sparse fp16 GEMM {M}x{N}x{K} (MI355X; dense-equivalent TFLOPS)",
          ["kernel", "ms", "TFLOPS", "sparse speed-up"], rows, a.out, "matmul_sp", {"best": best})


if __name__ == "__main__":
    main()
