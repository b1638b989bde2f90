"""User-level MFMA-emitter GEMM (reference: benchmark/matmul/benchmark_matmul_intrinsic.py).

The kernel is examples/gemm/example_gemm_intrinsics.py: the program issues the matrix-core
instructions itself through ``tilelang.intrinsics.MatrixCoreIntrinEmitter`` (ldmatrix_a/b into
registers, ``v_mfma_f32_{16x16x32,32x32x16}_f16`` / i8, stmatrix) instead of ``T.gemm``.  Every
candidate warp tiling is compiled, checked against fp32 and timed cold; the fastest is reported
next to the ``T.gemm`` kernel (examples/gemm/example_gemm.py) and hipBLASLt in the same process.
Default shape as the reference script: M = N = K = 16384, fp16 in, fp16 out.

    python benchmarks/matmul/benchmark_matmul_intrinsic.py [--m 16384 --n 16384 --k 16384] [--dtype int8]
"""
import argparse
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from common import bench, table, tune  # noqa: E402

import torch  # noqa: E402

from example_gemm_intrinsics import tl_matmul  # noqa: E402


def configs(dtype, quick):
    out = []
    for (brw, bcw), (wr, wc), ms, stage in itertools.product([(2, 4), (4, 2), (2, 2)], [(128, 64), (64, 128), (64, 64)],
                                                             [32, 16], [2, 3]):
        if stage == 3 and brw * wr * bcw * wc > 128 * 128:
            continue  # three 128-deep stages of a 256-wide tile exceed the 160 KB of LDS
        out.append(dict(block_row_warps=brw, block_col_warps=bcw, warp_row_tiles=wr, warp_col_tiles=wc, micro_size=ms,
                        stage=stage))
    return out[:2] if quick else out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--k", type=int, default=16384)
    ap.add_argument("--dtype", default="float16", choices=["float16", "int8"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--quick", action="store_true")
    a = ap.parse_args()
    M, N, K = a.m, a.n, a.k
    i8 = a.dtype == "int8"
    out_dtype, accum = ("int32", "int32") if i8 else ("float16", "float32")
    torch.manual_seed(0)
    if i8:
        A = torch.randint(-8, 8, (M, K), device="cuda", dtype=torch.int8)
        B = torch.randint(-8, 8, (N, K), device="cuda", dtype=torch.int8)
    else:
        A = torch.randn(M, K, device="cuda").half()
        B = torch.randn(N, K, device="cuda").half()
    sel = torch.randint(0, M, (32, ), device="cuda")
    ref = A[sel].float() @ B.float().T

    def build(cfg):
        k = tl_matmul(M, N, K, a.dtype, out_dtype, accum, **cfg)
        return lambda: k(A, B)

    def check(fn):
        C = fn()
        if i8:
            assert torch.equal(C[sel].float(), ref)
        else:
            torch.testing.assert_close(C[sel].float(), ref, rtol=1e-2, atol=2e-2 * K**0.5)

    best = tune(f"intrinsic {a.dtype} {M}x{N}x{K}", configs(a.dtype, a.quick), build, check)
    flops = 2.0 * M * N * K
    rows = [["MFMA emitter (example_gemm_intrinsics)", f"{best['ms']:.4f}", f"{flops / best['ms'] * 1e-9:.0f}"]]
    if not i8:
        from example_gemm import matmul
        kg = matmul(M, N, K, 256, 256, 64, 512, 2, trans_B=True, staged_epilogue=True)
        rows.append(["T.gemm (example_gemm, 256x256x64)", f"{bench(lambda: kg(A, B)):.4f}", ""])
        for _ in range(3):
            torch.matmul(A, B.T)
        rows.append(["hipBLASLt (torch.matmul)", f"{bench(lambda: torch.matmul(A, B.T)):.4f}", ""])
        for r in rows[1:]:
            r[2] = f"{flops / float(r[1]) * 1e-9:.0f}"
    table(f"MFMA-intrinsic GEMM {a.dtype} {M}x{N}x{K} (MI355X)", ["kernel", "ms", "TFLOPS"], rows, a.out,
          f"matmul_intrinsic_{a.dtype}", {"best": best})


if __name__ == "__main__":
    main()
