"""Ragged-shape NT GEMMs on the quad main loop (tl::gemm_quad_nt_x with range-checked A / B rows and a
zero-filled last K tile) against the aligned 4096^3 kernel, TFLOPS per useful FLOP, one process,
round-robin after a pre-warm; hipBLASLt (torch.matmul, same layout) beside each.

    python scripts/gemm_ragged_ab.py [--shapes 4096x4096x4096,4000x4096x4096,...]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "gemm")]

import torch  # noqa: E402

import tilelang  # noqa: E402
from example_gemm import matmul  # noqa: E402

DEFAULT = "4096x4096x4096,4000x4096x4096,4096x4000x4096,4096x4096x4000,4000x4000x4000,8192x8192x4000"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default=DEFAULT)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    shapes = [tuple(int(x) for x in s.split("x")) for s in a.shapes.split(",")]
    runs = []
    for M, N, K in shapes:
        f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, "float16", trans_B=True, staged_epilogue=True)
        k = tilelang.compile(f, out_idx=[-1], target="hip")
        quad = "gemm_quad_nt_x" in k.get_kernel_source()
        A = torch.randn(M, K, device="cuda").half()
        B = torch.randn(N, K, device="cuda").half()
        C = k(A, B)
        ref = A.float() @ B.float().t()
        err = ((C.float() - ref).abs().max() / ref.abs().max()).item()
        print(f"{M}x{N}x{K}: quad={quad} rel err {err:.2e}", flush=True)
        runs.append(((M, N, K), quad, lambda k=k, A=A, B=B: k(A, B), lambda A=A, B=B: torch.matmul(A, B.t())))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        for _, _, f, g in runs:
            f()
            g()
        torch.cuda.synchronize()
    res = {r[0]: ([], []) for r in runs}
    for _ in range(5):
        for shp, _, f, g in runs:
            for i, fn in enumerate((f, g)):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[shp][i].append(e0.elapsed_time(e1) / a.reps)
    base = None
    for shp, quad, _, _ in runs:
        M, N, K = shp
        fl = 2.0 * M * N * K
        ours, ven = (sorted(x)[len(x) // 2] for x in res[shp])
        tf, tv = fl / ours * 1e-9, fl / ven * 1e-9
        base = base or tf
        print(f"{M}x{N}x{K}: ours {tf:.1f} TF ({tf / base:.3f} of the first shape), hipBLASLt {tv:.1f} TF, "
              f"ratio {tf / tv:.3f}, main loop {'quad' if quad else 'generic'}", flush=True)


if __name__ == "__main__":
    main()
