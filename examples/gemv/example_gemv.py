"""GEMV y = A x (reference: examples/gemv/example_gemv.py).

A is [N, K] row-major (fp16/bf16), x is [K].  GEMV is HBM-bound (2 bytes/FLOP), so the
schedule is about streaming A at full bandwidth: each block owns ``block_N`` rows, every
lane reads 16 B (8 halves) of a row per step with a plain vector load (no LDS round trip --
each A element is used once), multiplies by the matching x slice (L2-resident, shared by
all blocks) into fp32 partial sums, and one cross-lane reduction per row finishes.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def gemv(N, K, block_N=8, block_K=512, threads=256, dtype="float16", accum_dtype="float", nt=True):
    """``nt``: the weight matrix is streamed once -- non-temporal 16-byte loads."""
    pol = "evict_first" if nt else None

    @T.prim_func
    def main(A: T.Tensor((N, K), dtype), x: T.Tensor((K, ), dtype), y: T.Tensor((N, ), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), threads=threads) as bn:
            a_frag = T.alloc_fragment((block_N, block_K), dtype)
            acc = T.alloc_fragment((block_N, block_K), accum_dtype)
            row = T.alloc_fragment((block_N, ), accum_dtype)
            T.clear(acc)
            for ko in T.serial(T.ceildiv(K, block_K)):
                T.copy(A[bn * block_N, ko * block_K], a_frag, eviction_policy=pol)
                for i, j in T.Parallel(block_N, block_K):
                    acc[i, j] += T.Cast(accum_dtype, a_frag[i, j]) * T.Cast(accum_dtype, x[ko * block_K + j])
            T.reduce_sum(acc, row, dim=1)
            for i in T.Parallel(block_N):
                y[bn * block_N + i] = row[i]

    return main


def ref_program(A, x):
    return (A.float() @ x.float()).to(A.dtype)


def main(N=16384, K=16384):
    import torch
    kernel = gemv(N, K)
    A = torch.randn(N, K, device="cuda", dtype=torch.float16)
    x = torch.randn(K, device="cuda", dtype=torch.float16)
    torch.testing.assert_close(kernel(A, x), ref_program(A, x), rtol=1e-2, atol=1e-1)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(A, x))
    print(f"gemv {N}x{K}: {lat:.4f} ms, {N * K * 2 / lat * 1e-6:.1f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=16384)
    p.add_argument("--k", type=int, default=16384)
    a = p.parse_args()
    main(a.n, a.k)
