"""Elementwise add (reference: examples/elementwise/example_elementwise_add.py:13-57).

C = A + B over an [M, N] tensor.  Each block stages a ``block_M x block_N`` tile through
registers: the ``T.Parallel`` nest is partitioned over the 64-lane waves with 128-bit
vector loads/stores (8 x fp16 / 4 x fp32 per lane), so the kernel is a straight HBM stream.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def elementwise_add(M, N, block_M=32, block_N=256, threads=256, in_dtype="float32", out_dtype="float32", nt=True):
    """``nt``: A, B and C are streamed once -- non-temporal 16-byte accesses (evict_first)."""
    pol = "evict_first" if nt else None

    @T.prim_func
    def main(A: T.Tensor((M, N), in_dtype), B: T.Tensor((M, N), in_dtype), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_local = T.alloc_fragment((block_M, block_N), in_dtype)
            B_local = T.alloc_fragment((block_M, block_N), in_dtype)
            C_local = T.alloc_fragment((block_M, block_N), out_dtype)
            T.copy(A[by * block_M, bx * block_N], A_local, eviction_policy=pol)
            T.copy(B[by * block_M, bx * block_N], B_local, eviction_policy=pol)
            for i, j in T.Parallel(block_M, block_N):
                C_local[i, j] = A_local[i, j] + B_local[i, j]
            T.copy(C_local, C[by * block_M, bx * block_N], eviction_policy=pol)

    return main


def get_configs():
    return [dict(block_M=bm, block_N=bn, threads=t) for bm in (16, 32, 64) for bn in (128, 256, 512)
            for t in (128, 256)]


def main(M=1024, N=1024, dtype="float32"):
    import torch
    kernel = elementwise_add(M, N, in_dtype=dtype, out_dtype=dtype)
    tdt = getattr(torch, dtype)
    a = torch.randn(M, N, device="cuda", dtype=tdt)
    b = torch.randn(M, N, device="cuda", dtype=tdt)
    torch.testing.assert_close(kernel(a, b), a + b, rtol=1e-2, atol=1e-2)
    print("All check passed.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b))
    nbytes = 3 * M * N * a.element_size()
    print(f"elementwise add {M}x{N}: {lat:.4f} ms, {nbytes / lat * 1e-6:.1f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1024)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--dtype", default="float32")
    a = p.parse_args()
    main(a.m, a.n, a.dtype)
