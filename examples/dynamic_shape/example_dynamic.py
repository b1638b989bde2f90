"""Dynamic-shape GEMM: one compiled kernel for every (M, N, K) (reference:
examples/dynamic_shape/example_dynamic.py).

``T.dynamic("m")`` shape symbols become runtime kernel arguments bound from the tensors by the
native launcher (which also checks every other shape/stride against them).  ``tl.dynamic_alignment``
promises the dynamic extents are multiples of 8, so the tile copies stay 16-byte vectorised with
bounds guards only on the tile edges (``tl.disable_dynamic_tail_split``: guarded tails, no split loop).
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(pass_configs={"tl.disable_dynamic_tail_split": True, "tl.dynamic_alignment": 8})
def matmul_dynamic_mnk(block_M, block_N, block_K, trans_A, trans_B, in_dtype, out_dtype, accum_dtype, num_stages,
                       threads):
    M = T.dynamic("m")
    N = T.dynamic("n")
    K = T.dynamic("k")
    A_shape = (K, M) if trans_A else (M, K)
    B_shape = (N, K) if trans_B else (K, N)
    A_shared_shape = (block_K, block_M) if trans_A else (block_M, block_K)
    B_shared_shape = (block_N, block_K) if trans_B else (block_K, block_N)

    @T.prim_func
    def dynamic_matmul(A: T.Tensor(A_shape, in_dtype), B: T.Tensor(B_shape, in_dtype),
                       C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared(A_shared_shape, in_dtype)
            B_shared = T.alloc_shared(B_shared_shape, in_dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                if trans_A:
                    T.copy(A[k * block_K, by * block_M], A_shared)
                else:
                    T.copy(A[by * block_M, k * block_K], A_shared)
                if trans_B:
                    T.copy(B[bx * block_N, k * block_K], B_shared)
                else:
                    T.copy(B[k * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local, trans_A, trans_B)
            T.copy(C_local, C[by * block_M, bx * block_N])

    return dynamic_matmul


def matmul_dynamic(M, N, K, block_M, block_N, block_K, trans_A, trans_B, in_dtype, out_dtype, accum_dtype, num_stages,
                   threads, device="cuda"):
    import torch
    kernel = matmul_dynamic_mnk(block_M, block_N, block_K, trans_A, trans_B, in_dtype, out_dtype, accum_dtype,
                                num_stages, threads)
    tdt = getattr(torch, in_dtype)
    A = torch.randn(K, M, device=device, dtype=tdt) if trans_A else torch.randn(M, K, device=device, dtype=tdt)
    B = torch.randn(N, K, device=device, dtype=tdt) if trans_B else torch.randn(K, N, device=device, dtype=tdt)
    C = torch.empty(M, N, device=device, dtype=getattr(torch, out_dtype))
    kernel(A, B, C)
    ref = (A.T if trans_A else A).float() @ (B.T if trans_B else B).float()
    torch.testing.assert_close(C.float(), ref, rtol=1e-2, atol=1e-2)
    return kernel


def main(M=16384, N=16384, K=16384):
    kernel = matmul_dynamic(M, N, K, 128, 128, 32, False, False, "float16", "float16", "float32", 3, 256)
    for m, n, k in ((1024, 1024, 1024), (776, 1536, 2048), (M, N, K)):
        matmul_dynamic(m, n, k, 128, 128, 32, False, False, "float16", "float16", "float32", 3, 256)
    import torch
    A = torch.randn(M, K, device="cuda", dtype=torch.float16)
    B = torch.randn(K, N, device="cuda", dtype=torch.float16)
    C = torch.empty(M, N, device="cuda", dtype=torch.float16)
    lat = kernel.get_profiler().do_bench(lambda: kernel(A, B, C))
    print(f"dynamic-shape GEMM {M}x{N}x{K}: {lat:.3f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=16384)
    p.add_argument("--n", type=int, default=16384)
    p.add_argument("--k", type=int, default=16384)
    a = p.parse_args()
    main(a.m, a.n, a.k)
