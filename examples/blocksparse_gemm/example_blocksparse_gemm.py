"""Block-sparse GEMM (reference: examples/blocksparse_gemm/example_blocksparse_gemm.py).

C = A B where only the (block_M x block_K) x (block_K x block_N) products enabled in
``BlockMask[M/bm, N/bn, K/bk]`` contribute.  Each block walks its K range and skips disabled
K-blocks entirely (no HBM traffic, no MFMA), so the cost scales with the mask density.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def blocksparse_matmul(M, N, K, block_M=128, block_N=128, block_K=32, threads=256, dtype="float16",
                       accum_dtype="float"):
    mask_shape = (M // block_M, N // block_N, K // block_K)

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), BlockMask: T.Tensor(mask_shape, "bool"),
             C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            C_cast = T.alloc_fragment((block_M, block_N), dtype)
            T.clear(C_local)
            for k in T.serial(K // block_K):
                if BlockMask[by, bx, k]:
                    T.copy(A[by * block_M, k * block_K], A_shared)
                    T.copy(B[k * block_K, bx * block_N], B_shared)
                    T.gemm(A_shared, B_shared, C_local)
            T.copy(C_local, C_cast)
            T.copy(C_cast, C[by * block_M, bx * block_N])

    return main


def ref_program(A, B, mask, block_M, block_N, block_K):
    import torch
    M, K = A.shape
    N = B.shape[1]
    C = torch.zeros(M, N, dtype=torch.float32, device=A.device)
    for i in range(M // block_M):
        for j in range(N // block_N):
            for k in range(K // block_K):
                if mask[i, j, k]:
                    C[i * block_M:(i + 1) * block_M, j * block_N:(j + 1) * block_N] += (
                        A[i * block_M:(i + 1) * block_M, k * block_K:(k + 1) * block_K].float()
                        @ B[k * block_K:(k + 1) * block_K, j * block_N:(j + 1) * block_N].float())
    return C.to(A.dtype)


def main(M=1024, N=1024, K=1024, sparsity=0.5):
    import torch
    kernel = blocksparse_matmul(M, N, K)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    mask = torch.rand(M // 128, N // 128, K // 32, device="cuda") > sparsity
    torch.testing.assert_close(kernel(a, b, mask).float(), ref_program(a, b, mask, 128, 128, 32).float(), rtol=1e-2,
                               atol=1e-1)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b, mask))
    print(f"block-sparse GEMM {M}x{N}x{K} density {1 - sparsity:.2f}: {lat:.4f} ms")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1024)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--k", type=int, default=1024)
    p.add_argument("--sparsity", type=float, default=0.5)
    a = p.parse_args()
    main(a.m, a.n, a.k, a.sparsity)
