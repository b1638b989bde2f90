"""Split-K GEMM (reference: examples/gemm_splitk/example_tilelang_gemm_splitk.py:5-43).

C[M,N] (fp32, zero-initialised) += A[:, kslice] @ B[kslice, :] for ``split_k`` K slices in
parallel: grid (N/bn, M/bm, split_k).  Small-M/N, large-K problems otherwise leave most of
the 256 CUs idle; splitting K multiplies the block count.  Each block finishes with a
tile-wide ``T.atomic_add`` into C (``global_atomic_add_f32`` per element for fp32 output; for
fp16 / bf16 output the lowering pairs the two adjacent columns each lane holds into one
``global_atomic_pk_add_{f16,bf16}`` -- AtomicAddVectorize, tests/test_language_atomic.py).
For fp32 output the accumulator tile goes through a row-padded LDS tile first, so each wave
instruction adds 64 consecutive floats (lower_tile_op.lower_atomic_staged): at 1024x1024x16384
split 8 that took the kernel from 0.162 to 0.088 ms (0.074 ms with the 64-deep K tile default,
0.068 ms at split 4; torch 0.109 ms -- profiles/r6/splitk_sweep.log).
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit
def matmul_splitk(M, N, K, block_M=128, block_N=128, block_K=64, split_k=4, threads=256, num_stages=2,
                  dtype="float16", accum_dtype="float", out_dtype="float32"):
    splitK = K // split_k

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), split_k, threads=threads) as (bx, by, bz):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.clear(C_local)
            for ko in T.Pipelined(T.ceildiv(splitK, block_K), num_stages=num_stages):
                T.copy(A[by * block_M, bz * splitK + ko * block_K], A_shared)
                T.copy(B[bz * splitK + ko * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local)
            T.atomic_add(C[by * block_M, bx * block_N], C_local)

    return main


@tilelang.jit
def matmul_splitk_elementwise(M, N, K, block_M=128, block_N=128, block_K=32, split_k=4, threads=256,
                              dtype="float16", accum_dtype="float", out_dtype="float32"):
    """Same schedule with the reference's per-element atomics inside a ``T.Parallel`` nest."""
    splitK = K // split_k

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), split_k, threads=threads) as (bx, by, bz):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.clear(C_local)
            for ko in T.Pipelined(T.ceildiv(splitK, block_K), num_stages=2):
                T.copy(A[by * block_M, bz * splitK + ko * block_K], A_shared)
                T.copy(B[bz * splitK + ko * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local)
            for i, j in T.Parallel(block_M, block_N):
                T.atomic_add(C[by * block_M + i, bx * block_N + j], C_local[i, j])

    return main


def main(M=1024, N=1024, K=8192, split_k=8):
    import torch
    kernel = matmul_splitk(M, N, K, split_k=split_k)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = torch.zeros(M, N, device="cuda", dtype=torch.float32)
    kernel(a, b, c)
    torch.testing.assert_close(c, a.float() @ b.float(), rtol=1e-2, atol=1e-1)
    print("All checks pass.")

    def run():
        c.zero_()
        kernel(a, b, c)

    lat = kernel.get_profiler().do_bench(run)
    print(f"split-K GEMM {M}x{N}x{K} (split {split_k}): {lat:.4f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1024)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--k", type=int, default=8192)
    p.add_argument("--split_k", type=int, default=8)
    a = p.parse_args()
    main(a.m, a.n, a.k, a.split_k)
