"""GEMM written with the user-level MFMA emitter (reference: examples/gemm/example_gemm_intrinsics.py).

The tile loop stages A/B into LDS with ``T.Parallel`` copies, then for every 32-deep (64 for
int8) K step each wave loads its register fragments with ``ldmatrix_a/b`` and issues one
``v_mfma_*_16x16x*`` per warp-tile pair through ``mma``; ``stmatrix`` writes the accumulators
to an LDS tile in the reference's [M/16, N/16, 16, 16] layout, copied out by a ``T.Parallel``
store.  ``T.gemm`` does all of this (plus swizzles, LDS-DMA and the phased schedule) by itself;
this form is for programs that need to own the instruction stream.
"""
import argparse

import tilelang
import tilelang.language as T
from tilelang.intrinsics import MatrixCoreIntrinEmitter


@tilelang.jit(out_idx=[2])
def tl_matmul(M, N, K, in_dtype="float16", out_dtype="float16", accum_dtype="float32", block_row_warps=2,
              block_col_warps=2, warp_row_tiles=64, warp_col_tiles=64, chunk=None, stage=2):
    if chunk is None:
        chunk = 64 if in_dtype == "int8" else 32
    emitter = MatrixCoreIntrinEmitter(in_dtype, in_dtype, accum_dtype, a_transposed=False, b_transposed=True,
                                      block_row_warps=block_row_warps, block_col_warps=block_col_warps,
                                      warp_row_tiles=warp_row_tiles, warp_col_tiles=warp_col_tiles, chunk=chunk)
    block_M = block_row_warps * warp_row_tiles
    block_N = block_col_warps * warp_col_tiles
    block_K = chunk
    C_shared_shape = (block_M // 16, block_N // 16, 16, 16)

    @T.prim_func
    def gemm_intrinsics(A: T.Tensor((M, K), in_dtype), B: T.Tensor((N, K), in_dtype),
                        C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=emitter.threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), in_dtype)
            B_shared = T.alloc_shared((block_N, block_K), in_dtype)
            C_shared = T.alloc_shared(C_shared_shape, out_dtype)
            A_local = T.alloc_local((emitter.warp_rows * emitter.local_size_a, ), in_dtype)
            B_local = T.alloc_local((emitter.warp_cols * emitter.local_size_b, ), in_dtype)
            C_local = T.alloc_local((emitter.warp_rows * emitter.warp_cols * emitter.local_size_out, ), accum_dtype)
            T.use_swizzle(panel_size=8)
            T.clear(C_local)
            for ko in T.Pipelined(K // block_K, num_stages=stage):
                for i, k in T.Parallel(block_M, block_K):
                    A_shared[i, k] = A[by * block_M + i, ko * block_K + k]
                for j, k in T.Parallel(block_N, block_K):
                    B_shared[j, k] = B[bx * block_N + j, ko * block_K + k]
                for ki in T.serial(block_K // emitter.micro_size_k):
                    emitter.ldmatrix_a(A_local, A_shared, ki)
                    emitter.ldmatrix_b(B_local, B_shared, ki)
                    emitter.mma(A_local, B_local, C_local)
            emitter.stmatrix(C_local, C_shared)
            for i, j in T.Parallel(block_M, block_N):
                C[by * block_M + i, bx * block_N + j] = C_shared[i // 16, j // 16, i % 16, j % 16]

    return gemm_intrinsics


def ref_program(A, B):
    return A.float() @ B.float().T


def main(M=4096, N=4096, K=4096, in_dtype="float16"):
    import torch
    out_dtype = "int32" if in_dtype == "int8" else "float16"
    accum = "int32" if in_dtype == "int8" else "float32"
    kernel = tl_matmul(M, N, K, in_dtype, out_dtype, accum)
    if in_dtype == "int8":
        a = torch.randint(-8, 8, (M, K), device="cuda", dtype=torch.int8)
        b = torch.randint(-8, 8, (N, K), device="cuda", dtype=torch.int8)
    else:
        a = torch.randn(M, K, device="cuda", dtype=torch.float16)
        b = torch.randn(N, K, device="cuda", dtype=torch.float16)
    c = kernel(a, b)
    torch.testing.assert_close(c.float(), ref_program(a, b), rtol=1e-2, atol=1e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b))
    print(f"intrinsic-emitter GEMM {M}x{N}x{K} {in_dtype}: {lat:.3f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=4096)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--k", type=int, default=4096)
    p.add_argument("--dtype", default="float16")
    a = p.parse_args()
    main(a.m, a.n, a.k, a.dtype)
