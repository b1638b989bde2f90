"""Tile GEMM (reference: examples/gemm/example_gemm.py) — C = A @ B on MI355X.

``T.gemm`` lowers to CDNA4 MFMA 16x16x32 fragments; the two ``T.copy`` calls in the
``T.Pipelined`` loop become LDS-DMA (``global_load_lds_dwordx4``) issued ``num_stages-1``
tiles ahead into bank-conflict-free swizzled LDS tiles.
"""
import argparse

import tilelang
import tilelang.language as T
from tilelang.layout import PaddedLayout


@tilelang.jit(out_idx=[-1])
def matmul(M, N, K, block_M=128, block_N=128, block_K=32, threads=256, num_stages=3, dtype="float16",
           accum_dtype="float", trans_B=False, swizzle=True, panel=8, staged_epilogue=False):

    B_shape = (N, K) if trans_B else (K, N)

    @T.prim_func
    def gemm(
            A: T.Tensor((M, K), dtype),
            B: T.Tensor(B_shape, dtype),
            C: T.Tensor((M, N), dtype),
    ):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_N, block_K) if trans_B else (block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            if swizzle:
                T.use_swizzle(panel_size=panel)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A[by * block_M, k * block_K], A_shared)
                if trans_B:
                    T.copy(B[bx * block_N, k * block_K], B_shared)
                else:
                    T.copy(B[k * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local, transpose_B=trans_B)
            if staged_epilogue:
                # row-contiguous 16-byte stores: MFMA fragment -> LDS (reuses the A/B ring's
                # space, dead after the loop) -> global
                C_shared = T.alloc_shared((block_M, block_N), dtype)
                # 16-byte row pad: the 16 rows one MFMA store instruction touches land on distinct banks
                T.annotate_layout({C_shared: PaddedLayout((block_M, block_N), 8)})
                T.copy(C_local, C_shared)
                T.copy(C_shared, C[by * block_M, bx * block_N])
            else:
                T.copy(C_local, C[by * block_M, bx * block_N])

    return gemm


def main(M=1024, N=1024, K=1024):
    import torch
    kernel = matmul(M, N, K)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = kernel(a, b)
    torch.testing.assert_close(c, a @ b, rtol=1e-2, atol=1e-2)
    print("All check passed.")
    latency = kernel.get_profiler().do_bench()
    print(f"tilelang Latency: {latency:.4f} ms, {2 * M * N * K / latency * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1024)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--k", type=int, default=1024)
    a = p.parse_args()
    main(a.m, a.n, a.k)
