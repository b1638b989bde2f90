"""Persistent GEMM (reference: examples/gemm/example_gemm_persistent.py, ``T.Persistent`` in src/ir.cc:115-187).

The grid is sized to what the chip holds at once (``num_cus * blocks_per_cu`` blocks); each block
walks output tiles ``bid, bid + wave, ...`` in grouped (L2-panel) order, so the prologue/epilogue
cost of a block is paid once per CU instead of once per tile and the tail wave is balanced.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def matmul_persistent(M, N, K, block_M=256, block_N=256, block_K=64, threads=512, num_stages=2, num_cus=256,
                      blocks_per_cu=1, group_size=8, dtype="float16", accum_dtype="float", trans_B=False,
                      staged_epilogue=False):
    """``trans_B``: B given as [N, K] (the 256x256 NT tile then runs the quad GEMM loop).
    ``staged_epilogue``: each tile's C leaves through a row-padded LDS tile as 16-byte row stores;
    the tile loop is ``lds_iteration_local`` so that tile takes the operand ring's bytes."""
    from tilelang.layout import PaddedLayout
    tiles_m = (M + block_M - 1) // block_M
    tiles_n = (N + block_N - 1) // block_N
    wave = min(num_cus * blocks_per_cu, tiles_m * tiles_n)
    B_shape = (N, K) if trans_B else (K, N)
    B_tile = (block_N, block_K) if trans_B else (block_K, block_N)

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor(B_shape, dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(wave, threads=threads) as bid:
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared(B_tile, dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            C_cast = T.alloc_fragment((block_M, block_N), dtype)
            for bm, bn in T.Persistent([tiles_m, tiles_n], wave, bid, group_size,
                                       lds_iteration_local=staged_epilogue):
                T.clear(C_local)
                for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                    T.copy(A[bm * block_M, k * block_K], A_shared)
                    if trans_B:
                        T.copy(B[bn * block_N, k * block_K], B_shared)
                    else:
                        T.copy(B[k * block_K, bn * block_N], B_shared)
                    T.gemm(A_shared, B_shared, C_local, transpose_B=trans_B)
                if staged_epilogue:
                    C_s = T.alloc_shared((block_M, block_N), dtype)
                    T.annotate_layout({C_s: PaddedLayout((block_M, block_N), 8)})
                    T.copy(C_local, C_s)
                    T.copy(C_s, C[bm * block_M, bn * block_N])
                else:
                    T.copy(C_local, C_cast)
                    T.copy(C_cast, C[bm * block_M, bn * block_N])

    return main


def main(M=4096, N=4096, K=4096):
    import torch
    kernel = matmul_persistent(M, N, K)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    torch.testing.assert_close(kernel(a, b), a @ b, rtol=1e-2, atol=1e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, b))
    print(f"persistent GEMM {M}x{N}x{K}: {lat:.4f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=4096)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--k", type=int, default=4096)
    a = p.parse_args()
    main(a.m, a.n, a.k)
