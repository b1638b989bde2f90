"""Stream-K GEMM (reference: examples/gemm_streamk/example_tilelang_gemm_streamk.py).

C = A B^T.  The K-iterations of the first ``streamk_tiles`` output tiles are split evenly over
``programs`` blocks (one per CU): a block that finishes a tile's last K-iteration writes it, a
block holding a partial range adds its partial sum with fp32 atomics.  The remaining tiles are
computed data-parallel (one per block per round).  This removes the tail-wave imbalance when the
tile count is not a multiple of the CU count (e.g. 24 tiles on 256 CUs).
"""
import argparse

import tilelang
import tilelang.language as T


def streamk_schedule(M, N, K, block_M, block_N, block_K, programs):
    tiles = ((M + block_M - 1) // block_M) * ((N + block_N - 1) // block_N)
    iters_per_tile = (K + block_K - 1) // block_K
    sk_tiles = tiles % programs
    if tiles - sk_tiles > programs:
        sk_tiles += programs
    dp_tiles = tiles - sk_tiles
    sk_iters = sk_tiles * iters_per_tile
    return dict(tiles=tiles, iters_per_tile=iters_per_tile, sk_tiles=sk_tiles, dp_rounds=dp_tiles // programs,
                full=sk_iters // programs, partial=sk_iters % programs)


@tilelang.jit
def matmul_streamk(M, N, K, block_M=64, block_N=128, block_K=64, programs=256, threads=256, num_stages=2,
                   dtype="float16", accum_dtype="float"):
    sch = streamk_schedule(M, N, K, block_M, block_N, block_K, programs)
    ipt = sch["iters_per_tile"]
    tiles_n = (N + block_N - 1) // block_N
    full, partial, sk_tiles, dp_rounds = sch["full"], sch["partial"], sch["sk_tiles"], sch["dp_rounds"]

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((N, K), dtype), C: T.Tensor((M, N), "float32")):
        with T.Kernel(programs, threads=threads) as pid:
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_N, block_K), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            start = T.alloc_var("int32")
            end_it = T.alloc_var("int32")
            start = pid * full + T.min(pid, partial)
            last = (pid + 1) * full + T.min(pid + 1, partial)
            while start < last:
                end_it = T.min(start + (ipt - start % ipt), last)
                tile = start // ipt
                pm = tile // tiles_n
                pn = tile % tiles_n
                k0 = start % ipt
                T.clear(C_local)
                for k in T.serial(end_it - start):
                    T.copy(A[pm * block_M, (k0 + k) * block_K], A_shared)
                    T.copy(B[pn * block_N, (k0 + k) * block_K], B_shared)
                    T.gemm(A_shared, B_shared, C_local, transpose_B=True)
                T.atomic_add(C[pm * block_M, pn * block_N], C_local)
                start = end_it
            for r in T.serial(dp_rounds):
                tile = sk_tiles + r * programs + pid
                pm = tile // tiles_n
                pn = tile % tiles_n
                T.clear(C_local)
                for k in T.Pipelined(ipt, num_stages=num_stages):
                    T.copy(A[pm * block_M, k * block_K], A_shared)
                    T.copy(B[pn * block_N, k * block_K], B_shared)
                    T.gemm(A_shared, B_shared, C_local, transpose_B=True)
                T.copy(C_local, C[pm * block_M, pn * block_N])

    return main


def main(M=256, N=1024, K=512, programs=256):
    import torch
    kernel = matmul_streamk(M, N, K, programs=programs)
    A = torch.rand(M, K, device="cuda", dtype=torch.float16) * 2 - 1
    B = torch.rand(N, K, device="cuda", dtype=torch.float16) * 2 - 1
    C = torch.zeros(M, N, device="cuda")
    kernel(A, B, C)
    torch.testing.assert_close(C, A.float() @ B.float().t(), rtol=1e-2, atol=1e-2)
    print("All checks pass.")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=256)
    p.add_argument("--n", type=int, default=1024)
    p.add_argument("--k", type=int, default=512)
    a = p.parse_args()
    main(a.m, a.n, a.k)
