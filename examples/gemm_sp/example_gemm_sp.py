"""2:4 structured-sparse GEMM on the gfx950 sparse matrix cores (``v_smfmac_f32_16x16x64``).

Reference: ``examples/gemm_sp/example_gemm_sp.py`` (NVIDIA ``mma.sp`` with CUTLASS metadata,
4090/H20 configs).  Here ``A`` is compressed with ``tilelang.utils.sparse.compress`` to
``A_sparse [M, K/2]`` + ``E [M, K/16]`` int16 smfmac indices; each 64-wide K step of a 16x16
tile is one smfmac, i.e. twice the dense MFMA K per instruction.  A, E and B stream through an
LDS-DMA ring; the accumulator lives in the direct MFMA layout and is staged through LDS for
16-byte global stores.
"""
import argparse

import torch

import tilelang
import tilelang.language as T
from tilelang.layout import make_metadata_layout
from tilelang.utils.sparse import compress, randn_semi_sparse

E_FACTOR, E_DTYPE = 16, "int16"


@tilelang.jit(out_idx=[-1])
def matmul_sp(M, N, K, block_M=256, block_N=256, block_K=64, num_stages=2, threads=512, dtype="float16",
              accum_dtype="float", out_dtype="float16", trans_B=False):
    b_shape = (N, K) if trans_B else (K, N)
    b_tile = (block_N, block_K) if trans_B else (block_K, block_N)

    @T.prim_func
    def gemm_sp(A_sparse: T.Tensor((M, K // 2), dtype), E: T.Tensor((M, K // E_FACTOR), E_DTYPE),
                B: T.Tensor(b_shape, dtype), C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K // 2), dtype)
            E_shared = T.alloc_shared((block_M, block_K // E_FACTOR), E_DTYPE)
            B_shared = T.alloc_shared(b_tile, dtype)
            C_shared = T.alloc_shared((block_M, block_N), out_dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.annotate_layout({E_shared: make_metadata_layout(E_shared)})
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A_sparse[by * block_M, k * block_K // 2], A_shared)
                T.copy(E[by * block_M, k * block_K // E_FACTOR], E_shared)
                if trans_B:
                    T.copy(B[bx * block_N, k * block_K], B_shared)
                else:
                    T.copy(B[k * block_K, bx * block_N], B_shared)
                T.gemm_sp(A_shared, E_shared, B_shared, C_local, False, trans_B)
            T.copy(C_local, C_shared)
            T.copy(C_shared, C[by * block_M, bx * block_N])

    return gemm_sp


def ref_program(A, B, trans_B=False):
    return (A.float() @ (B.float().t() if trans_B else B.float())).to(torch.float16)


def main(M=8192, N=8192, K=8192, trans_B=False, bench=True):
    kernel = matmul_sp(M, N, K, trans_B=trans_B)
    a = randn_semi_sparse(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn((N, K) if trans_B else (K, N), device="cuda", dtype=torch.float16)
    a_sp, e = compress(a)
    c = kernel(a_sp, e, b)
    torch.testing.assert_close(c.float(), ref_program(a, b, trans_B).float(), rtol=1e-2, atol=1e-1)
    print("2:4 sparse GEMM matches the dense fp32 reference")
    if bench:
        from tilelang.profiler import do_bench
        ms = do_bench(lambda: kernel(a_sp, e, b))
        dense = do_bench(lambda: a @ (b.t() if trans_B else b))
        flops = 2.0 * M * N * K
        print(f"sparse: {ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOPS (dense-equivalent)")
        print(f"torch dense (hipBLASLt): {dense:.3f} ms  {flops / dense / 1e9:.1f} TFLOPS")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--k", type=int, default=8192)
    ap.add_argument("--trans_b", action="store_true")
    args = ap.parse_args()
    main(args.m, args.n, args.k, args.trans_b)
