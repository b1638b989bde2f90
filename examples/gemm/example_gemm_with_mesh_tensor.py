"""GEMM over MeshTensor arguments (reference: examples/gemm/example_gemm_with_mesh_tensor.py).

``T.MeshTensor(shape, policy, mesh, dtype)`` declares the GLOBAL shape of a tensor sharded over
a ``mesh`` of cores/GPUs; inside the program the parameter has the per-core SHARD shape, so the
same kernel body serves any mesh.  With mesh (1, 1) this is a plain single-GPU GEMM; with
``MeshShardingPolicy(x=1, y=0)`` on a (2, 4) mesh each of the 8 MI355X (one process per GPU)
holds a [M/2, K/4] slice of A and so on (see tests/test_mesh_tensor.py for the sharding
arithmetic and tests/test_mesh_comm.py for the T.comm collectives that move tiles between them).
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def matmul(M, N, K, block_M=128, block_N=128, block_K=64, mesh=(1, 1), dtype="float16", accum_dtype="float"):

    @T.prim_func
    def gemm(A: T.MeshTensor((M, K), T.MeshShardingPolicy(x=1, y=0), mesh, dtype),
             B: T.MeshTensor((K, N), T.MeshShardingPolicy(x=1, y=0), mesh, dtype),
             C: T.MeshTensor((M, N), T.MeshShardingPolicy(x=1, y=0), mesh, dtype)):
        sM, sK = A.shape  # per-core shard shape
        _, sN = B.shape
        with T.Kernel(T.ceildiv(sN, block_N), T.ceildiv(sM, block_M), threads=256) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(sK, block_K), num_stages=2):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(B[k * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local)
            T.copy(C_local, C[by * block_M, bx * block_N])

    return gemm


def main(M=1024, N=1024, K=1024):
    import torch
    kernel = matmul(M, N, K)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    torch.testing.assert_close(kernel(a, b), a @ b, rtol=1e-2, atol=1e-2)
    print("All checks pass.")
    print(f"latency: {kernel.get_profiler().do_bench():.4f} ms")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1024)
    a = p.parse_args()
    main(a.m, a.m, a.m)
