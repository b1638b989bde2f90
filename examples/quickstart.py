"""Quickstart (reference: examples/quickstart.py): write a tiled GEMM in the tile DSL, JIT it for
gfx950, check it against PyTorch and time it.

    python examples/quickstart.py           # on an MI355X
    python examples/quickstart.py --cpu     # the same program on the CPU plumbing target
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def matmul(M, N, K, block_M=128, block_N=128, block_K=64, dtype="float16", accum_dtype="float"):

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), B: T.Tensor((K, N), dtype), C: T.Tensor((M, N), dtype)):
        # one workgroup per C tile; 256 threads = 4 wavefronts of 64 lanes
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=256) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            B_shared = T.alloc_shared((block_K, block_N), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            T.use_swizzle(panel_size=8)  # XCD-aware, L2-friendly tile order
            T.clear(C_local)
            # K tiles stream into LDS through the LDS-DMA engine, 2 stages deep
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=2):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(B[k * block_K, bx * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local)  # MFMA 16x16x32
            T.copy(C_local, C[by * block_M, bx * block_N])

    return main


def main(M=1024, N=1024, K=1024, cpu=False):
    import torch
    dev = "cpu" if cpu else "cuda"
    if cpu:
        kernel = tilelang.compile(matmul.get_tir(M, N, K), out_idx=[-1], target="cpu")
    else:
        kernel = matmul(M, N, K)
    a = torch.randn(M, K, device=dev, dtype=torch.float16)
    b = torch.randn(K, N, device=dev, dtype=torch.float16)
    c = kernel(a, b)
    torch.testing.assert_close(c.float(), a.float() @ b.float(), rtol=1e-2, atol=1e-1)
    print("Kernel output matches PyTorch.")
    print(kernel.get_kernel_source()[:400] if not cpu else "(CPU target)")
    if not cpu:
        lat = kernel.get_profiler().do_bench()
        print(f"latency {lat:.4f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--cpu", action="store_true")
    a = p.parse_args()
    main(cpu=a.cpu) if not a.cpu else main(256, 256, 256, cpu=True)
