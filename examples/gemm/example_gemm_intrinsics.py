"""GEMM written with the user-level MFMA emitter (reference: examples/gemm/example_gemm_intrinsics.py,
testing/python/amd/test_tilelang_gemm_mfma_intrinsic.py / _preshuffle.py).

The tile loop stages A/B into XOR-swizzled LDS tiles with ``T.copy`` (LDS-DMA, pipelined), then
for every K step each wave loads its register fragments with ``ldmatrix_a/b`` (16-byte runs)
and issues its MFMAs through ``mfma``; ``stmatrix`` writes the accumulators straight to C.
``T.gemm`` does all of this (plus the phased K-half schedule) by itself; this form is for programs
that need to own the instruction stream.

``b_preshuffle``: B is stored tile-major (``shuffle_weight``) and each wave loads its fragments
directly from global memory (coalesced 1 KiB per wave and tile), so only A goes through LDS.
"""
import argparse

import tilelang
import tilelang.language as T
from tilelang.intrinsics import MatrixCoreIntrinEmitter, make_mfma_swizzle_layout


@tilelang.jit(out_idx=[2])
def tl_matmul(M, N, K, in_dtype="float16", out_dtype="float16", accum_dtype="float32", block_row_warps=2,
              block_col_warps=4, warp_row_tiles=128, warp_col_tiles=64, chunk=None, stage=2, micro_size=32,
              k_pack=1, b_preshuffle=False, b_transposed=True, fp8_k_dim=None, reduce_k=1):
    """``reduce_k``: split every K stage over that many wave groups (thread binding 1) and sum the
    partial accumulators through LDS before the store (the reference emitter's ``reduce_k``)."""
    emitter = MatrixCoreIntrinEmitter(in_dtype, in_dtype, accum_dtype, a_transposed=False, b_transposed=b_transposed,
                                      block_row_warps=block_row_warps, block_col_warps=block_col_warps,
                                      warp_row_tiles=warp_row_tiles, warp_col_tiles=warp_col_tiles,
                                      chunk=chunk or 1 << 30, micro_size=micro_size, k_pack=k_pack,
                                      b_preshuffle=b_preshuffle, fp8_k_dim=fp8_k_dim, reduce_k=reduce_k)
    pk = emitter.micro_size_k * k_pack
    if chunk is None:
        chunk = max(pk, 128 // (1 if in_dtype.startswith(("float8", "int8")) else 2))
    emitter.chunk = chunk  # K per wave group per stage
    assert chunk % pk == 0
    assert not (reduce_k > 1 and b_preshuffle), "reduce_k with LDS-staged operands only"
    block_M = block_row_warps * warp_row_tiles
    block_N = block_col_warps * warp_col_tiles
    block_K = chunk * reduce_k
    threads = emitter.threads if reduce_k == 1 else (emitter.threads // reduce_k, reduce_k)
    ms = micro_size
    if b_preshuffle:
        B_shape = (N // ms, K // pk, ms, pk) if b_transposed else (K // pk, N // ms, pk, ms)
    else:
        B_shape = (N, K) if b_transposed else (K, N)
    B_sh = (block_N, block_K) if b_transposed else (block_K, block_N)

    @T.prim_func
    def gemm_intrinsics(A: T.Tensor((M, K), in_dtype), B: T.Tensor(B_shape, in_dtype),
                        C: T.Tensor((M, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), in_dtype)
            A_local = T.alloc_local((emitter.warp_rows * emitter.local_size_a, ), in_dtype)
            B_local = T.alloc_local((emitter.warp_cols * emitter.local_size_b, ), in_dtype)
            C_local = T.alloc_local((emitter.warp_rows * emitter.warp_cols * emitter.local_size_out, ), accum_dtype)
            if not b_preshuffle:
                B_shared = T.alloc_shared(B_sh, in_dtype)
                T.annotate_layout({A_shared: make_mfma_swizzle_layout(A_shared),
                                   B_shared: make_mfma_swizzle_layout(B_shared)})
            else:
                T.annotate_layout({A_shared: make_mfma_swizzle_layout(A_shared)})
            T.use_swizzle(panel_size=8)
            T.clear(C_local)
            rk = T.get_thread_binding(1) if reduce_k > 1 else 0
            for ko in T.Pipelined(K // block_K, num_stages=stage):
                T.copy(A[by * block_M, ko * block_K], A_shared)
                if not b_preshuffle:
                    if b_transposed:
                        T.copy(B[bx * block_N, ko * block_K], B_shared)
                    else:
                        T.copy(B[ko * block_K, bx * block_N], B_shared)
                for ki in T.unroll(chunk // pk):
                    emitter.ldmatrix_a(A_local, A_shared, ki, rk=rk)
                    if b_preshuffle:
                        emitter.ldmatrix_b(B_local, B, ko * (block_K // pk) + ki, pid_m=by, pid_n=bx)
                    else:
                        emitter.ldmatrix_b(B_local, B_shared, ki, rk=rk)
                    emitter.mfma(A_local, B_local, C_local)
            if reduce_k > 1:
                C_red = T.alloc_shared(emitter.reduce_k_scratch_shape(), accum_dtype)
                emitter.reduce_k_sum(C_local, C_red)
                if rk == 0:
                    emitter.stmatrix(C_local, C, pid_m=by, pid_n=bx)
            else:
                emitter.stmatrix(C_local, C, pid_m=by, pid_n=bx)

    return gemm_intrinsics


def ref_program(A, B, b_transposed=True):
    return A.float() @ (B.float().T if b_transposed else B.float())


def main(M=4096, N=4096, K=4096, in_dtype="float16", micro_size=32, b_preshuffle=False):
    import torch
    from tilelang.intrinsics import shuffle_weight
    out_dtype = "int32" if in_dtype == "int8" else "float16" if in_dtype == "float16" else "float32"
    accum = "int32" if in_dtype == "int8" else "float32"
    kernel = tl_matmul(M, N, K, in_dtype, out_dtype, accum, micro_size=micro_size, b_preshuffle=b_preshuffle)
    if in_dtype == "int8":
        a = torch.randint(-8, 8, (M, K), device="cuda", dtype=torch.int8)
        b = torch.randint(-8, 8, (N, K), device="cuda", dtype=torch.int8)
    else:
        tdt = getattr(torch, in_dtype)
        a = torch.randn(M, K, device="cuda").to(tdt)
        b = torch.randn(N, K, device="cuda").to(tdt)
    bk = b
    if b_preshuffle:
        pk = MatrixCoreIntrinEmitter(in_dtype, in_dtype, accum, micro_size=micro_size, chunk=256).micro_size_k
        bk = shuffle_weight(b, (micro_size, pk), is_transpose=True)
    c = kernel(a, bk)
    torch.testing.assert_close(c.float(), ref_program(a, b), rtol=1e-2, atol=1e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(a, bk))
    print(f"intrinsic-emitter GEMM {M}x{N}x{K} {in_dtype} mfma{micro_size} preshuffle={b_preshuffle}: {lat:.3f} ms, "
          f"{2 * M * N * K / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=4096)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--k", type=int, default=4096)
    p.add_argument("--dtype", default="float16")
    p.add_argument("--micro", type=int, default=32)
    p.add_argument("--preshuffle", action="store_true")
    a = p.parse_args()
    main(a.m, a.n, a.k, a.dtype, a.micro, a.preshuffle)
