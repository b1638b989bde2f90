"""Weight-only int4 GEMM (W4A16) with group-wise scales
(reference: examples/dequantize_gemm/example_dequant_gemm_fine_grained.py,
example_dequant_gemv_fp16xint4.py, tilelang/quantize/quantization.py).

C[M, N] = A[M, K] (fp16/bf16) @ dequant(Bq)^T where Bq is [N, K/2] uint8 holding two signed
int4 values per byte (low nibble = even k) and ``Scales`` is [N, K/group] in the activation
dtype: w = int4 * scale.  MI355X schedule: the packed tile (half the bytes of an fp16 tile)
streams through the LDS-DMA ring; each step the waves expand it in registers (nibble extract,
sign extend, scale) into an fp16 LDS tile laid out for the MFMA B reads, then run the
16x16x32 MFMAs -- HBM traffic for B is 4x smaller than fp16 weights, which is what matters for
the small-M (decode) shapes this kernel serves.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def dequant_gemm_w4a16(M, N, K, group_size=128, block_M=64, block_N=128, block_K=64, threads=256, num_stages=2,
                       dtype="float16", accum_dtype="float", unroll=2):
    """``unroll``: the K loop emitted twice per trip (constant LDS ring slots): 16x8192x8192
    0.269 -> 0.205 ms (profiles/r6/unroll_sweep_examples.log)."""
    assert K % group_size == 0 and group_size % block_K == 0 and block_K % 2 == 0

    @T.prim_func
    def main(A: T.Tensor((M, K), dtype), Bq: T.Tensor((N, K // 2), "uint8"),
             Scales: T.Tensor((N, K // group_size), dtype), C: T.Tensor((M, N), dtype)):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(M, block_M), threads=threads) as (bx, by):
            A_shared = T.alloc_shared((block_M, block_K), dtype)
            Bq_shared = T.alloc_shared((block_N, block_K // 2), "uint8")
            B_shared = T.alloc_shared((block_N, block_K), dtype)
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            C_cast = T.alloc_fragment((block_M, block_N), dtype)
            T.use_swizzle(panel_size=8)
            T.clear(C_local)
            for k in T.Pipelined(K // block_K, num_stages=num_stages, unroll=unroll):
                T.copy(A[by * block_M, k * block_K], A_shared)
                T.copy(Bq[bx * block_N, k * (block_K // 2)], Bq_shared)
                for n, kk in T.Parallel(block_N, block_K):
                    byte = Bq_shared[n, kk // 2]
                    nib = (byte >> ((kk % 2) * 4)) & 15
                    q = T.Cast("int32", nib) - T.if_then_else(nib >= 8, 16, 0)
                    B_shared[n, kk] = T.Cast(dtype, T.Cast("float32", q) * T.Cast(
                        "float32", Scales[bx * block_N + n, (k * block_K + kk) // group_size]))
                T.gemm(A_shared, B_shared, C_local, transpose_B=True)
            T.copy(C_local, C_cast)
            T.copy(C_cast, C[by * block_M, bx * block_N])

    return main


def quantize_int4(W, group_size=128):
    """W [N, K] float -> (Bq [N, K/2] uint8, scales [N, K/group]) with symmetric int4."""
    import torch
    N, K = W.shape
    g = W.float().view(N, K // group_size, group_size)
    scales = (g.abs().amax(-1) / 7.0).clamp(min=1e-8)
    q = torch.clamp(torch.round(g / scales.unsqueeze(-1)), -8, 7).to(torch.int32).view(N, K)
    u = (q & 0xF).to(torch.uint8)
    packed = u[:, 0::2] | (u[:, 1::2] << 4)
    return packed.contiguous(), scales.to(W.dtype)


def dequantize_int4(Bq, scales, group_size=128):
    import torch
    lo = (Bq & 0xF).to(torch.int32)
    hi = (Bq >> 4).to(torch.int32)
    q = torch.stack([lo, hi], -1).view(Bq.shape[0], -1)
    q = q - (q >= 8).to(torch.int32) * 16
    N, K = q.shape
    return (q.float().view(N, K // group_size, group_size) * scales.float().unsqueeze(-1)).view(N, K)


def ref_program(A, Bq, scales, group_size=128):
    return (A.float() @ dequantize_int4(Bq, scales, group_size).t()).to(A.dtype)


def main(M=16, N=8192, K=8192):
    import torch
    kernel = dequant_gemm_w4a16(M, N, K)
    A = torch.randn(M, K, device="cuda", dtype=torch.float16)
    W = torch.randn(N, K, device="cuda", dtype=torch.float16)
    Bq, s = quantize_int4(W)
    c = kernel(A, Bq, s)
    torch.testing.assert_close(c.float(), ref_program(A, Bq, s).float(), rtol=1e-2, atol=5e-1)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(A, Bq, s))
    print(f"w4a16 GEMM {M}x{N}x{K}: {lat:.4f} ms, {2 * M * N * K / lat * 1e-9:.1f} TFLOPS, "
          f"{(N * K // 2 + M * K * 2) / lat * 1e-6:.1f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=16)
    p.add_argument("--n", type=int, default=8192)
    p.add_argument("--k", type=int, default=8192)
    a = p.parse_args()
    main(a.m, a.n, a.k)
