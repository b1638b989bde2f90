"""fp16 x int4 GEMV / skinny GEMM for decode (reference:
examples/dequantize_gemm/example_dequant_gemv_fp16xint4.py:11-155).

C[M, N] = A[M, K] @ dequant(B)^T for small M (decode batch).  B [N, K/2] uint8 packs two
nibbles per byte (low nibble = even k); ``source_format`` "uint" reads them as 0..15 (the
reference's default), "int" as two's complement -8..7; ``with_scaling`` multiplies group-wise
scales Scale [N, K/group_size].

Decode GEMV is HBM-bound on the weights (0.5 byte per MAC), so the schedule streams B at full
bandwidth and never stages it through LDS: each workgroup owns ``block_N`` rows for all M
activations, every lane reads 16 packed bytes (32 weights) of a row per step with one vector
load, decodes the nibbles in registers (bitfield extract, optional sign fix, one convert),
multiplies by the L2-resident activation slice with fp32 accumulation, and one cross-lane
reduction per (row, m) finishes.  The reference's ``fast_decoding`` (an NVIDIA LOP3 weight
interleave) has no counterpart: the plain nibble order decodes with the same VALU count here.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def dequantize_gemv(M, N, K, in_dtype="float16", out_dtype="float16", accum_dtype="float", source_format="uint",
                    group_size=-1, with_scaling=False, block_N=8, block_K=1024, threads=256):
    """Call as kernel(A, B[, Scale]) -> C."""
    assert source_format in ("uint", "int")
    if group_size == -1:
        group_size = K
    assert K % block_K == 0 and K % group_size == 0
    KB = block_K // 2

    def decode(byte, hi):
        nib = T.Cast("int32", (byte >> (hi * 4)) & 15)
        if source_format == "int":
            nib = nib - ((nib & 8) << 1)
        return T.Cast(accum_dtype, nib)

    @T.macro
    def body(A, B, Scale, C):
        with T.Kernel(T.ceildiv(N, block_N), threads=threads) as bn:
            b_frag = T.alloc_fragment((block_N, KB), "uint8")
            acc = T.alloc_fragment((M, block_N, KB), accum_dtype)
            row = T.alloc_fragment((M, block_N), accum_dtype)
            T.clear(acc)
            for ko in T.serial(K // block_K):
                T.copy(B[bn * block_N, ko * KB], b_frag)
                for mi, i, j in T.Parallel(M, block_N, KB):
                    k0 = ko * block_K + 2 * j
                    w0 = decode(b_frag[i, j], 0)
                    w1 = decode(b_frag[i, j], 1)
                    if with_scaling:
                        s = T.Cast(accum_dtype, Scale[bn * block_N + i, k0 // group_size])
                        w0 = w0 * s
                        w1 = w1 * s
                    acc[mi, i, j] += w0 * T.Cast(accum_dtype, A[mi, k0]) + w1 * T.Cast(accum_dtype, A[mi, k0 + 1])
            T.reduce_sum(acc, row, dim=2)
            for mi, i in T.Parallel(M, block_N):
                if bn * block_N + i < N:
                    C[mi, bn * block_N + i] = T.Cast(out_dtype, row[mi, i])

    if with_scaling:

        @T.prim_func
        def main(A: T.Tensor((M, K), in_dtype), B: T.Tensor((N, K // 2), "uint8"),
                 Scale: T.Tensor((N, K // group_size), in_dtype), C: T.Tensor((M, N), out_dtype)):
            body(A, B, Scale, C)
    else:

        @T.prim_func
        def main(A: T.Tensor((M, K), in_dtype), B: T.Tensor((N, K // 2), "uint8"), C: T.Tensor((M, N), out_dtype)):
            body(A, B, None, C)

    return main


def dequant_ref(qB, source_format="uint", scale=None, group_size=-1):
    import torch
    lo, hi = (qB & 15).to(torch.int16), (qB >> 4).to(torch.int16)
    w = torch.stack([lo, hi], -1).flatten(-2)
    if source_format == "int":
        w = w - ((w & 8) << 1)
    w = w.float()
    if scale is not None:
        gs = w.shape[1] if group_size == -1 else group_size
        w = w * scale.float().repeat_interleave(gs, -1)
    return w


def ref_program(A, qB, source_format="uint", scale=None, group_size=-1):
    return A.float() @ dequant_ref(qB, source_format, scale, group_size).t()


def main(M=1, N=16384, K=16384, source_format="int", with_scaling=True, group_size=128):
    import torch
    kernel = dequantize_gemv(M, N, K, source_format=source_format, group_size=group_size, with_scaling=with_scaling)
    A = torch.randn(M, K, device="cuda", dtype=torch.float16)
    qB = torch.randint(0, 256, (N, K // 2), dtype=torch.uint8, device="cuda")
    args = [A, qB]
    scale = None
    if with_scaling:
        scale = (torch.rand(N, K // group_size, device="cuda") * 0.02).half()
        args.append(scale)
    C = kernel(*args)
    ref = ref_program(A, qB, source_format, scale, group_size)
    torch.testing.assert_close(C.float(), ref, rtol=1e-2, atol=1e-2 * float(ref.abs().max()))
    print("All checks pass.")
    lat = tilelang.profiler.do_bench(lambda: kernel(*args))
    nbytes = N * K // 2 + (scale.numel() * 2 if with_scaling else 0)
    print(f"fp16 x int4 gemv M{M} N{N} K{K}: {lat * 1e3:.1f} us, {nbytes / lat * 1e-6:.0f} GB/s weight stream")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=1)
    p.add_argument("--n", type=int, default=16384)
    p.add_argument("--k", type=int, default=16384)
    a = p.parse_args()
    main(a.m, a.n, a.k)
