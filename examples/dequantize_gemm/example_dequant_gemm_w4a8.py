"""W4A8 GEMM: int8 activations x signed int4 weights, int32 accumulation
(reference: examples/dequantize_gemm/example_dequant_gemm_w4a8.py:92-160).

Ct[N, M] = dequant(B)[N, K] @ A[M, K]^T in int32 (the reference's transposed output), A int8,
B [N, K/2] uint8 with two two's-complement nibbles per byte (low nibble = even k).

MI355X schedule: the packed weight tile (half the bytes of an int8 tile) and the int8
activation tile stream through the LDS-DMA ring; the waves sign-extend the nibbles into an int8
LDS tile (shift left 4, arithmetic shift right 4 — two VALU ops per value, no table) and the
tile GEMM runs on ``v_mfma_i32_16x16x64_i8`` (gfx950's int8 rate is the fp8 rate, 2x bf16),
exact integer accumulation.  The weights sit on the MFMA M side (Ct = B A^T), so for decode-sized
M the N dimension spreads over the workgroups.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[2])
def matmul_int8xint4(M, N, K, block_M=128, block_N=128, block_K=128, num_stages=2, threads=256):
    assert K % block_K == 0

    @T.prim_func
    def main(A: T.Tensor((M, K), "int8"), B: T.Tensor((N, K // 2), "uint8"), Ct: T.Tensor((N, M), "int32")):
        with T.Kernel(T.ceildiv(M, block_M), T.ceildiv(N, block_N), threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, block_K), "int8")
            Bq_s = T.alloc_shared((block_N, block_K // 2), "uint8")
            B_s = T.alloc_shared((block_N, block_K), "int8")
            Ct_local = T.alloc_fragment((block_N, block_M), "int32")
            T.use_swizzle(panel_size=8)
            T.clear(Ct_local)
            for k in T.Pipelined(K // block_K, num_stages=num_stages):
                T.copy(A[bx * block_M, k * block_K], A_s)
                T.copy(B[by * block_N, k * (block_K // 2)], Bq_s)
                for n, kk in T.Parallel(block_N, block_K):
                    nib = T.Cast("int32", (Bq_s[n, kk // 2] >> ((kk % 2) * 4)) & 15)
                    B_s[n, kk] = T.Cast("int8", nib - ((nib & 8) << 1))
                T.gemm(B_s, A_s, Ct_local, transpose_B=True)
            T.copy(Ct_local, Ct[by * block_N, bx * block_M])

    return main


def unpack_int4(qB):
    """[N, K/2] uint8 -> [N, K] int8 (signed nibbles, low nibble first)."""
    import torch
    lo = (qB & 15).to(torch.int16)
    hi = (qB >> 4).to(torch.int16)
    v = torch.stack([lo, hi], -1).flatten(-2)
    return (v - ((v & 8) << 1)).to(torch.int8)


def ref_program(A, qB):
    B = unpack_int4(qB)
    return (B.double() @ A.double().t()).to(dtype=__import__("torch").int32)


def main(m=512, n=4096, k=4096):
    import torch
    kernel = matmul_int8xint4(m, n, k)
    A = torch.randint(-128, 128, (m, k), dtype=torch.int8, device="cuda")
    qB = torch.randint(0, 256, (n, k // 2), dtype=torch.uint8, device="cuda")
    Ct = kernel(A, qB)
    torch.testing.assert_close(Ct, ref_program(A, qB), rtol=0, atol=0)
    print("All checks pass.")
    lat = tilelang.profiler.do_bench(lambda: kernel(A, qB))
    print(f"w4a8 {m}x{n}x{k}: {lat:.4f} ms, {2 * m * n * k / lat * 1e-9:.1f} TOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=512)
    p.add_argument("--n", type=int, default=4096)
    p.add_argument("--k", type=int, default=4096)
    a = p.parse_args()
    main(a.m, a.n, a.k)
