"""Grouped GEMM (MoE expert FFN building block) on MI355X.

Reference: ``examples/grouped_gemm/example_grouped_gemm_fwd.py`` — A ``[sum(m_g), K]`` holds
the tokens of every group back to back, B ``[G, K, N]`` (or ``[G, N, K]`` with ``trans_b``)
one weight per group; grid = (sum of per-group M tiles, N tiles); each tile finds its group
from the padded tile offsets.

MI355X schedule: both operand tiles stream through the LDS-DMA pipeline even though the row
offset and the group id are data dependent — leaving the tensor along its outer dim is caught
by the buffer resource's hardware bound check (zero fill), so no register staging; MFMA
16x16x32 with a 256-thread block; the tail rows of a group are masked in the epilogue.
"""
import argparse
import math

import torch

import tilelang
import tilelang.language as T


def torch_gmm(a, b, batch_sizes, trans_b=False):
    out = torch.empty((a.shape[0], b.shape[1] if trans_b else b.shape[2]), device=a.device, dtype=a.dtype)
    start = 0
    for i, size in enumerate(batch_sizes):
        end = start + int(size)
        w = b[i].transpose(0, 1) if trans_b else b[i]
        out[start:end] = (a[start:end].float() @ w.float()).to(a.dtype)
        start = end
    return out


@tilelang.jit(out_idx=[2])
def grouped_gemm(batch_sizes_list, K, N, block_M=128, block_N=128, block_K=64, num_stages=2, threads=256,
                 dtype="float16", trans_b=False):
    batch_sum = sum(batch_sizes_list)
    batch_count = len(batch_sizes_list)
    accum_dtype = "float32"
    total_m_blocks = sum((s + block_M - 1) // block_M for s in batch_sizes_list)
    b_shape = [batch_count, N, K] if trans_b else [batch_count, K, N]
    bs_shape = [block_N, block_K] if trans_b else [block_K, block_N]

    @T.prim_func
    def kernel(A: T.Tensor([batch_sum, K], dtype), B: T.Tensor(b_shape, dtype), C: T.Tensor([batch_sum, N], dtype),
               batch_sizes: T.Tensor([batch_count], "int32"), batch_offsets: T.Tensor([batch_count], "int32"),
               batch_padded_offsets: T.Tensor([batch_count], "int32")):
        with T.Kernel(total_m_blocks, T.ceildiv(N, block_N), threads=threads) as (bx, by):
            A_shared = T.alloc_shared([block_M, block_K], dtype)
            B_shared = T.alloc_shared(bs_shape, dtype)
            C_local = T.alloc_fragment([block_M, block_N], accum_dtype)
            g = T.alloc_var("int32")
            m_start_padded = bx * block_M
            g = 0
            for i in T.unroll(batch_count):
                if m_start_padded >= batch_padded_offsets[i]:
                    g = i
            m_start = m_start_padded - batch_padded_offsets[g] + batch_offsets[g]
            actual_rows = T.max(0, T.min(block_M, batch_sizes[g] + batch_padded_offsets[g] - m_start_padded))
            T.clear(C_local)
            for k in T.Pipelined(T.ceildiv(K, block_K), num_stages=num_stages):
                T.copy(A[m_start, k * block_K], A_shared)
                if trans_b:
                    T.copy(B[g, by * block_N, k * block_K], B_shared)
                else:
                    T.copy(B[g, k * block_K, by * block_N], B_shared)
                T.gemm(A_shared, B_shared, C_local, transpose_B=trans_b)
            for i, j in T.Parallel(block_M, block_N):
                if i < actual_rows:
                    C[m_start + i, by * block_N + j] = C_local[i, j]

    return kernel


def construct_inputs(batch_sizes_list, K, N, trans_b, padding_M, device="cuda", dtype=torch.float16):
    batch_sum = sum(batch_sizes_list)
    G = len(batch_sizes_list)
    offs = [0]
    padded = [0]
    for i in range(G - 1):
        offs.append(offs[-1] + batch_sizes_list[i])
        padded.append(padded[-1] + math.ceil(batch_sizes_list[i] / padding_M) * padding_M)
    A = torch.randn(batch_sum, K, device=device, dtype=dtype)
    B = torch.randn(G, N, K, device=device, dtype=dtype) if trans_b else torch.randn(G, K, N, device=device,
                                                                                   dtype=dtype)
    mk = lambda x: torch.tensor(x, device=device, dtype=torch.int32)  # noqa: E731
    return A, B, mk(batch_sizes_list), mk(offs), mk(padded)


def run(batch_sizes_list, K, N, block_M=128, block_N=128, block_K=64, trans_b=False, num_stages=2, threads=256,
        profile=False):
    kernel = grouped_gemm(tuple(batch_sizes_list), K, N, block_M, block_N, block_K, num_stages, threads,
                          "float16", trans_b)
    A, B, bs, bo, bpo = construct_inputs(batch_sizes_list, K, N, trans_b, block_M)
    out = kernel(A, B, bs, bo, bpo)
    ref = torch_gmm(A, B, batch_sizes_list, trans_b)
    torch.testing.assert_close(out, ref, rtol=1e-2, atol=1e-2)
    if profile:
        from tilelang.profiler import do_bench
        ms = do_bench(lambda: kernel(A, B, bs, bo, bpo), warmup=50, rep=200)
        tf = 2 * sum(batch_sizes_list) * K * N / ms * 1e-9
        print(f"grouped gemm {batch_sizes_list} K={K} N={N}: {ms:.4f} ms  {tf:.1f} TFLOPS")
        return tf
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_sizes", type=str, default="64,128")
    ap.add_argument("--K", type=int, default=8192)
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--trans_b", action="store_true")
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    run([int(x) for x in a.batch_sizes.split(",")], a.K, a.M, trans_b=a.trans_b, profile=a.profile)
    print("ok")
