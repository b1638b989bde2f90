"""Grouped GEMM backward + autograd (reference: examples/grouped_gemm/example_grouped_gemm_bwd.py).

Forward C_g = A_g B_g (A [sum m_g, K], B [G, K, N]).  Backward:
* dA_g = dC_g B_g^T -- the forward kernel with ``trans_b`` (B read as [G, N, K]);
* dB_g = A_g^T dC_g -- one block per (group, K tile, N tile) reduces over the group's rows:
  full ``block_R``-row tiles stream through the LDS-DMA pipeline (A tile read transposed by
  the MFMA operand load), the ragged last tile is loaded with row masks into separate tiles so
  no row of the next group leaks in.
"""
import argparse

import torch

import tilelang
import tilelang.language as T
from example_grouped_gemm_fwd import construct_inputs, grouped_gemm


@tilelang.jit(out_idx=[2])
def grouped_gemm_dw(batch_sizes_list, K, N, block_K=128, block_N=128, block_R=64, num_stages=2, threads=256,
                    dtype="float16"):
    """dB[g] = A_g^T dC_g, A [sum m, K], dC [sum m, N] -> dB [G, K, N] (fp32 accumulation)."""
    batch_sum = sum(batch_sizes_list)
    G = len(batch_sizes_list)
    accum_dtype = "float32"

    @T.prim_func
    def kernel(A: T.Tensor([batch_sum, K], dtype), dC: T.Tensor([batch_sum, N], dtype), dB: T.Tensor([G, K, N], dtype),
               batch_sizes: T.Tensor([G], "int32"), batch_offsets: T.Tensor([G], "int32")):
        with T.Kernel(T.ceildiv(N, block_N), T.ceildiv(K, block_K), G, threads=threads) as (bn, bk, g):
            A_s = T.alloc_shared([block_R, block_K], dtype)
            C_s = T.alloc_shared([block_R, block_N], dtype)
            At_s = T.alloc_shared([block_R, block_K], dtype)
            Ct_s = T.alloc_shared([block_R, block_N], dtype)
            acc = T.alloc_fragment([block_K, block_N], accum_dtype)
            out = T.alloc_fragment([block_K, block_N], dtype)
            size = batch_sizes[g]
            start = batch_offsets[g]
            n_full = size // block_R
            T.clear(acc)
            for r in T.Pipelined(n_full, num_stages=num_stages):
                T.copy(A[start + r * block_R, bk * block_K], A_s)
                T.copy(dC[start + r * block_R, bn * block_N], C_s)
                T.gemm(A_s, C_s, acc, transpose_A=True)
            if size % block_R != 0:
                r0 = start + n_full * block_R
                for i, j in T.Parallel(block_R, block_K):
                    At_s[i, j] = T.if_then_else(r0 + i < start + size, A[r0 + i, bk * block_K + j], 0)
                for i, j in T.Parallel(block_R, block_N):
                    Ct_s[i, j] = T.if_then_else(r0 + i < start + size, dC[r0 + i, bn * block_N + j], 0)
                T.gemm(At_s, Ct_s, acc, transpose_A=True)
            T.copy(acc, out)
            T.copy(out, dB[g, bk * block_K, bn * block_N])

    return kernel


class GroupedGEMM(torch.autograd.Function):
    """C = grouped_gemm(A, B) with tilelang kernels for forward, dA and dB."""

    @staticmethod
    def forward(ctx, a, b, batch_sizes_list, bs, bo, bpo, block_M):
        K, N = b.shape[1], b.shape[2]
        ctx.save_for_backward(a, b, bs, bo, bpo)
        ctx.cfg = (tuple(batch_sizes_list), block_M)
        return grouped_gemm(tuple(batch_sizes_list), K, N, block_M)(a, b, bs, bo, bpo)

    @staticmethod
    def backward(ctx, dc):
        a, b, bs, bo, bpo = ctx.saved_tensors
        sizes, block_M = ctx.cfg
        K, N = b.shape[1], b.shape[2]
        dc = dc.contiguous()
        da = grouped_gemm(sizes, N, K, block_M, trans_b=True)(dc, b, bs, bo, bpo)  # dC B^T, B as [G, K, N]
        db = grouped_gemm_dw(sizes, K, N)(a, dc, bs, bo)
        return da, db, None, None, None, None, None


def main(batch_sizes=(64, 300, 1024, 17), K=1024, N=2048):
    a, b, bs, bo, bpo = construct_inputs(list(batch_sizes), K, N, False, 128)
    a.requires_grad_()
    b.requires_grad_()
    c = GroupedGEMM.apply(a, b, list(batch_sizes), bs, bo, bpo, 128)
    dc = torch.randn_like(c)
    c.backward(dc)
    ga, gb = a.grad.clone(), b.grad.clone()
    a.grad = b.grad = None
    ref = torch.cat([a[s:s + n].float() @ b[i].float() for i, (s, n) in
                     enumerate(zip(bo.tolist(), batch_sizes))])
    ref.backward(dc.float())
    torch.testing.assert_close(c.float(), ref.detach(), rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(ga.float(), a.grad.float(), rtol=2e-2, atol=2e-1)
    torch.testing.assert_close(gb.float(), b.grad.float(), rtol=2e-2, atol=5e-1)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    kd = grouped_gemm_dw(tuple(batch_sizes), K, N)
    ms = do_bench(lambda: kd(a, dc, bs, bo))
    tf = 2 * sum(batch_sizes) * K * N / ms * 1e-9
    print(f"grouped dW {list(batch_sizes)} K={K} N={N}: {ms:.4f} ms, {tf:.1f} TFLOPS")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_sizes", type=str, default="64,300,1024,17")
    a = ap.parse_args()
    main(tuple(int(x) for x in a.batch_sizes.split(",")))
