"""MoE grouped GEMM with MXFP4 expert weights and bf16 activations
(reference: examples/dequantize_gemm/example_dequant_groupedgemm_bf16_mxfp4_hopper.py:43-330).

C[m, t, :] = topk_weight[m*topk+t] * (A[m] @ dequant(B[e])^T + Bias[e])  for every routed
(token m, slot t) pair, e its expert.  ``sorted_token_ids`` [padding_M] lists the (m*topk+t) pairs
grouped by expert, each group padded with -1 to a multiple of ``block_M``; ``expert_ids``
[padding_M / block_M] is the expert of every row block (the moe_align layout).  B [E, N, K/2]
holds two e2m1 codes per byte (low nibble = even k), Scale [E, N, K/32] the per-32 exponents:
w = e2m1 * 2^(Scale - scale_bias) (the reference's 2^Scale is scale_bias = 0; OCP e8m0 is 127).

MI355X schedule (one workgroup per (row block, N tile)):

* the token rows of a block are gathered straight from A with ``T.gather_rows`` (per-lane row
  addresses on the buffer LDS-DMA; padding rows resolve to an out-of-range index and read
  zeros) into the pipelined ring, next to the packed expert tile and its scales — the reference
  gathers A with per-thread 16-element register copies;
* the expert tile is expanded into a bf16 LDS tile by integer ops only: the e2m1 code and its
  exponent scale are assembled directly as bf16 bit patterns (no fp32 multiply, no table);
* bias is the accumulator's initial value, the router weight multiplies in the epilogue, and each
  valid row scatters to C[m, t] with a row-guarded store.

The reference's ``fast_dequant`` flag selects an NVIDIA bit-twiddled weight layout (LOP3
decode); this kernel consumes the plain nibble order, so that layout does not exist here.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[-1])
def matmul(M, N, K, topk, E, padding_M, in_dtype="bfloat16", out_dtype="bfloat16", accum_dtype="float32",
           num_bits=4, scale_size=32, scale_bias=0, with_bias=False, block_M=128, block_N=128, block_K=128,
           num_stages=2, threads=256):
    """Call as kernel(A, B, Scale, Bias, topk_weights, sorted_token_ids, expert_ids) -> C [M, topk, N]."""
    assert num_bits == 4 and scale_size == 32 and in_dtype == "bfloat16"
    assert K % block_K == 0 and block_K % scale_size == 0 and padding_M % block_M == 0
    QK = K // 2
    sc_off = 127 - scale_bias  # bf16 exponent field of 2^(s - scale_bias) * 2^(e - 1)

    @T.prim_func
    def main(A: T.Tensor((M, K), in_dtype), B: T.Tensor((E, N, QK), "uint8"),
             Scale: T.Tensor((E, N, K // scale_size), "uint8"), Bias: T.Tensor((E, N), out_dtype),
             topk_weights: T.Tensor((M * topk, ), out_dtype), sorted_token_ids: T.Tensor((padding_M, ), "int32"),
             expert_ids: T.Tensor((padding_M // block_M, ), "int32"), C: T.Tensor((M, topk, N), out_dtype)):
        with T.Kernel(T.ceildiv(N, block_N), padding_M // block_M, threads=threads) as (bx, by):
            A_s = T.alloc_shared((block_M, block_K), in_dtype)
            Bq_s = T.alloc_shared((block_N, block_K // 2), "uint8")
            S_s = T.alloc_shared((block_N, block_K // scale_size), "uint8")
            B_s = T.alloc_shared((block_N, block_K), in_dtype)
            rows = T.alloc_shared((block_M, ), "int32")
            ids = T.alloc_shared((block_M, ), "int32")
            C_local = T.alloc_fragment((block_M, block_N), accum_dtype)
            e = expert_ids[by]
            for i in T.Parallel(block_M):
                tid = sorted_token_ids[by * block_M + i]
                ids[i] = tid
                rows[i] = T.if_then_else(tid >= 0, tid // topk, -1)
            for i, j in T.Parallel(block_M, block_N):
                if with_bias:
                    C_local[i, j] = T.Cast(accum_dtype, Bias[e, bx * block_N + j])
                else:
                    C_local[i, j] = 0.0
            for k in T.Pipelined(K // block_K, num_stages=num_stages):
                T.gather_rows(A[:, k * block_K:(k + 1) * block_K], rows, A_s)
                T.copy(B[e, bx * block_N, k * (block_K // 2)], Bq_s)
                T.copy(Scale[e, bx * block_N, k * (block_K // scale_size)], S_s)
                for n, kk in T.Parallel(block_N, block_K):
                    nib = T.Cast("int32", (Bq_s[n, kk // 2] >> ((kk % 2) * 4)) & 15)
                    sc = T.Cast("int32", S_s[n, kk // scale_size]) + sc_off
                    ex = (nib >> 1) & 3
                    sgn = (nib & 8) << 12
                    bits = T.if_then_else(ex == 0, T.if_then_else((nib & 1) == 1, sgn | ((sc - 1) << 7), sgn),
                                          sgn | ((ex + sc - 1) << 7) | ((nib & 1) << 6))
                    B_s[n, kk] = T.reinterpret(T.Cast("uint16", bits), in_dtype)
                T.gemm(A_s, B_s, C_local, transpose_B=True)
            for i, j in T.Parallel(block_M, block_N):
                if ids[i] >= 0:
                    C[ids[i] // topk, ids[i] % topk, bx * block_N + j] = T.Cast(
                        out_dtype, C_local[i, j] * T.Cast(accum_dtype, topk_weights[ids[i]]))

    return main


def moe_align(tokens_experts, E, block_M):
    """(sorted_token_ids padded with -1 per expert to block_M, expert_ids per row block) — the
    reference's get_data layout (stable sort by expert)."""
    import torch
    vals, order = torch.sort(tokens_experts, stable=True)
    ids, eids = [], []
    for e in range(E):
        sel = order[vals == e]
        if sel.numel() == 0:
            continue
        pad = -(-sel.numel() // block_M) * block_M - sel.numel()
        ids.append(torch.cat([sel.int(), torch.full((pad, ), -1, dtype=torch.int32, device=sel.device)]))
        eids += [e] * (-(-sel.numel() // block_M))
    return torch.cat(ids), torch.tensor(eids, dtype=torch.int32, device=tokens_experts.device)


def get_data(m, n, k, scale_size, topk, E, block_M, device="cuda", scale_bias=0):
    import torch
    A = torch.empty(m, k, dtype=torch.bfloat16, device=device).uniform_(-1, 1)
    qB = torch.randint(0, 256, (E, n, k // 2), dtype=torch.uint8, device=device)
    Scale = torch.randint(scale_bias, scale_bias + 8, (E, n, k // scale_size), dtype=torch.uint8, device=device)
    Bias = torch.empty(E, n, dtype=torch.bfloat16, device=device).uniform_(-1, 1)
    weights = torch.empty(m, E, dtype=torch.bfloat16, device=device).uniform_(-1, 1)
    topk_weights, tokens_experts = torch.topk(weights, topk, dim=-1)
    topk_weights = (topk_weights / topk_weights.sum(dim=-1, keepdim=True)).reshape(m * topk)
    sorted_token_ids, expert_ids = moe_align(tokens_experts.reshape(m * topk), E, block_M)
    return A, qB, Scale, Bias, topk_weights, sorted_token_ids, expert_ids, sorted_token_ids.numel()


def dequant_ref(qB, Scale, scale_bias=0):
    """[E, N, K/2] e2m1 pairs + [E, N, K/32] exponents -> fp32 [E, N, K]."""
    import torch
    from tilelang.quantize import e2m1_to_float_torch
    lo, hi = (qB & 15).long(), (qB >> 4).long()
    codes = torch.stack([lo, hi], -1).flatten(-2)
    w = e2m1_to_float_torch(codes)
    return w * torch.exp2(Scale.float() - scale_bias).repeat_interleave(32, -1)


def ref_moe(A, qB, Scale, Bias, topk_weights, sorted_token_ids, expert_ids, block_M, with_bias=False, scale_bias=0):
    import torch
    M, K = A.shape
    E, N, _ = qB.shape
    topk = topk_weights.shape[0] // M
    W = dequant_ref(qB, Scale, scale_bias)
    C = torch.zeros(M, topk, N, device=A.device)
    ids = sorted_token_ids.tolist()
    eids = expert_ids.tolist()
    for r, t in enumerate(ids):
        if t < 0:
            continue
        e = eids[r // block_M]
        out = A[t // topk].float() @ W[e].t()
        if with_bias:
            out = out + Bias[e].float()
        C[t // topk, t % topk] = out * topk_weights[t].float()
    return C


def main(m=256, n=256, k=256, scale_size=32, topk=4, E=32, with_bias=False, block_M=128):
    import torch
    A, qB, Scale, Bias, tw, sids, eids, padding_M = get_data(m, n, k, scale_size, topk, E, block_M)
    kernel = matmul(m, n, k, topk, E, padding_M, with_bias=with_bias, block_M=block_M)
    out = kernel(A, qB, Scale, Bias, tw, sids, eids)
    ref = ref_moe(A, qB, Scale, Bias, tw, sids, eids, block_M, with_bias)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
    print("All checks pass.")
    lat = tilelang.profiler.do_bench(lambda: kernel(A, qB, Scale, Bias, tw, sids, eids))
    print(f"grouped bf16 x mxfp4 m{m} n{n} k{k} topk{topk} E{E}: {lat:.4f} ms, "
          f"{2 * m * n * k * topk / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--m", type=int, default=256)
    p.add_argument("--n", type=int, default=256)
    p.add_argument("--k", type=int, default=256)
    p.add_argument("--topk", type=int, default=4)
    p.add_argument("--E", type=int, default=32)
    p.add_argument("--with_bias", action="store_true")
    a = p.parse_args()
    main(a.m, a.n, a.k, 32, a.topk, a.E, a.with_bias)
