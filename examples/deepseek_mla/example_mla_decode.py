"""DeepSeek MLA decode with split-KV (reference: examples/deepseek_mla/amd/benchmark_mla_decode_amd_tilelang.py).

Q [b, h, 512] + Q_pe [b, h, 64] attend to a shared latent KV cache [b, s, 1, 512] + K_pe
[b, s, 1, 64].  Each block owns ``block_H`` heads of one batch element and one KV split;
the latent tile KV_shared is read twice per step — row-wise for S = Q KV^T and transposed
(``ds_read_b64_tr_b16``) for O += P KV — so its LDS swizzle is chosen against both read
patterns.  A second kernel of the same program combines the splits with their LSEs.
"""
import argparse

import tilelang
import tilelang.language as T


@tilelang.jit(out_idx=[6], pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def mla_decode(batch, heads, kv_head_num, seqlen_kv, dim, pe_dim, block_N=64, block_H=64, num_split=4,
               threads=None, num_stages=2, dtype="float16", wide=None, sum_mfma=None):
    """``wide`` (default for 64-head blocks): 8 waves, S on a 4x2 wave grid, P through LDS and
    O = P KV split over the 512 latent columns (see tilelang/ops/dsa.py sparse_mla_fwd).
    ``sum_mfma`` (wide): the softmax row sums come from the matrix cores -- P (already in LDS for
    P KV) times a ones tile accumulates next to O and is rescaled with it -- instead of a per-tile
    cross-wave reduction through LDS (its barrier and shuffles leave the loop): b128 h128 kv8192
    727 -> 756 TF (default with ``wide``; profiles/r6/mla_sum_mfma_ab.log)."""
    if wide is None:
        wide = block_H == 64
    if sum_mfma is None:
        sum_mfma = wide
    if threads is None:
        threads = 512 if wide else 256
    s_policy = T.GemmWarpPolicy.Square if wide else T.GemmWarpPolicy.FullRow
    scale = (1.0 / (dim + pe_dim))**0.5 * 1.44269504  # softmax in base 2
    accum_dtype = "float"
    kv_group_num = heads // kv_head_num
    VALID_BLOCK_H = min(block_H, kv_group_num)
    assert kv_head_num == 1, "MLA decode expects one latent KV head"
    split_len = seqlen_kv // num_split

    @T.macro
    def attention_split(Q, Q_pe, KV, K_pe, glse, Output_partial):
        with T.Kernel(batch, heads // VALID_BLOCK_H, num_split, threads=threads) as (bx, by, bz):
            Q_local = T.alloc_fragment([block_H, dim], dtype)
            Q_pe_local = T.alloc_fragment([block_H, pe_dim], dtype)
            KV_shared = T.alloc_shared([block_N, dim], dtype)
            K_pe_shared = T.alloc_shared([block_N, pe_dim], dtype)
            acc_s = T.alloc_fragment([block_H, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_H, block_N], dtype)
            P_shared = T.alloc_shared([block_H, block_N], dtype)
            sc_shared = T.alloc_shared([block_H], accum_dtype)
            acc_o = T.alloc_fragment([block_H, dim], accum_dtype)
            scores_max = T.alloc_fragment([block_H], accum_dtype)
            scores_max_prev = T.alloc_fragment([block_H], accum_dtype)
            scores_scale = T.alloc_fragment([block_H], accum_dtype)
            scores_sum = T.alloc_fragment([block_H], accum_dtype)
            logsum = T.alloc_fragment([block_H], accum_dtype)

            T.copy(Q[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, :], Q_local)
            T.copy(Q_pe[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, :], Q_pe_local)
            any_s = T.alloc_shared([2], "int32")
            use_sm = wide and sum_mfma
            if use_sm:
                ones_s = T.alloc_shared([block_N, 32], dtype)
                acc_l = T.alloc_fragment([block_H, 32], accum_dtype)
                T.fill(ones_s, 1.0)
                T.clear(acc_l)
            T.fill(acc_o, 0)
            T.fill(logsum, 0)
            # wide: lazy rescale (a row keeps its max until a score beats it by 2^8, P <= 256), so
            # the D-split O accumulator is rescaled only on tiles where some row moved (flag in LDS)
            T.fill(scores_max, -(2.0**30) if wide else -T.infinity(accum_dtype))

            # lazy-rescale flag, double-buffered by iteration parity: iteration t resets the slot
            # of t + 1 (ordered by the stage barrier against t - 1's readers and t + 1's setters)
            for z in T.Parallel(2):
                any_s[z] = 0
            for k in T.Pipelined(T.ceildiv(split_len, block_N), num_stages=num_stages):
                kv_start = split_len * bz + k * block_N
                T.copy(KV[bx, kv_start:kv_start + block_N, 0, :], KV_shared)
                T.copy(K_pe[bx, kv_start:kv_start + block_N, 0, :], K_pe_shared)
                T.clear(acc_s)
                T.gemm(Q_local, KV_shared, acc_s, transpose_B=True, policy=s_policy)
                T.gemm(Q_pe_local, K_pe_shared, acc_s, transpose_B=True, policy=s_policy)
                if wide:
                    for z in T.Parallel(1):  # previous tile's readers are past the stage barrier
                        any_s[z + (k + 1) % 2] = 0
                    T.copy(scores_max, scores_max_prev)
                    T.reduce_max(acc_s, scores_max_prev, dim=1, clear=False)  # candidate max
                    for i in T.Parallel(block_H):
                        if (scores_max_prev[i] - scores_max[i]) * scale > 8.0:
                            scores_scale[i] = T.exp2((scores_max[i] - scores_max_prev[i]) * scale)
                            scores_max[i] = scores_max_prev[i]
                            any_s[k % 2] = 1
                        else:
                            scores_scale[i] = 1.0
                else:
                    T.copy(scores_max, scores_max_prev)
                    T.reduce_max(acc_s, scores_max, dim=1, clear=False)
                    for i in T.Parallel(block_H):
                        scores_scale[i] = T.exp2(scores_max_prev[i] * scale - scores_max[i] * scale)
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.exp2(acc_s[i, j] * scale - scores_max[i] * scale)
                if not use_sm:
                    T.reduce_sum(acc_s, scores_sum, dim=1)
                    for i in T.Parallel(block_H):
                        logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                if wide:
                    T.copy(scores_scale, sc_shared)
                    T.copy(acc_s, P_shared)
                    if any_s[k % 2] != 0:
                        for i, j in T.Parallel(block_H, dim):
                            acc_o[i, j] *= sc_shared[i]
                        if use_sm:
                            for i, j in T.Parallel(block_H, 32):
                                acc_l[i, j] *= sc_shared[i]
                    T.gemm(P_shared, KV_shared, acc_o)
                    if use_sm:
                        T.gemm(P_shared, ones_s, acc_l)
                else:
                    T.copy(acc_s, acc_s_cast)
                    for i, j in T.Parallel(block_H, dim):
                        acc_o[i, j] *= scores_scale[i]
                    T.gemm(acc_s_cast, KV_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            if use_sm:
                for i, j in T.Parallel(block_H, 32):  # every column of P x ones is the row sum
                    if j == 0:
                        sc_shared[i] = acc_l[i, j]
                for i in T.Parallel(block_H):
                    logsum[i] = sc_shared[i]
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] /= sc_shared[i]
            elif wide:
                T.copy(logsum, sc_shared)
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] /= sc_shared[i]
            else:
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] /= logsum[i]
            for i in T.Parallel(block_H):
                logsum[i] = T.log2(logsum[i]) + scores_max[i] * scale
            T.copy(logsum, glse[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, bz])
            T.copy(acc_o, Output_partial[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, bz, :])

    @T.macro
    def combine(glse, Output_partial, Output):
        with T.Kernel(heads, batch, threads=128) as (hy, bz):
            o_acc = T.alloc_fragment([dim], accum_dtype)
            lse_max = T.alloc_local([1], accum_dtype)
            lse_sum = T.alloc_local([1], accum_dtype)
            sc = T.alloc_local([1], accum_dtype)
            T.clear(o_acc)
            lse_max[0] = -T.infinity(accum_dtype)
            for k in T.serial(num_split):
                lse_max[0] = T.max(lse_max[0], T.Cast(accum_dtype, glse[bz, hy, k]))
            lse_sum[0] = 0.0
            for k in T.serial(num_split):
                lse_sum[0] += T.exp2(T.Cast(accum_dtype, glse[bz, hy, k]) - lse_max[0])
            lse_sum[0] = T.log2(lse_sum[0]) + lse_max[0]
            for k in T.serial(num_split):
                sc[0] = T.exp2(T.Cast(accum_dtype, glse[bz, hy, k]) - lse_sum[0])
                for i in T.Parallel(dim):
                    o_acc[i] += Output_partial[bz, hy, k, i] * sc[0]
            for i in T.Parallel(dim):
                Output[bz, hy, i] = o_acc[i]

    @T.prim_func
    def main(
            Q: T.Tensor([batch, heads, dim], dtype),
            Q_pe: T.Tensor([batch, heads, pe_dim], dtype),
            KV: T.Tensor([batch, seqlen_kv, kv_head_num, dim], dtype),
            K_pe: T.Tensor([batch, seqlen_kv, kv_head_num, pe_dim], dtype),
            glse: T.Tensor([batch, heads, num_split], accum_dtype),
            Output_partial: T.Tensor([batch, heads, num_split, dim], accum_dtype),
            Output: T.Tensor([batch, heads, dim], dtype),
    ):
        attention_split(Q, Q_pe, KV, K_pe, glse, Output_partial)
        combine(glse, Output_partial, Output)

    return main


def ref_program(q, q_pe, kv, k_pe):
    import torch
    dim = q.shape[-1]
    pe_dim = q_pe.shape[-1]
    s = (torch.einsum("bhd,bsd->bhs", q.float(), kv[:, :, 0].float()) +
         torch.einsum("bhd,bsd->bhs", q_pe.float(), k_pe[:, :, 0].float())) / (dim + pe_dim)**0.5
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhs,bsd->bhd", p, kv[:, :, 0].float()).to(q.dtype)


def flops(batch, heads, seqlen_kv, dim, pe_dim):
    return 2 * batch * heads * seqlen_kv * (dim + pe_dim) + 2 * batch * heads * seqlen_kv * dim


def auto_split(batch, heads, block_H=64, cus=256):
    """Smallest KV split that puts at least one block on every CU: at b128 h128 (256 blocks without a
    split) split 1 runs 711.5 TF against 642.3 for split 4 (profiles/r6/mla_bf16_sweep.log); small
    batches split more to fill the chip (the LSE combine kernel sums the partials)."""
    blocks = batch * max(1, heads // block_H)
    split = 1
    while blocks * split < cus and split < 16:
        split *= 2
    return split


def main(batch=128, heads=128, kv_heads=1, kv_ctx=8192, dim=512, pe_dim=64, num_split=None):
    import torch
    num_split = num_split or auto_split(batch, heads)
    kernel = mla_decode(batch, heads, kv_heads, kv_ctx, dim, pe_dim, num_split=num_split)
    q = torch.randn(batch, heads, dim, device="cuda", dtype=torch.float16)
    q_pe = torch.randn(batch, heads, pe_dim, device="cuda", dtype=torch.float16)
    kv = torch.randn(batch, kv_ctx, kv_heads, dim, device="cuda", dtype=torch.float16)
    k_pe = torch.randn(batch, kv_ctx, kv_heads, pe_dim, device="cuda", dtype=torch.float16)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, dim, device="cuda")
    out = kernel(q, q_pe, kv, k_pe, glse, part)
    torch.testing.assert_close(out.float(), ref_program(q, q_pe, kv, k_pe).float(), rtol=2e-2, atol=2e-2)
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, q_pe, kv, k_pe, glse, part))
    print(f"MLA decode b{batch} h{heads} kv{kv_ctx}: {lat:.3f} ms, "
          f"{flops(batch, heads, kv_ctx, dim, pe_dim) / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--heads", type=int, default=128)
    p.add_argument("--kv_ctx", type=int, default=8192)
    p.add_argument("--num_split", type=int, default=None, help="default: auto_split (one block per CU at least)")
    a = p.parse_args()
    main(a.batch, a.heads, 1, a.kv_ctx, 512, 64, a.num_split)
