"""Persistent DeepSeek MLA decode: split-KV attention and the LSE combine in ONE kernel
(reference: examples/deepseek_mla/example_mla_decode_persistent.py).

The grid is one 8-wave workgroup per CU (256 on MI355X).  Each workgroup walks the
(batch, head block, KV split) tiles ``block_id, block_id + 256, ...``; tiles are numbered so that
the head blocks reading the same latent KV slice are 8 apart, i.e. they run on the same XCD
(blockIdx round-robins over the 8 XCDs) and the second read of the slice hits that XCD's L2.
``T.sync_grid()`` (cooperative launch: the whole grid is resident) separates the attention
phase from the combine phase, which then walks (batch, head) rows the same way.
"""
import argparse

import tilelang
import tilelang.language as T

from example_mla_decode import ref_program, flops


@tilelang.jit(out_idx=[6], pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def mla_decode_persistent(batch, heads, kv_head_num, seqlen_kv, dim, pe_dim, block_N=64, block_H=64, num_split=4,
                          num_cu=256, threads=512, num_stages=2, dtype="float16", sum_mfma=True):
    """``sum_mfma``: row sums as P x ones on the MFMA (example_mla_decode.py)."""
    scale = (1.0 / (dim + pe_dim))**0.5 * 1.44269504
    accum_dtype = "float"
    assert kv_head_num == 1, "MLA decode expects one latent KV head"
    VALID_BLOCK_H = min(block_H, heads)
    n_hb = heads // VALID_BLOCK_H
    split_len = seqlen_kv // num_split
    n_kv_tiles = batch * num_split
    total_tiles = n_kv_tiles * n_hb
    xcd_group = 8 if n_kv_tiles % 8 == 0 else 1  # head blocks of one KV slice share an XCD
    attn_waves = (total_tiles + num_cu - 1) // num_cu
    comb_waves = (batch * heads + num_cu - 1) // num_cu

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
        with T.Kernel(num_cu, threads=threads) as (block_id):
            Q_local = T.alloc_fragment([block_H, dim], dtype)
            Q_pe_local = T.alloc_fragment([block_H, pe_dim], dtype)
            KV_shared = T.alloc_shared([block_N, dim], dtype)
            K_pe_shared = T.alloc_shared([block_N, pe_dim], dtype)
            acc_s = T.alloc_fragment([block_H, block_N], accum_dtype)
            P_shared = T.alloc_shared([block_H, block_N], dtype)
            sc_shared = T.alloc_shared([block_H], accum_dtype)
            any_s = T.alloc_shared([2], "int32")
            acc_o = T.alloc_fragment([block_H, dim], accum_dtype)
            if sum_mfma:
                ones_s = T.alloc_shared([block_N, 32], dtype)
                acc_l = T.alloc_fragment([block_H, 32], accum_dtype)
                T.fill(ones_s, 1.0)
            scores_max = T.alloc_fragment([block_H], accum_dtype)
            scores_max_prev = T.alloc_fragment([block_H], accum_dtype)
            scores_scale = T.alloc_fragment([block_H], accum_dtype)
            scores_sum = T.alloc_fragment([block_H], accum_dtype)
            logsum = T.alloc_fragment([block_H], accum_dtype)
            o_acc = T.alloc_fragment([dim], accum_dtype)
            lse_max = T.alloc_local([1], accum_dtype)
            lse_sum = T.alloc_local([1], accum_dtype)
            sc = T.alloc_local([1], accum_dtype)

            for w in T.serial(attn_waves):
                t = w * num_cu + block_id
                hid = (t // xcd_group) % n_hb
                kvt = (t % xcd_group) + xcd_group * (t // (xcd_group * n_hb))
                bid = kvt // num_split
                sid = kvt % num_split
                if t < total_tiles:
                    T.copy(Q[bid, hid * VALID_BLOCK_H:(hid + 1) * VALID_BLOCK_H, :], Q_local)
                    T.copy(Q_pe[bid, hid * VALID_BLOCK_H:(hid + 1) * VALID_BLOCK_H, :], Q_pe_local)
                    T.fill(acc_o, 0)
                    T.fill(logsum, 0)
                    if sum_mfma:
                        T.clear(acc_l)
                    T.fill(scores_max, -(2.0**30))  # lazy rescale (example_mla_decode.py)
                    # lazy-rescale flag, double-buffered by iteration parity: iteration t resets the slot
                    # of t + 1 (ordered by the stage barrier against t - 1's readers and t + 1's setters)
                    for z in T.Parallel(2):
                        any_s[z] = 0
                    for k in T.Pipelined(T.ceildiv(split_len, block_N), num_stages=num_stages):
                        kv_start = split_len * sid + k * block_N
                        T.copy(KV[bid, kv_start:kv_start + block_N, 0, :], KV_shared)
                        T.copy(K_pe[bid, kv_start:kv_start + block_N, 0, :], K_pe_shared)
                        T.clear(acc_s)
                        T.gemm(Q_local, KV_shared, acc_s, transpose_B=True)
                        T.gemm(Q_pe_local, K_pe_shared, acc_s, transpose_B=True)
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
                        for i, j in T.Parallel(block_H, block_N):
                            acc_s[i, j] = T.exp2(acc_s[i, j] * scale - scores_max[i] * scale)
                        if not sum_mfma:
                            T.reduce_sum(acc_s, scores_sum, dim=1)
                            for i in T.Parallel(block_H):
                                logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                        T.copy(scores_scale, sc_shared)
                        T.copy(acc_s, P_shared)
                        if any_s[k % 2] != 0:
                            for i, j in T.Parallel(block_H, dim):
                                acc_o[i, j] *= sc_shared[i]
                            if sum_mfma:
                                for i, j in T.Parallel(block_H, 32):
                                    acc_l[i, j] *= sc_shared[i]
                        T.gemm(P_shared, KV_shared, acc_o)
                        if sum_mfma:
                            T.gemm(P_shared, ones_s, acc_l)
                    if sum_mfma:
                        for i, j in T.Parallel(block_H, 32):  # every column of P x ones is the row sum
                            if j == 0:
                                sc_shared[i] = acc_l[i, j]
                        for i in T.Parallel(block_H):
                            logsum[i] = sc_shared[i]
                    T.copy(logsum, sc_shared)
                    for i, j in T.Parallel(block_H, dim):
                        acc_o[i, j] /= sc_shared[i]
                    for i in T.Parallel(block_H):
                        logsum[i] = T.log2(logsum[i]) + scores_max[i] * scale
                    T.copy(logsum, glse[bid, hid * VALID_BLOCK_H:(hid + 1) * VALID_BLOCK_H, sid])
                    T.copy(acc_o, Output_partial[bid, hid * VALID_BLOCK_H:(hid + 1) * VALID_BLOCK_H, sid, :])

            T.sync_grid()

            for w in T.serial(comb_waves):
                t = w * num_cu + block_id
                bid = t // heads
                hy = t % heads
                if t < batch * heads:
                    T.clear(o_acc)
                    lse_max[0] = -T.infinity(accum_dtype)
                    for k in T.serial(num_split):
                        lse_max[0] = T.max(lse_max[0], glse[bid, hy, k])
                    lse_sum[0] = 0.0
                    for k in T.serial(num_split):
                        lse_sum[0] += T.exp2(glse[bid, hy, k] - lse_max[0])
                    lse_sum[0] = T.log2(lse_sum[0]) + lse_max[0]
                    for k in T.serial(num_split):
                        sc[0] = T.exp2(glse[bid, hy, k] - lse_sum[0])
                        for i in T.Parallel(dim):
                            o_acc[i] += Output_partial[bid, hy, k, i] * sc[0]
                    for i in T.Parallel(dim):
                        Output[bid, hy, i] = o_acc[i]

    return main


def main(batch=128, heads=128, kv_ctx=8192, dim=512, pe_dim=64, num_split=4):
    import torch
    kernel = mla_decode_persistent(batch, heads, 1, kv_ctx, dim, pe_dim, num_split=num_split)
    q = torch.randn(batch, heads, dim, device="cuda", dtype=torch.float16)
    q_pe = torch.randn(batch, heads, pe_dim, device="cuda", dtype=torch.float16)
    kv = torch.randn(batch, kv_ctx, 1, dim, device="cuda", dtype=torch.float16)
    k_pe = torch.randn(batch, kv_ctx, 1, pe_dim, device="cuda", dtype=torch.float16)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, dim, device="cuda")
    out = kernel(q, q_pe, kv, k_pe, glse, part)
    torch.testing.assert_close(out.float(), ref_program(q, q_pe, kv, k_pe).float(), rtol=2e-2, atol=2e-2)
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, q_pe, kv, k_pe, glse, part))
    print(f"persistent MLA decode b{batch} h{heads} kv{kv_ctx}: {lat:.3f} ms, "
          f"{flops(batch, heads, kv_ctx, dim, pe_dim) / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--heads", type=int, default=128)
    p.add_argument("--kv_ctx", type=int, default=8192)
    p.add_argument("--num_split", type=int, default=4)
    a = p.parse_args()
    main(a.batch, a.heads, a.kv_ctx, 512, 64, a.num_split)
