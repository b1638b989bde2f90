"""GQA flash-decoding with split-KV, contiguous and paged KV caches
(reference: examples/flash_decoding/example_gqa_decode.py, example_gqa_decode_varlen_logits_paged.py).

Q [batch, heads, dim] (one new token per sequence) attends to a KV cache with ``groups`` KV
heads (``heads // groups`` query heads share one).  Decode is HBM-bound on the KV read, so the
schedule maximises concurrent KV streams:

* one block per (sequence, KV head, KV split): the ``heads // groups`` query heads of a KV
  head are padded to the 16-row MFMA M dimension (``block_H``) so S = Q K^T and O = P V run
  on matrix cores while every KV byte is read exactly once;
* ``num_split`` splits multiply the block count (batch * groups is far below 256 CUs x
  occupancy for small batches); a second kernel of the same program merges the splits with
  their base-2 log-sum-exps;
* ``cache_seqlens`` masks each sequence's tail (ragged batches), and the paged variant
  gathers KV pages through ``block_table`` with data-dependent LDS-DMA addresses.
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


def _decode_program(batch, heads, groups, dim, block_N, block_H, num_split, threads, num_stages, dtype, paged,
                    seqlen_kv=None, num_pages=None, page_size=None, max_pages=None):
    scale = (1.0 / dim)**0.5 * LOG2E
    accum_dtype = "float"
    kv_group_num = heads // groups
    valid_h = min(block_H, kv_group_num)
    assert kv_group_num % valid_h == 0
    if paged:
        assert page_size % block_N == 0
        max_len = max_pages * page_size
        # every split starts on a block boundary, so a block never straddles two pages
        assert (-(-max_len // num_split)) % block_N == 0, "paged: max_pages * page_size / num_split % block_N"
        k_shape = [num_pages, page_size, groups, dim]
    else:
        max_len = seqlen_kv
        k_shape = [batch, seqlen_kv, groups, dim]
    split_len = T.ceildiv(max_len, num_split)
    n_blocks = -(-(-(-max_len // num_split)) // block_N)

    @T.macro
    def attention_split(Q, K, V, cache_seqlens, block_table, glse, Output_partial):
        with T.Kernel(batch, heads // valid_h, num_split, threads=threads) as (bx, by, bz):
            Q_shared = T.alloc_shared([block_H, dim], dtype)
            K_shared = T.alloc_shared([block_N, dim], dtype)
            V_shared = T.alloc_shared([block_N, dim], dtype)
            acc_s = T.alloc_fragment([block_H, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_H, block_N], dtype)
            acc_o = T.alloc_fragment([block_H, dim], accum_dtype)
            scores_max = T.alloc_fragment([block_H], accum_dtype)
            scores_max_prev = T.alloc_fragment([block_H], accum_dtype)
            scores_scale = T.alloc_fragment([block_H], accum_dtype)
            scores_sum = T.alloc_fragment([block_H], accum_dtype)
            logsum = T.alloc_fragment([block_H], accum_dtype)
            g = by * valid_h // kv_group_num
            seqlen = cache_seqlens[bx]

            T.clear(Q_shared)
            T.copy(Q[bx, by * valid_h:(by + 1) * valid_h, :], Q_shared[0:valid_h, :])
            T.fill(acc_o, 0)
            T.fill(logsum, 0)
            T.fill(scores_max, -T.infinity(accum_dtype))
            for k in T.Pipelined(n_blocks, num_stages=num_stages):
                kv_start = bz * split_len + k * block_N
                if paged:
                    page = block_table[bx, kv_start // page_size]
                    # block-granular in-page offset: provably off + block_N <= page_size (LDS-DMA)
                    off = (kv_start // block_N) % (page_size // block_N) * block_N
                    T.copy(K[page, off:off + block_N, g, :], K_shared)
                    T.copy(V[page, off:off + block_N, g, :], V_shared)
                else:
                    T.copy(K[bx, kv_start:kv_start + block_N, g, :], K_shared)
                    T.copy(V[bx, kv_start:kv_start + block_N, g, :], V_shared)
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.if_then_else(
                        (kv_start + j < seqlen) & (k * block_N + j < split_len), 0, -T.infinity(accum_dtype))
                T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(scores_max, scores_max_prev)
                T.reduce_max(acc_s, scores_max, dim=1, clear=False)
                for i in T.Parallel(block_H):
                    scores_scale[i] = T.if_then_else(
                        scores_max[i] == -T.infinity(accum_dtype), 1.0,
                        T.exp2(scores_max_prev[i] * scale - scores_max[i] * scale))
                for i, j in T.Parallel(block_H, block_N):
                    # masked scores select a -inf exponent (exp2(-inf) = 0): no per-element branch
                    ninf = -T.infinity(accum_dtype)
                    acc_s[i, j] = T.exp2(T.if_then_else(acc_s[i, j] == ninf, ninf,
                                                        acc_s[i, j] * scale - scores_max[i] * scale))
                T.reduce_sum(acc_s, scores_sum, dim=1)
                for i in T.Parallel(block_H):
                    logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] *= scores_scale[i]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for i, j in T.Parallel(block_H, dim):
                acc_o[i, j] = T.if_then_else(logsum[i] > 0, acc_o[i, j] / logsum[i], 0.0)
            for i in T.Parallel(block_H):
                logsum[i] = T.if_then_else(logsum[i] > 0, T.log2(logsum[i]) + scores_max[i] * scale,
                                           -T.infinity(accum_dtype))
            T.copy(logsum[0:valid_h], glse[bx, by * valid_h:(by + 1) * valid_h, bz])
            T.copy(acc_o[0:valid_h, :], Output_partial[bx, by * valid_h:(by + 1) * valid_h, bz, :])

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
                lse_max[0] = T.max(lse_max[0], glse[bz, hy, k])
            lse_sum[0] = 0.0
            for k in T.serial(num_split):
                lse_sum[0] += T.exp2(glse[bz, hy, k] - lse_max[0])
            lse_sum[0] = T.log2(lse_sum[0]) + lse_max[0]
            for k in T.serial(num_split):
                sc[0] = T.exp2(glse[bz, hy, k] - lse_sum[0])
                for i in T.Parallel(dim):
                    o_acc[i] += Output_partial[bz, hy, k, i] * sc[0]
            for i in T.Parallel(dim):
                Output[bz, hy, i] = o_acc[i]

    if paged:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, dim], dtype), K: T.Tensor(k_shape, dtype), V: T.Tensor(k_shape, dtype),
                 cache_seqlens: T.Tensor([batch], "int32"), block_table: T.Tensor([batch, max_pages], "int32"),
                 glse: T.Tensor([batch, heads, num_split], accum_dtype),
                 Output_partial: T.Tensor([batch, heads, num_split, dim], accum_dtype),
                 Output: T.Tensor([batch, heads, dim], dtype)):
            attention_split(Q, K, V, cache_seqlens, block_table, glse, Output_partial)
            combine(glse, Output_partial, Output)
    else:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, dim], dtype), K: T.Tensor(k_shape, dtype), V: T.Tensor(k_shape, dtype),
                 cache_seqlens: T.Tensor([batch], "int32"), glse: T.Tensor([batch, heads, num_split], accum_dtype),
                 Output_partial: T.Tensor([batch, heads, num_split, dim], accum_dtype),
                 Output: T.Tensor([batch, heads, dim], dtype)):
            attention_split(Q, K, V, cache_seqlens, None, glse, Output_partial)
            combine(glse, Output_partial, Output)

    return main


@tilelang.jit(out_idx=[-1], pass_configs=FAST_MATH)
def gqa_decode(batch, heads, groups, seqlen_kv, dim, block_N=64, block_H=16, num_split=4, threads=64,
               num_stages=2, dtype="float16"):
    return _decode_program(batch, heads, groups, dim, block_N, block_H, num_split, threads, num_stages, dtype, False,
                           seqlen_kv=seqlen_kv)


@tilelang.jit(out_idx=[-1], pass_configs=FAST_MATH)
def gqa_decode_paged(batch, heads, groups, num_pages, page_size, max_pages, dim, block_N=64, block_H=16,
                     num_split=4, threads=64, num_stages=2, dtype="float16"):
    return _decode_program(batch, heads, groups, dim, block_N, block_H, num_split, threads, num_stages, dtype, True,
                           num_pages=num_pages, page_size=page_size, max_pages=max_pages)


def ref_program(q, k, v, cache_seqlens):
    """q [b,h,d]; k/v [b,s,g,d] (contiguous cache)."""
    import torch
    b, h, d = q.shape
    g = k.shape[2]
    out = torch.empty_like(q)
    for i in range(b):
        n = int(cache_seqlens[i])
        kk = k[i, :n].float().repeat_interleave(h // g, dim=1)  # [n, h, d]
        vv = v[i, :n].float().repeat_interleave(h // g, dim=1)
        s = torch.einsum("hd,nhd->hn", q[i].float(), kk) / d**0.5
        out[i] = torch.einsum("hn,nhd->hd", torch.softmax(s, -1), vv).to(q.dtype)
    return out


def paged_to_contiguous(kc, block_table, max_pages, page_size):
    import torch
    b = block_table.shape[0]
    return torch.stack([kc[block_table[i].long()].reshape(max_pages * page_size, *kc.shape[2:]) for i in range(b)])


def main(batch=16, heads=32, groups=8, seqlen_kv=8192, dim=128, num_split=8):
    import torch
    kernel = gqa_decode(batch, heads, groups, seqlen_kv, dim, num_split=num_split)
    q = torch.randn(batch, heads, dim, device="cuda", dtype=torch.float16)
    k = torch.randn(batch, seqlen_kv, groups, dim, device="cuda", dtype=torch.float16)
    v = torch.randn_like(k)
    lens = torch.randint(seqlen_kv // 2, seqlen_kv + 1, (batch, ), device="cuda", dtype=torch.int32)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, dim, device="cuda")
    out = kernel(q, k, v, lens, glse, part)
    torch.testing.assert_close(out, ref_program(q, k, v, lens), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v, lens, glse, part))
    kv_bytes = 2 * int(lens.sum()) * groups * dim * 2
    print(f"gqa decode b{batch} h{heads} g{groups} kv{seqlen_kv}: {lat:.4f} ms, {kv_bytes / lat * 1e-6:.1f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--heads", type=int, default=32)
    p.add_argument("--groups", type=int, default=8)
    p.add_argument("--kv_ctx", type=int, default=8192)
    p.add_argument("--dim", type=int, default=128)
    a = p.parse_args()
    main(a.batch, a.heads, a.groups, a.kv_ctx, a.dim)
