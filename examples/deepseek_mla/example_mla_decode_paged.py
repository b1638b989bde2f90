"""DeepSeek MLA decode over a paged latent KV cache with per-sequence lengths (reference:
examples/deepseek_mla/example_mla_decode_paged.py).

KV pages [num_pages, page_size, 512] + K_pe pages [num_pages, page_size, 64]; ``BlockTable[b, i]``
is the page holding tokens [i*page_size, (i+1)*page_size) of sequence b and ``CacheSeqlens[b]``
its length.  Split-KV as in example_mla_decode.py: every split owns a contiguous token range
(rounded to ``block_N``), each step reads one ``block_N`` slice of one page -- a data-dependent
offset along the OUTERMOST (page) dim, which stays an LDS-DMA producer of ``T.Pipelined``
(buffer resource over the whole pool).  Tokens past the sequence end are masked; a split with
no tokens writes lse = -inf and is ignored by the combine kernel.
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}


@tilelang.jit(out_idx=[8], pass_configs=FAST_MATH)
def mla_decode_paged(batch, heads, max_seqlen, num_pages, page_size, dim=512, pe_dim=64, block_N=64, block_H=64,
                     num_split=4, threads=None, num_stages=2, dtype="bfloat16", wide=None, sum_mfma=None):
    """``sum_mfma`` (default with ``wide``): row sums as P x ones on the MFMA (example_mla_decode.py)."""
    if wide is None:
        wide = block_H == 64  # 8 waves, O split over the latent columns (example_mla_decode.py)
    use_sm = wide and (sum_mfma is None or sum_mfma)
    if threads is None:
        threads = 512 if wide else 256
    s_policy = T.GemmWarpPolicy.Square if wide else T.GemmWarpPolicy.FullRow
    scale = (1.0 / (dim + pe_dim))**0.5 * 1.44269504
    accum_dtype = "float"
    VALID_H = min(block_H, heads)
    assert page_size % block_N == 0
    max_pages = (max_seqlen + page_size - 1) // page_size

    @T.prim_func
    def main(Q: T.Tensor([batch, heads, dim], dtype), Q_pe: T.Tensor([batch, heads, pe_dim], dtype),
             KV: T.Tensor([num_pages, page_size, dim], dtype), K_pe: T.Tensor([num_pages, page_size, pe_dim], dtype),
             BlockTable: T.Tensor([batch, max_pages], "int32"), CacheSeqlens: T.Tensor([batch], "int32"),
             glse: T.Tensor([batch, heads, num_split], accum_dtype),
             Output_partial: T.Tensor([batch, heads, num_split, dim], accum_dtype),
             Output: T.Tensor([batch, heads, dim], dtype)):
        with T.Kernel(batch, heads // VALID_H, num_split, threads=threads) as (bx, by, bz):
            Q_local = T.alloc_fragment([block_H, dim], dtype)
            Q_pe_local = T.alloc_fragment([block_H, pe_dim], dtype)
            KV_shared = T.alloc_shared([block_N, dim], dtype)
            K_pe_shared = T.alloc_shared([block_N, pe_dim], dtype)
            acc_s = T.alloc_fragment([block_H, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_H, block_N], dtype)
            P_shared = T.alloc_shared([block_H, block_N], dtype)
            sc_shared = T.alloc_shared([block_H], accum_dtype)
            any_s = T.alloc_shared([2], "int32")
            acc_o = T.alloc_fragment([block_H, dim], accum_dtype)
            m = T.alloc_fragment([block_H], accum_dtype)
            m_prev = T.alloc_fragment([block_H], accum_dtype)
            alpha = T.alloc_fragment([block_H], accum_dtype)
            r_sum = T.alloc_fragment([block_H], accum_dtype)
            l_sum = T.alloc_fragment([block_H], accum_dtype)
            seqlen = CacheSeqlens[bx]
            # this split's token range, whole block_N tiles
            n_tiles = T.ceildiv(seqlen, block_N)
            per_split = T.ceildiv(n_tiles, num_split)
            t_begin = T.min(bz * per_split, n_tiles)
            t_end = T.min(t_begin + per_split, n_tiles)
            T.copy(Q[bx, by * VALID_H:(by + 1) * VALID_H, :], Q_local)
            T.copy(Q_pe[bx, by * VALID_H:(by + 1) * VALID_H, :], Q_pe_local)
            if use_sm:
                ones_s = T.alloc_shared([block_N, 32], dtype)
                acc_l = T.alloc_fragment([block_H, 32], accum_dtype)
                T.fill(ones_s, 1.0)
                T.clear(acc_l)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            # lazy-rescale flag, double-buffered by iteration parity: iteration t resets the slot
            # of t + 1 (ordered by the stage barrier against t - 1's readers and t + 1's setters)
            for z in T.Parallel(2):
                any_s[z] = 0
            for t in T.Pipelined(t_begin, t_end, num_stages=num_stages):
                tok = t * block_N
                page = BlockTable[bx, tok // page_size]
                off = t % (page_size // block_N) * block_N  # == tok % page_size; provably + block_N <= page_size
                T.copy(KV[page, off:off + block_N, :], KV_shared)
                T.copy(K_pe[page, off:off + block_N, :], K_pe_shared)
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.if_then_else(tok + j < seqlen, 0, -T.infinity(accum_dtype))
                T.gemm(Q_local, KV_shared, acc_s, transpose_B=True, policy=s_policy)
                T.gemm(Q_pe_local, K_pe_shared, acc_s, transpose_B=True, policy=s_policy)
                if wide:  # lazy rescale + block-uniform skip flag (example_mla_decode.py)
                    for z in T.Parallel(1):
                        any_s[z + (t + 1) % 2] = 0
                    T.copy(m, m_prev)
                    T.reduce_max(acc_s, m_prev, dim=1, clear=False)  # candidate max
                    for i in T.Parallel(block_H):
                        if (m_prev[i] - m[i]) * scale > 8.0:
                            alpha[i] = T.exp2((m[i] - m_prev[i]) * scale)
                            m[i] = m_prev[i]
                            any_s[t % 2] = 1
                        else:
                            alpha[i] = 1.0
                else:
                    T.copy(m, m_prev)
                    T.reduce_max(acc_s, m, dim=1, clear=False)
                    for i in T.Parallel(block_H):
                        alpha[i] = T.exp2((m_prev[i] - m[i]) * scale)
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m[i] * scale)
                if not use_sm:
                    T.reduce_sum(acc_s, r_sum, dim=1)
                    for i in T.Parallel(block_H):
                        l_sum[i] = l_sum[i] * alpha[i] + r_sum[i]
                if wide:
                    T.copy(alpha, sc_shared)
                    T.copy(acc_s, P_shared)
                    if any_s[t % 2] != 0:
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
                        acc_o[i, j] *= alpha[i]
                    T.gemm(acc_s_cast, KV_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            if use_sm:
                for i, j in T.Parallel(block_H, 32):  # every column of P x ones is the row sum
                    if j == 0:
                        sc_shared[i] = acc_l[i, j]
                for i in T.Parallel(block_H):
                    l_sum[i] = sc_shared[i]
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] /= T.max(sc_shared[i], 1e-30)
            elif wide:
                T.copy(l_sum, sc_shared)
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] /= T.max(sc_shared[i], 1e-30)
            else:
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] /= T.max(l_sum[i], 1e-30)
            for i in T.Parallel(block_H):
                l_sum[i] = T.if_then_else(l_sum[i] > 0, T.log2(l_sum[i]) + m[i] * scale, -T.infinity(accum_dtype))
            T.copy(l_sum[0:VALID_H], glse[bx, by * VALID_H:(by + 1) * VALID_H, bz])
            T.copy(acc_o[0:VALID_H, :], Output_partial[bx, by * VALID_H:(by + 1) * VALID_H, bz, :])

        with T.Kernel(heads, batch, threads=128) as (hy, bz):
            o_acc = T.alloc_fragment([dim], accum_dtype)
            lse_max = T.alloc_var(accum_dtype)
            lse_sum = T.alloc_var(accum_dtype)
            sc = T.alloc_var(accum_dtype)
            T.clear(o_acc)
            lse_max = -(2.0**30)
            for k in T.serial(num_split):
                lse_max = T.max(lse_max, glse[bz, hy, k])
            lse_sum = 0.0
            for k in T.serial(num_split):
                lse_sum += T.exp2(glse[bz, hy, k] - lse_max)
            lse_sum = T.log2(lse_sum) + lse_max
            for k in T.serial(num_split):
                sc = T.exp2(glse[bz, hy, k] - lse_sum)
                for i in T.Parallel(dim):
                    o_acc[i] += T.if_then_else(sc > 0, Output_partial[bz, hy, k, i] * sc, 0.0)
            for i in T.Parallel(dim):
                Output[bz, hy, i] = o_acc[i]

    return main


def make_paged_cache(kv, k_pe, seqlens, page_size, num_pages=None, seed=0):
    """Scatter contiguous caches [b, s, d] into a randomly permuted page pool."""
    import torch
    b, s, _ = kv.shape
    max_pages = (s + page_size - 1) // page_size
    num_pages = num_pages or b * max_pages
    g = torch.Generator().manual_seed(seed)
    perm = torch.randperm(num_pages, generator=g)[:b * max_pages].view(b, max_pages).int().to(kv.device)
    kvp = torch.zeros(num_pages, page_size, kv.shape[-1], dtype=kv.dtype, device=kv.device)
    pep = torch.zeros(num_pages, page_size, k_pe.shape[-1], dtype=kv.dtype, device=kv.device)
    for i in range(b):
        for p in range(max_pages):
            n = min(page_size, s - p * page_size)
            kvp[perm[i, p], :n] = kv[i, p * page_size:p * page_size + n]
            pep[perm[i, p], :n] = k_pe[i, p * page_size:p * page_size + n]
    return kvp, pep, perm


def ref_program(q, q_pe, kv, k_pe, seqlens):
    import torch
    out = []
    for i in range(q.shape[0]):
        n = int(seqlens[i])
        s = (q[i].float() @ kv[i, :n].float().t() + q_pe[i].float() @ k_pe[i, :n].float().t())
        s = s / (q.shape[-1] + q_pe.shape[-1])**0.5
        out.append(torch.softmax(s, -1) @ kv[i, :n].float())
    return torch.stack(out).to(q.dtype)


def main(batch=64, heads=128, max_seqlen=8192, page_size=64, num_split=4):
    import torch
    q = torch.randn(batch, heads, 512, device="cuda", dtype=torch.bfloat16)
    q_pe = torch.randn(batch, heads, 64, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(batch, max_seqlen, 512, device="cuda", dtype=torch.bfloat16)
    k_pe = torch.randn(batch, max_seqlen, 64, device="cuda", dtype=torch.bfloat16)
    seqlens = torch.randint(max_seqlen // 2, max_seqlen + 1, (batch, ), device="cuda", dtype=torch.int32)
    kvp, pep, table = make_paged_cache(kv, k_pe, seqlens, page_size)
    kernel = mla_decode_paged(batch, heads, max_seqlen, kvp.shape[0], page_size, num_split=num_split)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, 512, device="cuda")
    o = kernel(q, q_pe, kvp, pep, table, seqlens, glse, part)
    torch.testing.assert_close(o[:2].float(), ref_program(q[:2], q_pe[:2], kv[:2], k_pe[:2], seqlens[:2]).float(),
                               rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, q_pe, kvp, pep, table, seqlens, glse, part))
    toks = int(seqlens.sum())
    flops = 2 * heads * toks * (512 + 64 + 512)
    print(f"paged MLA decode b{batch} h{heads} avg ctx {toks // batch}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--max_seqlen", type=int, default=8192)
    a = p.parse_args()
    main(a.batch, max_seqlen=a.max_seqlen)
