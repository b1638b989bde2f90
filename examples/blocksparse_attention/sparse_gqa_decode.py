"""Block-sparse GQA decoding over a KV cache (reference: examples/blocksparse_attention/
example_tilelang_sparse_gqa_decode_{varlen_indice,varlen_mask,paged}.py).

One new token per sequence (Q [batch, heads, dim]) attends only to selected ``block_size``-token
blocks of its KV cache, given per KV head either as an index list ``block_indices [batch, heads_kv,
max_selected]`` (-1 padded) or as a ``block_mask [batch, heads_kv, num_blocks]``; ``cache_seqlens``
masks each sequence's tail; the paged variant maps logical blocks to physical pages through
``block_table``.  Schedule as the dense GQA decoder (examples/flash_decoding): one workgroup per
(sequence, KV head, split) with the KV head's query heads padded to the 16-row MFMA M dimension,
the selected blocks divided over ``num_split`` workgroups (the KV read is what bounds decode, so
more concurrent streams), then a combine kernel merges the splits by their base-2 log-sum-exps.
"""
import tilelang
import tilelang.language as T

FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}
LOG2E = 1.44269504


def _program(mode, batch, heads, heads_kv, dim, block_size, max_sel, num_split, block_H, threads, num_stages, dtype,
             max_cache_seqlen=None, num_pages=None, page_size=None, max_pages=None):
    scale = (1.0 / dim)**0.5 * LOG2E
    accum = "float"
    G = heads // heads_kv
    valid_h = min(block_H, G)
    BN = block_size
    if mode == "paged":
        assert page_size % BN == 0
        k_shape = [num_pages, page_size, heads_kv, dim]
    else:
        k_shape = [batch, max_cache_seqlen, heads_kv, dim]
    per_split = (max_sel + num_split - 1) // num_split

    @T.macro
    def split_kernel(Q, K, V, Sel, cache_seqlens, block_table, glse, Opart):
        with T.Kernel(batch, heads // valid_h, num_split, threads=threads) as (bx, by, bz):
            Q_s = T.alloc_shared([block_H, dim], dtype)
            K_s = T.alloc_shared([BN, dim], dtype)
            V_s = T.alloc_shared([BN, dim], dtype)
            acc_s = T.alloc_fragment([block_H, BN], accum)
            acc_s_cast = T.alloc_fragment([block_H, BN], dtype)
            acc_o = T.alloc_fragment([block_H, dim], accum)
            m = T.alloc_fragment([block_H], accum)
            m_prev = T.alloc_fragment([block_H], accum)
            alpha = T.alloc_fragment([block_H], accum)
            l_sum = T.alloc_fragment([block_H], accum)
            r_sum = T.alloc_fragment([block_H], accum)
            g = by * valid_h // G
            seqlen = cache_seqlens[bx]
            T.clear(Q_s)
            T.copy(Q[bx, by * valid_h:(by + 1) * valid_h, :], Q_s[0:valid_h, :])
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            for it in T.Pipelined(per_split, num_stages=num_stages):
                slot = bz * per_split + it
                if mode == "mask":
                    blk = T.if_then_else(slot < max_sel, T.if_then_else(Sel[bx, g, T.min(slot, max_sel - 1)], slot, -1),
                                         -1)
                else:
                    blk = T.if_then_else(slot < max_sel, Sel[bx, g, T.min(slot, max_sel - 1)], -1)
                kv0 = T.max(blk, 0) * BN
                if mode == "paged":
                    page = block_table[bx, kv0 // page_size]
                    # == kv0 % page_size (kv0 is block aligned); provably off + BN <= page_size (LDS-DMA)
                    off = T.max(blk, 0) % (page_size // BN) * BN
                    T.copy(K[page, off:off + BN, g, :], K_s)
                    T.copy(V[page, off:off + BN, g, :], V_s)
                else:
                    T.copy(K[bx, kv0:kv0 + BN, g, :], K_s)
                    T.copy(V[bx, kv0:kv0 + BN, g, :], V_s)
                for i, j in T.Parallel(block_H, BN):
                    acc_s[i, j] = T.if_then_else((blk >= 0) & (kv0 + j < seqlen), 0, -T.infinity(accum))
                T.gemm(Q_s, K_s, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                # lazy rescale: O is rescaled only when a row's max moves by more than 2^8
                T.copy(m, m_prev)
                T.reduce_max(acc_s, m_prev, dim=1, clear=False)  # candidate max
                rescale = T.alloc_var("int32")
                rescale = 0
                for i in T.Parallel(block_H):
                    if (m_prev[i] - m[i]) * scale > 8.0:
                        alpha[i] = T.exp2((m[i] - m_prev[i]) * scale)
                        m[i] = m_prev[i]
                        rescale = 1
                    else:
                        alpha[i] = 1.0
                for i, j in T.Parallel(block_H, BN):
                    acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m[i] * scale)
                T.reduce_sum(acc_s, r_sum, dim=1)
                for i in T.Parallel(block_H):
                    l_sum[i] = l_sum[i] * alpha[i] + r_sum[i]
                if rescale != 0:
                    for i, d in T.Parallel(block_H, dim):
                        acc_o[i, d] *= alpha[i]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_s, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for i, d in T.Parallel(block_H, dim):
                acc_o[i, d] = T.if_then_else(l_sum[i] > 0, acc_o[i, d] / l_sum[i], 0.0)
            for i in T.Parallel(block_H):
                l_sum[i] = T.if_then_else(l_sum[i] > 0, T.log2(l_sum[i]) + m[i] * scale, -T.infinity(accum))
            T.copy(l_sum[0:valid_h], glse[bx, by * valid_h:(by + 1) * valid_h, bz])
            T.copy(acc_o[0:valid_h, :], Opart[bx, by * valid_h:(by + 1) * valid_h, bz, :])

    @T.macro
    def combine(glse, Opart, Output):
        with T.Kernel(heads, batch, threads=128) as (hy, bz):
            o_acc = T.alloc_fragment([dim], accum)
            mx = T.alloc_local([1], accum)
            tot = T.alloc_local([1], accum)
            sc = T.alloc_local([1], accum)
            T.clear(o_acc)
            mx[0] = -T.infinity(accum)
            for k in T.serial(num_split):
                mx[0] = T.max(mx[0], glse[bz, hy, k])
            tot[0] = 0.0
            for k in T.serial(num_split):
                tot[0] += T.exp2(glse[bz, hy, k] - mx[0])
            tot[0] = T.log2(tot[0]) + mx[0]
            for k in T.serial(num_split):
                sc[0] = T.exp2(glse[bz, hy, k] - tot[0])
                for i in T.Parallel(dim):
                    o_acc[i] += Opart[bz, hy, k, i] * sc[0]
            for i in T.Parallel(dim):
                Output[bz, hy, i] = o_acc[i]

    sel_dtype = "bool" if mode == "mask" else "int32"
    part = [batch, heads, num_split, dim]
    if mode == "paged":

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, dim], dtype), K: T.Tensor(k_shape, dtype), V: T.Tensor(k_shape, dtype),
                 block_indices: T.Tensor([batch, heads_kv, max_sel], sel_dtype),
                 cache_seqlens: T.Tensor([batch], "int32"), block_table: T.Tensor([batch, max_pages], "int32"),
                 glse: T.Tensor([batch, heads, num_split], accum), Opart: T.Tensor(part, accum),
                 Output: T.Tensor([batch, heads, dim], dtype)):
            split_kernel(Q, K, V, block_indices, cache_seqlens, block_table, glse, Opart)
            combine(glse, Opart, Output)
    else:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, dim], dtype), K: T.Tensor(k_shape, dtype), V: T.Tensor(k_shape, dtype),
                 block_sel: T.Tensor([batch, heads_kv, max_sel], sel_dtype), cache_seqlens: T.Tensor([batch], "int32"),
                 glse: T.Tensor([batch, heads, num_split], accum), Opart: T.Tensor(part, accum),
                 Output: T.Tensor([batch, heads, dim], dtype)):
            split_kernel(Q, K, V, block_sel, cache_seqlens, None, glse, Opart)
            combine(glse, Opart, Output)

    return main


@tilelang.jit(out_idx=[-3, -2, -1], pass_configs=FAST_MATH)
def sparse_gqa_decode_indice(batch, heads, heads_kv, dim, block_size, max_cache_seqlen, max_selected_blocks,
                             num_split=4, block_H=16, threads=64, num_stages=2, dtype="float16"):
    return _program("indice", batch, heads, heads_kv, dim, block_size, max_selected_blocks, num_split, block_H, threads,
                    num_stages, dtype, max_cache_seqlen=max_cache_seqlen)


@tilelang.jit(out_idx=[-3, -2, -1], pass_configs=FAST_MATH)
def sparse_gqa_decode_mask(batch, heads, heads_kv, dim, block_size, max_cache_seqlen, num_split=4, block_H=16,
                           threads=64, num_stages=2, dtype="float16"):
    nb = (max_cache_seqlen + block_size - 1) // block_size
    return _program("mask", batch, heads, heads_kv, dim, block_size, nb, num_split, block_H, threads, num_stages, dtype,
                    max_cache_seqlen=max_cache_seqlen)


@tilelang.jit(out_idx=[-3, -2, -1], pass_configs=FAST_MATH)
def sparse_gqa_decode_paged(batch, heads, heads_kv, dim, block_size, num_pages, page_size, max_pages,
                            max_selected_blocks, num_split=4, block_H=16, threads=64, num_stages=2, dtype="float16"):
    return _program("paged", batch, heads, heads_kv, dim, block_size, max_selected_blocks, num_split, block_H, threads,
                    num_stages, dtype, num_pages=num_pages, page_size=page_size, max_pages=max_pages)


def ref_program(q, k, v, block_indices, cache_seqlens, block_size):
    """q [b,h,d]; k/v [b,s,hk,d] contiguous; block_indices [b,hk,sel] (-1 = none).  (The kernels return
    (lse of the splits, partial outputs, output); the output is the last.)"""
    import torch
    b, h, d = q.shape
    hk = k.shape[2]
    G = h // hk
    out = torch.zeros(b, h, d, dtype=torch.float32, device=q.device)
    for i in range(b):
        n = int(cache_seqlens[i])
        for g in range(hk):
            toks = []
            for blk in block_indices[i, g].tolist():
                if blk >= 0:
                    toks.extend(t for t in range(blk * block_size, (blk + 1) * block_size) if t < n)
            if not toks:
                continue
            ix = torch.tensor(sorted(set(toks)), device=q.device)
            s = q[i, g * G:(g + 1) * G].float() @ k[i, ix, g].float().T / d**0.5
            out[i, g * G:(g + 1) * G] = torch.softmax(s, -1) @ v[i, ix, g].float()
    return out


def random_selection(batch, heads_kv, cache_seqlens, block_size, max_sel, device, seed=0):
    import torch
    g = torch.Generator().manual_seed(seed)
    idx = torch.full((batch, heads_kv, max_sel), -1, dtype=torch.int32)
    for i in range(batch):
        nb = (int(cache_seqlens[i]) + block_size - 1) // block_size
        for h in range(heads_kv):
            sel = torch.randperm(nb, generator=g)[:max_sel].sort().values
            idx[i, h, :len(sel)] = sel.int()
    return idx.to(device)


def indices_to_mask(idx, num_blocks):
    import torch
    mask = torch.zeros(idx.shape[0], idx.shape[1], num_blocks, dtype=torch.bool, device=idx.device)
    valid = idx >= 0
    b, h, _ = torch.nonzero(valid, as_tuple=True)
    mask[b, h, idx[valid].long()] = True
    return mask
