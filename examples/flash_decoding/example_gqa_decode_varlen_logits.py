"""GQA decode over a packed (varlen) or paged KV cache that also returns per-block attention
scores — the "attention pool" used to pick sparse KV blocks for the next step
(reference: examples/flash_decoding/example_gqa_decode_varlen_logits.py:212-350 and
example_gqa_decode_varlen_logits_paged.py:32-165).

Inputs: Q [batch, heads, dim] (one token per sequence), K/V packed [total_k, kv_heads, dim]
with ``cu_seqlens_k`` [batch+1] offsets (or, paged, a token pool addressed through
``block_table`` [batch, max_pages]), ``s_aux`` [heads] per-head attention-sink logits.
Outputs: O [batch, heads, dim] and S [batch, heads, ceil(max_seqlen/block_N)] where
S[b, h, j] = max over the keys of block j of softmax(q k^T * sm_scale (+ sink))[h] — the
probability of the most-attended key of the block, 0 past the sequence's end.

MI355X schedule (the reference runs one workgroup per (sequence, head-group) — batch 1 with 8 KV
heads would occupy 8 of 256 CUs):

* split-KV: grid (batch, heads / valid_h, num_split); every split streams a balanced range of
  the sequence's KV blocks through an LDS-DMA ring, S = Q K^T and O = P V on MFMA (the GQA
  group's query heads padded to the 16-row MFMA M dimension), and records each block's row max
  of the scaled logits (base 2) into an fp32 workspace;
* one combine kernel per (head, sequence) folds the splits' log-sum-exps and the sink into the
  final LSE, rescales the partial outputs, and turns the recorded block maxima into
  probabilities in the same pass: S = exp2(m_blk - LSE).  No second sweep over the logits.

The sink enters as exp(sink - max) in the softmax normaliser, as in the reference's Triton
kernel and torch reference (its TileLang kernel adds the raw sink value to the row sum, which
the reference's own check cannot tell apart for sinks ~0.1: that form is not reproduced).
"""
import argparse
import math

import tilelang
import tilelang.language as T

FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


def _program(batch, heads, k_heads, max_seqlen_kv, total_k, dim, has_sink, block_N, block_H, num_split, threads,
             num_stages, dtype, paged, page_size=None, max_pages=None):
    scale = (1.0 / dim)**0.5 * LOG2E
    accum = "float"
    group = heads // k_heads
    valid_h = min(block_H, group)
    assert group % valid_h == 0
    n_sblk = -(-max_seqlen_kv // block_N)
    if paged:
        assert page_size % block_N == 0
        table_shape = [batch, max_pages]

    @T.macro
    def split_kernel(Q, K, V, cu_seqlens_k, block_table, glse, O_part, S_raw):
        with T.Kernel(batch, heads // valid_h, num_split, threads=threads) as (bx, by, bz):
            Q_s = T.alloc_shared([block_H, dim], dtype)
            K_s = T.alloc_shared([block_N, dim], dtype)
            V_s = T.alloc_shared([block_N, dim], dtype)
            acc_s = T.alloc_fragment([block_H, block_N], accum)
            acc_s_cast = T.alloc_fragment([block_H, block_N], dtype)
            acc_o = T.alloc_fragment([block_H, dim], accum)
            m_blk = T.alloc_fragment([block_H], accum)
            m = T.alloc_fragment([block_H], accum)
            alpha = T.alloc_fragment([block_H], accum)
            r_sum = T.alloc_fragment([block_H], accum)
            l_sum = T.alloc_fragment([block_H], accum)
            g = by * valid_h // group
            k0 = cu_seqlens_k[bx]
            seqlen = cu_seqlens_k[bx + 1] - k0
            nb = T.ceildiv(seqlen, block_N)
            per = T.ceildiv(nb, num_split)
            b_lo = bz * per
            n_iter = T.max(T.min(nb - b_lo, per), 0)

            T.clear(Q_s)
            T.copy(Q[bx, by * valid_h:(by + 1) * valid_h, :], Q_s[0:valid_h, :])
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -T.infinity(accum))
            for k in T.Pipelined(n_iter, num_stages=num_stages):
                pos = (b_lo + k) * block_N
                if paged:
                    row = block_table[bx, pos // page_size] * page_size + pos % page_size
                    T.copy(K[row:row + block_N, g, :], K_s)
                    T.copy(V[row:row + block_N, g, :], V_s)
                else:
                    T.copy(K[k0 + pos:k0 + pos + block_N, g, :], K_s)
                    T.copy(V[k0 + pos:k0 + pos + block_N, g, :], V_s)
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.if_then_else(pos + j < seqlen, 0, -T.infinity(accum))
                T.gemm(Q_s, K_s, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.reduce_max(acc_s, m_blk, dim=1, clear=True)
                for i in T.Parallel(block_H):
                    if i < valid_h:
                        S_raw[bx, by * valid_h + i, b_lo + k] = m_blk[i] * scale
                for i in T.Parallel(block_H):
                    alpha[i] = T.exp2(m[i] * scale - T.max(m[i], m_blk[i]) * scale)
                    m[i] = T.max(m[i], m_blk[i])
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m[i] * scale)
                T.reduce_sum(acc_s, r_sum, dim=1)
                for i in T.Parallel(block_H):
                    l_sum[i] = l_sum[i] * alpha[i] + r_sum[i]
                for i, j in T.Parallel(block_H, dim):
                    acc_o[i, j] *= alpha[i]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_s, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for i, j in T.Parallel(block_H, dim):
                acc_o[i, j] = T.if_then_else(l_sum[i] > 0, acc_o[i, j] / l_sum[i], 0.0)
            for i in T.Parallel(block_H):
                l_sum[i] = T.if_then_else(l_sum[i] > 0, T.log2(l_sum[i]) + m[i] * scale, -T.infinity(accum))
            T.copy(l_sum[0:valid_h], glse[bx, by * valid_h:(by + 1) * valid_h, bz])
            T.copy(acc_o[0:valid_h, :], O_part[bx, by * valid_h:(by + 1) * valid_h, bz, :])

    @T.macro
    def combine(cu_seqlens_k, s_aux, glse, O_part, S_raw, Output, S):
        with T.Kernel(heads, batch, threads=128) as (hy, bz):
            o_acc = T.alloc_fragment([dim], accum)
            mx = T.alloc_var(accum)
            tot = T.alloc_var(accum)
            lse = T.alloc_var(accum)
            sc = T.alloc_var(accum)
            nb = T.ceildiv(cu_seqlens_k[bz + 1] - cu_seqlens_k[bz], block_N)
            T.clear(o_acc)
            mx = -T.infinity(accum)
            if has_sink:
                mx = s_aux[hy] * LOG2E
            for k in T.serial(num_split):
                mx = T.max(mx, glse[bz, hy, k])
            tot = 0.0
            if has_sink:
                tot = T.exp2(s_aux[hy] * LOG2E - mx)
            for k in T.serial(num_split):
                tot += T.exp2(glse[bz, hy, k] - mx)
            lse = T.log2(tot) + mx
            for k in T.serial(num_split):
                sc = T.exp2(glse[bz, hy, k] - lse)
                for i in T.Parallel(dim):
                    o_acc[i] += O_part[bz, hy, k, i] * sc
            for i in T.Parallel(dim):
                Output[bz, hy, i] = o_acc[i]
            for j in T.Parallel(n_sblk):
                S[bz, hy, j] = T.if_then_else(j < nb, T.exp2(S_raw[bz, hy, j] - lse), 0.0)

    ws = dict(glse=[batch, heads, num_split], part=[batch, heads, num_split, dim], sraw=[batch, heads, n_sblk])
    if paged:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, dim], dtype), K: T.Tensor([total_k, k_heads, dim], dtype),
                 V: T.Tensor([total_k, k_heads, dim], dtype), cu_seqlens_k: T.Tensor([batch + 1], "int32"),
                 s_aux: T.Tensor([heads], "float32"), block_table: T.Tensor(table_shape, "int32"),
                 glse: T.Tensor(ws["glse"], accum), O_part: T.Tensor(ws["part"], accum),
                 S_raw: T.Tensor(ws["sraw"], accum), Output: T.Tensor([batch, heads, dim], dtype),
                 S: T.Tensor([batch, heads, n_sblk], dtype)):
            split_kernel(Q, K, V, cu_seqlens_k, block_table, glse, O_part, S_raw)
            combine(cu_seqlens_k, s_aux, glse, O_part, S_raw, Output, S)
    else:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, dim], dtype), K: T.Tensor([total_k, k_heads, dim], dtype),
                 V: T.Tensor([total_k, k_heads, dim], dtype), cu_seqlens_k: T.Tensor([batch + 1], "int32"),
                 s_aux: T.Tensor([heads], "float32"), glse: T.Tensor(ws["glse"], accum),
                 O_part: T.Tensor(ws["part"], accum), S_raw: T.Tensor(ws["sraw"], accum),
                 Output: T.Tensor([batch, heads, dim], dtype), S: T.Tensor([batch, heads, n_sblk], dtype)):
            split_kernel(Q, K, V, cu_seqlens_k, None, glse, O_part, S_raw)
            combine(cu_seqlens_k, s_aux, glse, O_part, S_raw, Output, S)

    return main


@tilelang.jit(out_idx=[-2, -1], pass_configs=FAST_MATH)
def flashattn(batch, heads, k_heads, max_seqlen_kv, total_seqlen_k, dim, has_sink, block_N=64, block_H=16,
              num_split=8, num_stages=2, threads=64, dtype="float16"):
    """Reference-named entry (example_gqa_decode_varlen_logits.py:212): packed varlen KV cache.
    Call as kernel(Q, K, V, cu_seqlens_k, s_aux, glse, O_part, S_raw) -> (O, S)."""
    return _program(batch, heads, k_heads, max_seqlen_kv, total_seqlen_k, dim, has_sink, block_N, block_H, num_split,
                    threads, num_stages, dtype, False)


@tilelang.jit(out_idx=[-2, -1], pass_configs=FAST_MATH)
def flashattn_paged(batch, heads, k_heads, max_seqlen_kv, total_pool_tokens, dim, has_sink, page_block_size,
                    block_N=64, block_H=16, num_split=8, num_stages=2, threads=64, dtype="float16"):
    """Paged variant (example_gqa_decode_varlen_logits_paged.py:32): K/V are a token pool of pages of
    ``page_block_size`` tokens; ``block_table[b, p]`` is the pool page holding tokens
    [p * page_block_size, (p + 1) * page_block_size) of sequence b.  cu_seqlens_k only supplies the
    lengths.  Call as kernel(Q, K, V, cu_seqlens_k, s_aux, block_table, glse, O_part, S_raw)."""
    max_pages = -(-max_seqlen_kv // page_block_size)
    return _program(batch, heads, k_heads, max_seqlen_kv, total_pool_tokens, dim, has_sink, block_N, block_H,
                    num_split, threads, num_stages, dtype, True, page_size=page_block_size, max_pages=max_pages)


class AttnPoolDecode:
    """Owns the split workspaces; ``__call__`` matches flash_attn_with_attn_pool_decode_tilelang
    (reference :334-350): returns O and the head-pooled block scores."""

    def __init__(self, kernel, batch, heads, dim, num_split, max_seqlen_kv, block_N, device):
        import torch
        nsb = -(-max_seqlen_kv // block_N)
        self.kernel = kernel
        self.glse = torch.empty(batch, heads, num_split, device=device)
        self.part = torch.empty(batch, heads, num_split, dim, device=device)
        self.sraw = torch.empty(batch, heads, nsb, device=device)

    def __call__(self, q, k, v, cu_seqlens_k, s_aux, block_table=None, pool_heads=None):
        import torch
        args = (q, k, v, cu_seqlens_k, s_aux) + ((block_table, ) if block_table is not None else ())
        o, s = self.kernel(*args, self.glse, self.part, self.sraw)
        if pool_heads:
            s = torch.max_pool2d(s, kernel_size=(pool_heads, 1), stride=(pool_heads, 1))
        return o, s


def ref_program(q, k, v, cu_seqlens_k, sink, block_N):
    """fp32 reference: per sequence softmax(q k^T / sqrt(d)) with an optional sink in the
    normaliser; returns O [b,h,d] and S [b,h,ceil(max_len/block_N)] (block-max probabilities)."""
    import torch
    b, h, d = q.shape
    g = h // k.shape[1]
    lens = (cu_seqlens_k[1:] - cu_seqlens_k[:-1]).tolist()
    nsb = -(-max(lens) // block_N)
    out = torch.zeros(b, h, d, device=q.device)
    S = torch.zeros(b, h, nsb, device=q.device)
    for i in range(b):
        s0, n = int(cu_seqlens_k[i]), lens[i]
        kk = k[s0:s0 + n].float().repeat_interleave(g, 1)
        vv = v[s0:s0 + n].float().repeat_interleave(g, 1)
        logits = torch.einsum("hd,nhd->hn", q[i].float(), kk) / math.sqrt(d)
        mx = logits.max(-1, keepdim=True).values
        if sink is not None:
            mx = torch.maximum(mx, sink.view(h, 1))
        e = torch.exp(logits - mx)
        den = e.sum(-1, keepdim=True) + (torch.exp(sink.view(h, 1) - mx) if sink is not None else 0)
        p = e / den
        out[i] = torch.einsum("hn,nhd->hd", p, vv)
        nbi = -(-n // block_N)
        S[i, :, :nbi] = torch.nn.functional.pad(p, (0, nbi * block_N - n)).view(h, nbi, block_N).amax(-1)
    return out, S


def make_inputs(lens, heads, k_heads, dim, device, dtype, sink=True, page_size=None):
    import torch
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=device)
    total = int(cu[-1])
    q = torch.randn(len(lens), heads, dim, device=device, dtype=dtype)
    k = torch.randn(total, k_heads, dim, device=device, dtype=dtype)
    v = torch.randn(total, k_heads, dim, device=device, dtype=dtype)
    s_aux = (torch.randn(heads, device=device) * 0.1) if sink else torch.zeros(heads, device=device)
    if page_size is None:
        return q, k, v, cu, s_aux
    # scatter every sequence's pages to random pool pages
    max_pages = -(-max(lens) // page_size)
    n_pages = sum(-(-n // page_size) for n in lens)
    perm = torch.randperm(n_pages).tolist()
    table = torch.zeros(len(lens), max_pages, dtype=torch.int32)
    kp = torch.zeros(n_pages * page_size, k_heads, dim, dtype=dtype, device=device)
    vp = torch.zeros_like(kp)
    c = 0
    for i, n in enumerate(lens):
        for p in range(-(-n // page_size)):
            dst, src = perm[c], int(cu[i]) + p * page_size
            m = min(page_size, n - p * page_size)
            kp[dst * page_size:dst * page_size + m] = k[src:src + m]
            vp[dst * page_size:dst * page_size + m] = v[src:src + m]
            table[i, p] = dst
            c += 1
    return q, k, v, cu, s_aux, kp, vp, table.to(device)


def main(batch=1, q_heads=32, kv_heads=8, k_seqlen=8192, head_size=128, block_size=64, num_split=16,
         test_varlen=False, paged=False, page_block_size=128):
    import torch
    dtype = torch.float16
    lens = torch.randint(k_seqlen // 4, k_seqlen + 1, (batch, )).tolist() if test_varlen else [k_seqlen] * batch
    inp = make_inputs(lens, q_heads, kv_heads, head_size, "cuda", dtype, True,
                      page_block_size if paged else None)
    q, k, v, cu, s_aux = inp[:5]
    if paged:
        kp, vp, table = inp[5:]
        kern = flashattn_paged(batch, q_heads, kv_heads, max(lens), kp.shape[0], head_size, True, page_block_size,
                               block_N=block_size, num_split=num_split)
        run = AttnPoolDecode(kern, batch, q_heads, head_size, num_split, max(lens), block_size, "cuda")
        fn = lambda: run(q, kp, vp, cu, s_aux, table)  # noqa: E731
    else:
        kern = flashattn(batch, q_heads, kv_heads, max(lens), k.shape[0], head_size, True, block_N=block_size,
                         num_split=num_split)
        run = AttnPoolDecode(kern, batch, q_heads, head_size, num_split, max(lens), block_size, "cuda")
        fn = lambda: run(q, k, v, cu, s_aux)  # noqa: E731
    o, s = fn()
    ro, rs = ref_program(q, k, v, cu, s_aux, block_size)
    torch.testing.assert_close(o.float(), ro, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(s.float(), rs, rtol=1e-2, atol=1e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    lat = do_bench(fn)
    kv_bytes = 2 * sum(lens) * kv_heads * head_size * 2
    print(f"attn-pool decode b{batch} h{q_heads}/{kv_heads} kv{k_seqlen} paged={paged}: {lat * 1e3:.1f} us, "
          f"{kv_bytes / lat * 1e-6:.0f} GB/s")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch_size", type=int, default=1)
    p.add_argument("--q_heads", type=int, default=32)
    p.add_argument("--kv_heads", type=int, default=8)
    p.add_argument("--k_seqlen", type=int, default=8192)
    p.add_argument("--head_size", type=int, default=128)
    p.add_argument("--block_size", type=int, default=64)
    p.add_argument("--num_split", type=int, default=16)
    p.add_argument("--test_varlen", action="store_true")
    p.add_argument("--paged", action="store_true")
    p.add_argument("--page_block_size", type=int, default=128)
    a = p.parse_args()
    main(a.batch_size, a.q_heads, a.kv_heads, a.k_seqlen, a.head_size, a.block_size, a.num_split, a.test_varlen,
         a.paged, a.page_block_size)
