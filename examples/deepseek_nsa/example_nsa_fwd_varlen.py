"""Native Sparse Attention forward over packed variable-length sequences
(reference: examples/deepseek_nsa/example_tilelang_nsa_fwd_varlen.py:18-165).

Q [C, HQ, D] and K/V [C, H, D] hold the sequences of a batch back to back (C = total tokens),
``Offsets`` [N+1] are the sequence starts, ``TokenIndices`` [C, 2] = (sequence, position in
sequence) of every packed token (``prepare_token_indices``).  Token t of kv-head h attends to the
first ``BlockCounts[t, h]`` blocks of ``block_size`` keys listed in ``BlockIndices[t, h, :]``
(block numbers relative to the token's sequence), causal inside a block.

Schedule as ``example_nsa_fwd.py``: one workgroup per (packed token, kv head) — the reference's
grid repeats every (token, head) ``batch`` times — with the G >= 16 query heads of the kv head as
the MFMA M dimension (one wave per 16 heads, FullRow), each selected block streamed in
``block_T``-row steps through an LDS-DMA ring.  The trip count is the token's own block count
(data dependent), the block start is clamped into the sequence so every copy stays an LDS-DMA
producer, and rows past the sequence are masked (past the packed tensor they read zeros).
"""
import argparse

import tilelang
import tilelang.language as T

FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(pass_configs=FAST_MATH)
def native_sparse_attention_varlen(batch, heads, c_seq_len, dim, is_causal=True, scale=None, block_size=64,
                                   groups=16, selected_blocks=16, block_T=32, num_stages=2, dtype="float16",
                                   unroll=2):
    """Call as kernel(Q, K, V, O_slc, BlockIndices, BlockCounts, Offsets, TokenIndices) (O_slc written).
    ``unroll``: the block loop is emitted twice per trip (constant LDS ring slots): 0.774 -> 0.644 ms
    at the example's shape (profiles/r6/unroll_sweep_examples.log)."""
    scale = ((1.0 / dim)**0.5 if scale is None else scale) * LOG2E
    head_kv = heads // groups
    G, BS, S, D = groups, block_size, selected_blocks, dim
    BT = min(block_T, BS)
    assert BS % BT == 0
    NT = BS // BT
    assert G % 16 == 0, "the query heads of one kv head form the MFMA M dim (multiple of 16)"
    threads = 64 * (G // 16)
    accum = "float"

    @T.prim_func
    def main(Q: T.Tensor([c_seq_len, heads, D], dtype), K: T.Tensor([c_seq_len, head_kv, D], dtype),
             V: T.Tensor([c_seq_len, head_kv, D], dtype), O_slc: T.Tensor([c_seq_len, heads, D], dtype),
             BlockIndices: T.Tensor([c_seq_len, head_kv, S], "int32"),
             BlockCounts: T.Tensor([c_seq_len, head_kv], "int32"), Offsets: T.Tensor([batch + 1], "int32"),
             TokenIndices: T.Tensor([c_seq_len, 2], "int32")):
        with T.Kernel(c_seq_len, head_kv, threads=threads) as (bx, h):
            Q_s = T.alloc_shared([G, D], dtype)
            K_s = T.alloc_shared([BT, D], dtype)
            V_s = T.alloc_shared([BT, D], dtype)
            acc_s = T.alloc_fragment([G, BT], accum)
            acc_s_cast = T.alloc_fragment([G, BT], dtype)
            acc_o = T.alloc_fragment([G, D], accum)
            o_cast = T.alloc_fragment([G, D], dtype)
            m = T.alloc_fragment([G], accum)
            m_prev = T.alloc_fragment([G], accum)
            alpha = T.alloc_fragment([G], accum)
            l_sum = T.alloc_fragment([G], accum)
            r_sum = T.alloc_fragment([G], accum)
            i_n = TokenIndices[bx, 0]
            i_t = TokenIndices[bx, 1]
            bos = Offsets[i_n]
            seqlen = Offsets[i_n + 1] - bos
            ns = T.min(BlockCounts[bx, h], S)
            T.copy(Q[bx, h * G:(h + 1) * G, :], Q_s)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            for i in T.Pipelined(ns * NT, num_stages=num_stages, unroll=unroll):
                blk = BlockIndices[bx, h, i // NT]
                i_s = T.min(T.max(blk, 0), (seqlen - 1) // BS) * BS + (i % NT) * BT
                T.copy(K[bos + i_s:bos + i_s + BT, h, :], K_s)
                T.copy(V[bos + i_s:bos + i_s + BT, h, :], V_s)
                for g, j in T.Parallel(G, BT):
                    ok = (blk >= 0) & (blk * BS <= i_t) & (i_s + j < seqlen)
                    if is_causal:
                        ok = ok & (i_s + j <= i_t)
                    acc_s[g, j] = T.if_then_else(ok, 0, -T.infinity(accum))
                T.gemm(Q_s, K_s, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                # lazy rescale (example_nsa_fwd.py): O is rescaled only when a row's max moves by 2^8
                T.copy(m, m_prev)
                T.reduce_max(acc_s, m_prev, dim=1, clear=False)  # candidate max
                rescale = T.alloc_var("int32")
                rescale = 0
                for g in T.Parallel(G):
                    if (m_prev[g] - m[g]) * scale > 8.0:
                        alpha[g] = T.exp2((m[g] - m_prev[g]) * scale)
                        m[g] = m_prev[g]
                        rescale = 1
                    else:
                        alpha[g] = 1.0
                for g, j in T.Parallel(G, BT):
                    acc_s[g, j] = T.exp2(acc_s[g, j] * scale - m[g] * scale)
                T.reduce_sum(acc_s, r_sum, dim=1)
                for g in T.Parallel(G):
                    l_sum[g] = l_sum[g] * alpha[g] + r_sum[g]
                if rescale != 0:
                    for g, d in T.Parallel(G, D):
                        acc_o[g, d] *= alpha[g]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_s, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for g, d in T.Parallel(G, D):
                o_cast[g, d] = acc_o[g, d] / T.max(l_sum[g], 1e-30)
            T.copy(o_cast, O_slc[bx, h * G:(h + 1) * G, :])

    return main


def prepare_token_indices(offsets):
    """[C, 2] int32 (sequence id, position in sequence) for packed offsets [N+1] (fla's helper)."""
    import torch
    lens = (offsets[1:] - offsets[:-1]).tolist()
    seq = torch.cat([torch.full((n, ), i, dtype=torch.int32) for i, n in enumerate(lens)])
    pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens])
    return torch.stack([seq, pos], 1).to(offsets.device)


def make_inputs(lens, HQ, H, D, S, block_size, device="cpu", dtype=None, seed=0):
    import torch
    dtype = dtype or torch.float16
    g = torch.Generator().manual_seed(seed)
    offsets = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32)
    C = int(offsets[-1])
    q = torch.randn(C, HQ, D, generator=g).to(dtype)
    k = torch.randn(C, H, D, generator=g).to(dtype)
    v = torch.randn(C, H, D, generator=g).to(dtype)
    idx = torch.full((C, H, S), -1, dtype=torch.int32)
    cnt = torch.zeros(C, H, dtype=torch.int32)
    ti = prepare_token_indices(offsets)
    for c in range(C):
        t = int(ti[c, 1])
        nvis = t // block_size + 1
        for h in range(H):
            sel = torch.randperm(nvis, generator=g)[:S].int().sort()[0]
            idx[c, h, :len(sel)] = sel
            cnt[c, h] = int(torch.randint(1, len(sel) + 1, (1, ), generator=g))
    to = lambda x: x.to(device)  # noqa: E731
    return to(q), to(k), to(v), to(idx), to(cnt), to(offsets), to(ti)


def ref_program(q, k, v, block_indices, block_counts, offsets, block_size, scale=None, is_causal=True):
    """fp32 reference over the packed layout."""
    import torch
    C, HQ, D = q.shape
    H = k.shape[1]
    G = HQ // H
    scale = D**-0.5 if scale is None else scale
    out = torch.zeros(C, HQ, D)
    qf, kf, vf = q.float().cpu(), k.float().cpu(), v.float().cpu()
    bi, bc, off = block_indices.cpu(), block_counts.cpu(), offsets.cpu().tolist()
    for n in range(len(off) - 1):
        bos, eos = off[n], off[n + 1]
        for t in range(eos - bos):
            c = bos + t
            for h in range(H):
                toks = []
                for blk in bi[c, h, :int(bc[c, h])].tolist():
                    if blk < 0 or blk * block_size > t:
                        continue
                    hi = min(blk * block_size + block_size, t + 1 if is_causal else eos - bos)
                    toks.extend(range(bos + blk * block_size, bos + hi))
                if not toks:
                    continue
                ix = torch.tensor(toks)
                s = qf[c, h * G:(h + 1) * G] @ kf[ix, h].t() * scale
                out[c, h * G:(h + 1) * G] = torch.softmax(s, -1) @ vf[ix, h]
    return out.to(q.dtype)


def parallel_nsa(q, k, v, g_slc, block_indices, block_counts, offsets, block_size=64, scale=None, kernel=None):
    """Gated selected-block branch of NSA (reference parallel_nsa :170-265, window_size 0):
    o = NSA_slc(q, k, v) * g_slc over packed [C, ...] tensors."""
    import torch
    C, HQ, D = q.shape
    H, S = k.shape[1], block_indices.shape[-1]
    if kernel is None:
        kernel = native_sparse_attention_varlen(len(offsets) - 1, HQ, C, D, True, scale, block_size, HQ // H, S)
    o = torch.empty_like(q)
    kernel(q, k, v, o, block_indices, block_counts, offsets, prepare_token_indices(offsets))
    return o * g_slc.unsqueeze(-1)


def main(lens=(1000, 3000, 2500, 4096), HQ=64, H=4, D=128, S=16, block_size=64):
    import torch
    q, k, v, idx, cnt, off, ti = make_inputs(list(lens), HQ, H, D, S, block_size, "cuda")
    C = q.shape[0]
    kern = native_sparse_attention_varlen(len(lens), HQ, C, D, True, None, block_size, HQ // H, S)
    o = torch.empty_like(q)
    kern(q, k, v, o, idx, cnt, off, ti)
    sub = int(off[1])
    ref = ref_program(q[:sub], k[:sub], v[:sub], idx[:sub], cnt[:sub], off[:2], block_size)
    torch.testing.assert_close(o[:sub].float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    lat = do_bench(lambda: kern(q, k, v, o, idx, cnt, off, ti))
    # every selected (token, kv head, block) is G = HQ/H query rows x block_size keys x D, QK^T + PV
    flops = 4.0 * (HQ // H) * D * block_size * float(cnt.float().sum())
    print(f"NSA varlen fwd C{C} HQ{HQ} H{H} D{D} S{S}x{block_size}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS "
          f"(selected blocks incl. their masked tails)")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--HQ", type=int, default=64)
    p.add_argument("--H", type=int, default=4)
    p.add_argument("--D", type=int, default=128)
    p.add_argument("--S", type=int, default=16)
    a = p.parse_args()
    main(HQ=a.HQ, H=a.H, D=a.D, S=a.S)
