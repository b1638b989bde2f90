"""Native Sparse Attention (NSA) selected-block attention, forward and decode
(reference: examples/deepseek_nsa/example_tilelang_nsa_{fwd,decode}.py).

Every query token t (position ``t + SKV - SQ``) of kv-head h attends to the ``S`` key blocks of
``block_size`` tokens listed in ``BlockIndices[b, t, h, :]`` (causal inside a block; indices
that are negative or past the token are skipped).  The ``G = HQ / H`` query heads of one kv head
share the blocks, so they form the M dimension of the MFMA tile: one block = one (token, kv
head), one wave per 16 query heads (FullRow: P stays in registers).

MI355X choices: the block offset is clamped into the tensor, so the K/V block copies are
provably in bounds and become LDS-DMA producers of ``T.Pipelined`` (masked blocks are loaded
and discarded instead of branching around the pipeline); the running max starts finite so an
all-masked first block cannot produce NaNs.  Decode is the same kernel with SQ = 1.
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(out_idx=[-1], pass_configs=FAST_MATH)
def nsa_fwd(batch, heads, seq_len, seq_len_kv, dim, is_causal=True, scale=None, block_size=64, groups=16,
            selected_blocks=16, num_stages=2, block_T=32, dtype="bfloat16", unroll=2):
    """``block_T`` rows of a selected block per pipeline step (a 64-token block in two 32-row
    steps keeps LDS at ~36 KB, so 4 blocks share a CU).  ``unroll``: the lowered main loop is
    emitted twice per trip (the LDS ring slot of each copy a constant): 2.135 -> 1.777 ms at
    B4 SQ4096 HQ64 H4 D128 S16x64 (profiles/r6/secondary_sweep.log)."""
    scale = ((1.0 / dim)**0.5 if scale is None else scale) * LOG2E
    head_kv = heads // groups
    G, BS, S, D = groups, block_size, selected_blocks, dim
    BT = min(block_T, BS)
    assert BS % BT == 0
    NT = BS // BT
    assert G % 16 == 0, "the query heads of one kv head form the MFMA M dim (multiple of 16)"
    threads = 64 * (G // 16)
    past = seq_len_kv - seq_len
    accum_dtype = "float"

    @T.prim_func
    def main(Q: T.Tensor([batch, seq_len, heads, D], dtype), K: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             V: T.Tensor([batch, seq_len_kv, head_kv, D], dtype),
             BlockIndices: T.Tensor([batch, seq_len, head_kv, S], "int32"),
             Output: T.Tensor([batch, seq_len, heads, D], dtype)):
        with T.Kernel(seq_len, batch * head_kv, threads=threads) as (bx, bz):
            Q_shared = T.alloc_shared([G, D], dtype)
            K_shared = T.alloc_shared([BT, D], dtype)
            V_shared = T.alloc_shared([BT, D], dtype)
            acc_s = T.alloc_fragment([G, BT], accum_dtype)
            acc_s_cast = T.alloc_fragment([G, BT], dtype)
            acc_o = T.alloc_fragment([G, D], accum_dtype)
            o_cast = T.alloc_fragment([G, D], dtype)
            m = T.alloc_fragment([G], accum_dtype)
            m_prev = T.alloc_fragment([G], accum_dtype)
            alpha = T.alloc_fragment([G], accum_dtype)
            l_sum = T.alloc_fragment([G], accum_dtype)
            r_sum = T.alloc_fragment([G], accum_dtype)
            b = bz // head_kv
            h = bz % head_kv
            pos = bx + past
            T.copy(Q[b, bx, h * G:(h + 1) * G, :], Q_shared)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            for i in T.Pipelined(S * NT, num_stages=num_stages, unroll=unroll):
                blk = BlockIndices[b, bx, h, i // NT]
                # clamped into the tensor, so the copies are provably in bounds (LDS-DMA)
                i_s = T.min(T.max(blk, 0), seq_len_kv // BS - 1) * BS + (i % NT) * BT
                T.copy(K[b, i_s:i_s + BT, h, :], K_shared)
                T.copy(V[b, i_s:i_s + BT, h, :], V_shared)
                for g, j in T.Parallel(G, BT):
                    ok = (blk >= 0) & (blk * BS <= pos)
                    if is_causal:
                        ok = ok & (i_s + j <= pos)
                    acc_s[g, j] = T.if_then_else(ok, 0, -T.infinity(accum_dtype))
                T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                # lazy rescale: a row keeps its max until a score beats it by 2^8 (P <= 256), so
                # the O accumulator is rescaled only on the steps where one of the lane's rows moved
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
                if rescale != 0:  # per-thread flag: a wave whose rows all kept their max skips it
                    for g, d in T.Parallel(G, D):
                        acc_o[g, d] *= alpha[g]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for g, d in T.Parallel(G, D):
                o_cast[g, d] = acc_o[g, d] / T.max(l_sum[g], 1e-30)
            T.copy(o_cast, Output[b, bx, h * G:(h + 1) * G, :])

    return main


def make_block_indices(B, SQ, SKV, H, S, block_size, device="cpu", seed=0):
    """Random distinct visible blocks per (token, kv head), padded with -1, sorted."""
    import torch
    g = torch.Generator().manual_seed(seed)
    past = SKV - SQ
    idx = torch.full((B, SQ, H, S), -1, dtype=torch.int32)
    for b in range(B):
        for t in range(SQ):
            nvis = (t + past) // block_size + 1
            for h in range(H):
                sel = torch.randperm(nvis, generator=g)[:S].int()
                idx[b, t, h, :len(sel)] = sel.sort()[0]
    return idx.to(device)


def ref_program(q, k, v, block_indices, block_size, scale=None, is_causal=True):
    """fp32 reference: q [B,SQ,HQ,D], k/v [B,SKV,H,D], block_indices [B,SQ,H,S] (-1 = none)."""
    import torch
    B, SQ, HQ, D = q.shape
    SKV, H = k.shape[1], k.shape[2]
    G = HQ // H
    scale = D**-0.5 if scale is None else scale
    past = SKV - SQ
    out = torch.zeros(B, SQ, HQ, D)
    qf, kf, vf = q.float().cpu(), k.float().cpu(), v.float().cpu()
    bi = block_indices.cpu()
    for b in range(B):
        for t in range(SQ):
            pos = t + past
            for h in range(H):
                toks = []
                for blk in bi[b, t, h].tolist():
                    if blk < 0 or blk * block_size > pos:
                        continue
                    hi = min(blk * block_size + block_size, pos + 1 if is_causal else SKV)
                    toks.extend(range(blk * block_size, hi))
                if not toks:
                    continue
                ix = torch.tensor(toks)
                s = qf[b, t, h * G:(h + 1) * G] @ kf[b, ix, h].t() * scale
                out[b, t, h * G:(h + 1) * G] = torch.softmax(s, -1) @ vf[b, ix, h]
    return out.to(q.dtype)


def main(B=4, SQ=4096, SKV=4096, HQ=64, H=4, D=128, S=16, block_size=64):
    import torch
    kernel = nsa_fwd(B, HQ, SQ, SKV, D, True, None, block_size, HQ // H, S)
    q = torch.randn(B, SQ, HQ, D, device="cuda", dtype=torch.bfloat16)
    k = torch.randn(B, SKV, H, D, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(B, SKV, H, D, device="cuda", dtype=torch.bfloat16)
    g = torch.Generator(device="cuda").manual_seed(0)
    # vectorised random block selection: top-S of random keys over the visible blocks
    nb = SKV // block_size
    vis = (torch.arange(SQ, device="cuda")[:, None] + SKV - SQ) // block_size >= torch.arange(nb, device="cuda")
    r = torch.where(vis[None, :, None, :], torch.rand(B, SQ, H, nb, device="cuda", generator=g), -1.0)
    top = r.topk(min(S, nb), -1)
    bi = torch.where(top.values >= 0, top.indices, -1).int().sort(-1)[0].contiguous()
    o = kernel(q, k, v, bi)
    sub = slice(SQ - 2, SQ)
    ref = ref_program(q[:1, sub], k[:1], v[:1], bi[:1, sub], block_size)
    torch.testing.assert_close(o[:1, sub].float().cpu(), ref.float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v, bi))
    flops = 4 * B * SQ * HQ * D * S * block_size
    print(f"NSA fwd B{B} SQ{SQ} HQ{HQ} H{H} D{D} S{S}x{block_size}: {lat:.3f} ms, {flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=4)
    p.add_argument("--seq", type=int, default=4096)
    a = p.parse_args()
    main(B=a.batch, SQ=a.seq, SKV=a.seq)
