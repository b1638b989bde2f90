"""DeepSeek-V3.2 sparse MLA forward (DSA) (reference: examples/deepseek_v32/sparse_mla_fwd.py).

Every query token attends only to its ``topk`` selected latent-KV rows (chosen by the lightning
indexer).  Q is [B, S, H, D + D_tail] (D = 512 latent, D_tail = 64 rope), KV is
[B, S_kv, G, D + D_tail], Indices [B, S, G, topk] (entries > the query position, e.g. the
padding value S_kv, are masked -- causal).  MI355X schedule: one block per (query token,
64-head slice, batch*group); each step gathers ``block_I`` selected KV rows into LDS
(data-dependent row gather), runs S = Q KV^T (+ the rope tail) and O += P KV on MFMA with the
64 heads as M, and the online softmax in registers -- heads play the role of query rows, so a
single query token already gives a full MFMA tile.
"""
import argparse

import tilelang
import tilelang.language as T

LOG2E = 1.44269504


@tilelang.jit(out_idx=[3, 4])
def sparse_mla_fwd(batch, seq_len, seq_len_kv, heads, dim, tail_dim, topk, kv_group=1, sm_scale=None, block_I=64,
                   threads=256, dtype="bfloat16"):
    assert topk % block_I == 0
    if sm_scale is None:
        sm_scale = (1.0 / (dim + tail_dim))**0.5
    scale = sm_scale * LOG2E
    accum_dtype = "float"
    G = kv_group
    H = heads // G
    H_blk = min(64, max(16, H))
    assert H % H_blk == 0 or H < 16
    n_hblk = max(1, H // H_blk)
    valid_h = min(H, H_blk)
    D, DT = dim, tail_dim
    NI = topk // block_I
    past = seq_len_kv - seq_len

    @T.prim_func
    def main(Q: T.Tensor([batch, seq_len, heads, D + DT], dtype), KV: T.Tensor([batch, seq_len_kv, G, D + DT], dtype),
             Indices: T.Tensor([batch, seq_len, G, topk], "int32"), Output: T.Tensor([batch, seq_len, heads, D], dtype),
             Lse: T.Tensor([batch, seq_len, heads], accum_dtype)):
        with T.Kernel(seq_len, n_hblk, batch * G, threads=threads) as (bx, by, bz):
            b = bz // G
            g = bz % G
            h0 = g * H + by * H_blk
            Q_shared = T.alloc_shared([H_blk, D], dtype)
            Qt_shared = T.alloc_shared([H_blk, DT], dtype)
            KV_shared = T.alloc_shared([block_I, D], dtype)
            Kt_shared = T.alloc_shared([block_I, DT], dtype)
            valid = T.alloc_shared([block_I], "int32")
            acc_s = T.alloc_fragment([H_blk, block_I], accum_dtype)
            acc_s_cast = T.alloc_fragment([H_blk, block_I], dtype)
            acc_o = T.alloc_fragment([H_blk, D], accum_dtype)
            o_cast = T.alloc_fragment([H_blk, D], dtype)
            m_cur = T.alloc_fragment([H_blk], accum_dtype)
            m_prev = T.alloc_fragment([H_blk], accum_dtype)
            alpha = T.alloc_fragment([H_blk], accum_dtype)
            l_sum = T.alloc_fragment([H_blk], accum_dtype)
            r_sum = T.alloc_fragment([H_blk], accum_dtype)

            T.clear(Q_shared)
            T.clear(Qt_shared)
            T.copy(Q[b, bx, h0:h0 + valid_h, 0:D], Q_shared[0:valid_h, :])
            T.copy(Q[b, bx, h0:h0 + valid_h, D:D + DT], Qt_shared[0:valid_h, :])
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m_cur, -(2.0**30))
            for i in T.serial(NI):
                # gather the selected latent rows (masked rows read row 0 and are discarded)
                for r in T.Parallel(block_I):
                    idx = Indices[b, bx, g, i * block_I + r]
                    valid[r] = T.if_then_else((idx <= bx + past) & (idx >= 0), 1, 0)
                for r, d in T.Parallel(block_I, D):
                    idx = Indices[b, bx, g, i * block_I + r]
                    KV_shared[r, d] = KV[b, T.if_then_else((idx <= bx + past) & (idx >= 0), idx, 0), g, d]
                for r, d in T.Parallel(block_I, DT):
                    idx = Indices[b, bx, g, i * block_I + r]
                    Kt_shared[r, d] = KV[b, T.if_then_else((idx <= bx + past) & (idx >= 0), idx, 0), g, D + d]
                for h, r in T.Parallel(H_blk, block_I):
                    acc_s[h, r] = T.if_then_else(valid[r] == 1, 0, -T.infinity(accum_dtype))
                T.gemm(Q_shared, KV_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.gemm(Qt_shared, Kt_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.copy(m_cur, m_prev)
                T.reduce_max(acc_s, m_cur, dim=1, clear=False)
                for h in T.Parallel(H_blk):
                    alpha[h] = T.exp2((m_prev[h] - m_cur[h]) * scale)
                for h, r in T.Parallel(H_blk, block_I):
                    acc_s[h, r] = T.exp2(acc_s[h, r] * scale - m_cur[h] * scale)
                T.reduce_sum(acc_s, r_sum, dim=1)
                for h in T.Parallel(H_blk):
                    l_sum[h] = l_sum[h] * alpha[h] + r_sum[h]
                for h, d in T.Parallel(H_blk, D):
                    acc_o[h, d] *= alpha[h]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, KV_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for h, d in T.Parallel(H_blk, D):
                o_cast[h, d] = acc_o[h, d] / l_sum[h]
            for h in T.Parallel(H_blk):
                l_sum[h] = T.log2(l_sum[h]) + m_cur[h] * scale
            T.copy(o_cast[0:valid_h, :], Output[b, bx, h0:h0 + valid_h, :])
            T.copy(l_sum[0:valid_h], Lse[b, bx, h0:h0 + valid_h])

    return main


def ref_program(q, kv, indices, dim=512, sm_scale=None):
    """fp32 reference: q [B,S,H,D+T], kv [B,SKV,G,D+T], indices [B,S,G,topk] (> query pos = masked)."""
    import torch
    B, S, H, DQ = q.shape
    _, SKV, G, _ = kv.shape
    past = SKV - S
    sm_scale = DQ**-0.5 if sm_scale is None else sm_scale
    qf, kf = q.float(), kv.float()
    out = torch.zeros(B, S, H, dim)
    hpg = H // G
    for b in range(B):
        for s in range(S):
            for g in range(G):
                idx = indices[b, s, g].long()
                ok = (idx <= s + past) & (idx >= 0)
                sel = idx[ok]
                k = kf[b, sel, g]                        # [n, DQ]
                sc = qf[b, s, g * hpg:(g + 1) * hpg] @ k.t() * sm_scale
                p = torch.softmax(sc, -1)
                out[b, s, g * hpg:(g + 1) * hpg] = p @ k[:, :dim]
    return out.to(q.dtype)


def make_indices(B, S, SKV, G, topk, device="cpu", seed=0):
    import torch
    g = torch.Generator().manual_seed(seed)
    past = SKV - S
    idx = torch.full((B, S, G, topk), SKV, dtype=torch.int32)
    for b in range(B):
        for s in range(S):
            for gg in range(G):
                n = min(topk, s + past + 1)
                idx[b, s, gg, :n] = torch.randperm(s + past + 1, generator=g)[:n].int()
    return idx.to(device)


def main(B=1, S=1024, SKV=4096, H=128, DQK=576, DV=512, topk=2048):
    import torch
    kernel = sparse_mla_fwd(B, S, SKV, H, DV, DQK - DV, topk)
    q = torch.randn(B, S, H, DQK, device="cuda", dtype=torch.bfloat16)
    kv = torch.randn(B, SKV, 1, DQK, device="cuda", dtype=torch.bfloat16)
    idx = make_indices(B, S, SKV, 1, topk, "cuda")
    o, lse = kernel(q, kv, idx)
    sub = slice(S - 4, S)
    ref = ref_program(q[:, sub].cpu(), kv.cpu(), idx[:, sub].cpu() - 0, DV)
    torch.testing.assert_close(o[:, sub].float().cpu(), ref.float(), rtol=3e-2, atol=3e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, kv, idx))
    print(f"sparse MLA fwd: {lat:.3f} ms, {B * S * (DQK + DV) * topk * 2 * H / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--S", type=int, default=1024)
    p.add_argument("--SKV", type=int, default=4096)
    p.add_argument("--topk", type=int, default=2048)
    a = p.parse_args()
    main(S=a.S, SKV=a.SKV, topk=a.topk)
