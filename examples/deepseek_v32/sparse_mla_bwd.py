"""DeepSeek-V3.2 sparse MLA backward (reference: examples/deepseek_v32/sparse_mla_bwd.py).

Inputs as the forward (Q [B,S,H,576], KV [B,SKV,1,576], Indices [B,S,1,topk]) plus O, dO [B,S,H,512]
and the forward's base-2 LSE.  With P = exp2(S*scale - lse), V = KV[..., :512]:
    Delta = rowsum(O * dO);  dP = dO V^T;  dS = P (dP - Delta) sm_scale
    dQ = dS K;   dKV[idx] += dS^T Q  (+ P^T dO on the first 512 columns)
MI355X decomposition (LDS is 160 KB, so Q, dO and a KV tile cannot all stay resident):
* ``sparse_mla_bwd_dq``: one block per (token, 64-head slice), 4 waves x 16 heads (FullRow).
  The selected KV rows are gathered with ``T.gather_rows`` (LDS-DMA, one tile ahead); Q and dO
  comes from LDS, dO is a register A operand; dS stays in registers as the A operand of
  dQ += dS K; P and dS
  (bf16) are written out for the second kernel.
* ``sparse_mla_bwd_dkv``: one block per token keeps Q and dO in LDS (138 KB) and walks its
  ``topk`` rows in 32-row tiles: acc = dS^T Q + P^T dO on MFMA, then fp32 atomics scatter
  the 32 x 576 partial into dKV at the selected rows (different tokens select the same rows),
  staged through LDS so each wave atomic covers 64 consecutive floats of one row.
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(out_idx=[2], pass_configs=FAST_MATH)
def sparse_mla_bwd_preprocess(B, S, H, D=512, block=32, dtype="bfloat16"):
    """Delta[b, s, h] = sum_d O * dO."""

    @T.prim_func
    def main(O: T.Tensor([B, S, H, D], dtype), dO: T.Tensor([B, S, H, D], dtype),
             Delta: T.Tensor([B, S, H], "float32")):
        with T.Kernel(T.ceildiv(H, block), S, B, threads=256) as (bh, bs, bb):
            o = T.alloc_fragment([block, D], "float32")
            do = T.alloc_fragment([block, D], "float32")
            acc = T.alloc_fragment([block], "float32")
            T.copy(O[bb, bs, bh * block:(bh + 1) * block, :], o)
            T.copy(dO[bb, bs, bh * block:(bh + 1) * block, :], do)
            for i, j in T.Parallel(block, D):
                o[i, j] = o[i, j] * do[i, j]
            T.reduce_sum(o, acc, dim=1)
            T.copy(acc, Delta[bb, bs, bh * block:(bh + 1) * block])

    return main


@tilelang.jit(out_idx=[6, 7, 8], pass_configs=FAST_MATH)
def sparse_mla_bwd_dq(B, S, SKV, H, D, DT, topk, sm_scale=None, block_I=32, num_stages=2, dtype="bfloat16"):
    """Q is read from LDS (not registers) and KV tiles are 32 rows: with dO (64) and the dQ
    accumulator (144 registers per lane) that fits the register file without spilling."""
    if sm_scale is None:
        sm_scale = (D + DT)**-0.5
    scale = sm_scale * LOG2E
    H_blk = min(64, max(16, H))
    assert H % H_blk == 0 and topk % block_I == 0
    threads = 64 * (H_blk // 16)
    NI = topk // block_I
    past = SKV - S
    accum = "float"

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, D + DT], dtype), KV: T.Tensor([B, SKV, 1, D + DT], dtype),
             dO: T.Tensor([B, S, H, D], dtype), Indices: T.Tensor([B, S, 1, topk], "int32"),
             Lse: T.Tensor([B, S, H], accum), Delta: T.Tensor([B, S, H], accum),
             dQ: T.Tensor([B, S, H, D + DT], dtype), Pout: T.Tensor([B, S, H, topk], dtype),
             dSout: T.Tensor([B, S, H, topk], dtype)):
        with T.Kernel(S, H // H_blk, B, threads=threads) as (bx, by, bz):
            h0 = by * H_blk
            Q_frag = T.alloc_shared([H_blk, D], dtype)
            Qt_frag = T.alloc_shared([H_blk, DT], dtype)
            dO_frag = T.alloc_fragment([H_blk, D], dtype)
            KV_s = T.alloc_shared([block_I, D], dtype)
            Kt_s = T.alloc_shared([block_I, DT], dtype)
            idx_s = T.alloc_shared([block_I], "int32")
            s = T.alloc_fragment([H_blk, block_I], accum)
            dp = T.alloc_fragment([H_blk, block_I], accum)
            ds_cast = T.alloc_fragment([H_blk, block_I], dtype)
            p_cast = T.alloc_fragment([H_blk, block_I], dtype)
            dq = T.alloc_fragment([H_blk, D], accum)
            dqt = T.alloc_fragment([H_blk, DT], accum)
            lse = T.alloc_fragment([H_blk], accum)
            delta = T.alloc_fragment([H_blk], accum)
            T.copy(Q[bz, bx, h0:h0 + H_blk, 0:D], Q_frag)
            T.copy(Q[bz, bx, h0:h0 + H_blk, D:D + DT], Qt_frag)
            T.copy(dO[bz, bx, h0:h0 + H_blk, :], dO_frag)
            T.copy(Lse[bz, bx, h0:h0 + H_blk], lse)
            T.copy(Delta[bz, bx, h0:h0 + H_blk], delta)
            T.clear(dq)
            T.clear(dqt)
            for i in T.Pipelined(NI, num_stages=num_stages):
                T.gather_rows(KV[bz, :, 0, 0:D], Indices[bz, bx, 0, i * block_I:(i + 1) * block_I], KV_s)
                T.gather_rows(KV[bz, :, 0, D:D + DT], Indices[bz, bx, 0, i * block_I:(i + 1) * block_I], Kt_s)
                T.copy(Indices[bz, bx, 0, i * block_I:(i + 1) * block_I], idx_s)
                T.clear(s)
                T.gemm(Q_frag, KV_s, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.gemm(Qt_frag, Kt_s, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                T.clear(dp)
                T.gemm(dO_frag, KV_s, dp, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                for h, r in T.Parallel(H_blk, block_I):
                    ok = (idx_s[r] <= bx + past) & (idx_s[r] >= 0)
                    pv = T.if_then_else(ok, T.exp2(s[h, r] * scale - lse[h]), 0.0)
                    p_cast[h, r] = pv
                    ds_cast[h, r] = pv * (dp[h, r] - delta[h]) * sm_scale
                T.copy(p_cast, Pout[bz, bx, h0:h0 + H_blk, i * block_I:(i + 1) * block_I])
                T.copy(ds_cast, dSout[bz, bx, h0:h0 + H_blk, i * block_I:(i + 1) * block_I])
                T.gemm(ds_cast, KV_s, dq, policy=T.GemmWarpPolicy.FullRow)
                T.gemm(ds_cast, Kt_s, dqt, policy=T.GemmWarpPolicy.FullRow)
            T.copy(dq, dQ[bz, bx, h0:h0 + H_blk, 0:D])
            T.copy(dqt, dQ[bz, bx, h0:h0 + H_blk, D:D + DT])

    return main


@tilelang.jit(pass_configs=FAST_MATH)
def sparse_mla_bwd_dkv(B, S, SKV, H, D, DT, topk, block_I=32, block_C=64, threads=256, dtype="bfloat16"):
    """dKV[b, idx, 0, :] += dS^T Q (+ P^T dO on [0, D)); dKV is fp32 and zeroed by the caller.

    The MFMA accumulator is scattered in ``block_C``-column slices staged through LDS so every
    wave-wide fp32 atomic covers 64 consecutive floats of ONE selected row (two cache lines);
    atomics issued straight from the MFMA layout touch 16+ lines per instruction (measured at the
    reference shape: 61 ms -> 16 ms for this kernel)."""
    NI = topk // block_I
    assert D % block_C == 0 and DT <= block_C
    NC = D // block_C
    accum = "float"

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, D + DT], dtype), dO: T.Tensor([B, S, H, D], dtype),
             Indices: T.Tensor([B, S, 1, topk], "int32"), P: T.Tensor([B, S, H, topk], dtype),
             dS: T.Tensor([B, S, H, topk], dtype), dKV: T.Tensor([B, SKV, 1, D + DT], accum)):
        with T.Kernel(S, B, threads=threads) as (bx, bz):
            Q_s = T.alloc_shared([H, D], dtype)
            Qt_s = T.alloc_shared([H, DT], dtype)
            dO_s = T.alloc_shared([H, D], dtype)
            p_s = T.alloc_shared([H, block_I], dtype)
            ds_s = T.alloc_shared([H, block_I], dtype)
            idx_s = T.alloc_shared([block_I], "int32")
            stage = T.alloc_shared([block_I, block_C], accum)
            acc = T.alloc_fragment([block_I, D], accum)
            acct = T.alloc_fragment([block_I, DT], accum)
            T.copy(Q[bz, bx, :, 0:D], Q_s)
            T.copy(Q[bz, bx, :, D:D + DT], Qt_s)
            T.copy(dO[bz, bx, :, :], dO_s)
            for i in T.Pipelined(NI, num_stages=1):
                T.copy(P[bz, bx, :, i * block_I:(i + 1) * block_I], p_s)
                T.copy(dS[bz, bx, :, i * block_I:(i + 1) * block_I], ds_s)
                T.copy(Indices[bz, bx, 0, i * block_I:(i + 1) * block_I], idx_s)
                T.clear(acc)
                T.clear(acct)
                T.gemm(ds_s, Q_s, acc, transpose_A=True)
                T.gemm(p_s, dO_s, acc, transpose_A=True)
                T.gemm(ds_s, Qt_s, acct, transpose_A=True)
                for c in list(range(NC)):  # trace-time unrolled: static sub-tile bounds
                    T.copy(acc[:, c * block_C:(c + 1) * block_C], stage)
                    for r, j in T.Parallel(block_I, block_C, coalesced_width=1):  # lane j -> column j
                        if (idx_s[r] >= 0) & (idx_s[r] < SKV):
                            T.atomic_add(dKV[bz, idx_s[r], 0, c * block_C + j], stage[r, j])
                T.copy(acct, stage[:, 0:DT])
                for r, j in T.Parallel(block_I, DT, coalesced_width=1):
                    if (idx_s[r] >= 0) & (idx_s[r] < SKV):
                        T.atomic_add(dKV[bz, idx_s[r], 0, D + j], stage[r, j])

    return main


def sparse_mla_bwd(q, kv, o, do, indices, lse, sm_scale=None, target=None):
    """(dQ, dKV fp32) for the sparse MLA forward (tilelang.ops.dsa.sparse_mla_fwd)."""
    import torch
    B, S, H, DQK = q.shape
    SKV = kv.shape[1]
    D = o.shape[-1]
    DT = DQK - D
    topk = indices.shape[-1]
    tgt = target or ("cpu" if q.device.type == "cpu" else "hip")

    def k_(impl, *args, **kw):
        return tilelang.compile(impl.get_tir(*args, **kw), out_idx=impl.out_idx, target=tgt)

    delta = k_(sparse_mla_bwd_preprocess, B, S, H, D, dtype=_dt(q))(o, do)
    dq, p, ds = k_(sparse_mla_bwd_dq, B, S, SKV, H, D, DT, topk, sm_scale, dtype=_dt(q))(q, kv, do, indices, lse,
                                                                                      delta)
    dkv = torch.zeros(B, SKV, 1, DQK, dtype=torch.float32, device=q.device)
    k_(sparse_mla_bwd_dkv, B, S, SKV, H, D, DT, topk, dtype=_dt(q))(q, do, indices, p, ds, dkv)
    return dq, dkv


def _dt(t):
    import torch
    return {torch.bfloat16: "bfloat16", torch.float16: "float16"}[t.dtype]


def ref_bwd(q, kv, do, indices, D=512, sm_scale=None):
    """fp32 autograd reference of the sparse MLA forward."""
    import torch
    B, S, H, DQ = q.shape
    SKV = kv.shape[1]
    past = SKV - S
    sm_scale = DQ**-0.5 if sm_scale is None else sm_scale
    qf = q.float().detach().cpu().requires_grad_()
    kf = kv.float().detach().cpu().requires_grad_()
    idx = indices.long().cpu()[:, :, 0]                       # [B, S, topk]
    pos = torch.arange(S)[None, :, None] + past
    ok = (idx >= 0) & (idx <= pos) & (idx < SKV)
    g = torch.stack([kf[b, idx[b].clamp(0, SKV - 1), 0] for b in range(B)])   # [B, S, topk, DQ]
    sc = torch.einsum("bshd,bstd->bsht", qf, g) * sm_scale
    sc = sc.masked_fill(~ok[:, :, None, :], float("-inf"))
    o = torch.einsum("bsht,bstd->bshd", torch.softmax(sc, -1), g[..., :D])
    o.backward(do.float().cpu())
    return qf.grad, kf.grad


def main(B=1, S=4096, SKV=8192, H=64, topk=2048):
    import time

    import torch
    from tilelang.ops.dsa import sparse_mla_fwd
    q = (torch.randn(B, S, H, 576, device="cuda") / 10).to(torch.bfloat16)
    kv = (torch.randn(B, SKV, 1, 576, device="cuda") / 10).to(torch.bfloat16)
    do = torch.randn(B, S, H, 512, device="cuda", dtype=torch.bfloat16)
    past = SKV - S
    r = torch.rand(S, SKV, device="cuda")
    pos = torch.arange(S, device="cuda")[:, None] + past
    r = torch.where(torch.arange(SKV, device="cuda")[None, :] <= pos, r, torch.full_like(r, -1.0))
    idx = r.topk(topk, dim=-1).indices.int()
    idx = torch.where(torch.gather(r, 1, idx.long()) >= 0, idx, torch.full_like(idx, SKV)).view(B, S, 1, topk)
    o, lse = sparse_mla_fwd(B, S, SKV, H, 512, 64, topk)(q, kv, idx)
    dq, dkv = sparse_mla_bwd(q, kv, o, do, idx, lse)
    torch.cuda.synchronize()
    # correctness on a few tokens (the reference needs all tokens for dKV: use a small problem)
    Bs, Ss, SKVs, ts = 1, 64, 256, 128
    qs, kvs, dos = q[:, :Ss].contiguous(), kv[:, :SKVs].contiguous(), do[:, :Ss].contiguous()
    rs = torch.rand(Ss, SKVs, device="cuda")
    ps = torch.arange(Ss, device="cuda")[:, None] + SKVs - Ss
    rs = torch.where(torch.arange(SKVs, device="cuda")[None, :] <= ps, rs, torch.full_like(rs, -1.0))
    ids = rs.topk(ts, -1).indices.int()
    ids = torch.where(torch.gather(rs, 1, ids.long()) >= 0, ids, torch.full_like(ids, SKVs)).view(1, Ss, 1, ts)
    os_, ls = sparse_mla_fwd(Bs, Ss, SKVs, H, 512, 64, ts)(qs, kvs, ids)
    gq, gkv = sparse_mla_bwd(qs, kvs, os_, dos, ids, ls)
    rq, rkv = ref_bwd(qs, kvs, dos, ids)
    torch.testing.assert_close(gq.float().cpu(), rq, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(gkv.cpu(), rkv, rtol=3e-2, atol=3e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    ms = do_bench(lambda: sparse_mla_bwd(q, kv, o, do, idx, lse))
    flop = 2 * S * H * topk * (512 + 576 + 576 + 576 + 512)
    print(f"sparse MLA bwd B{B} S{S} SKV{SKV} H{H} topk{topk}: {ms:.3f} ms, {flop / ms * 1e-9:.1f} TFLOPS")
    t = time.time()


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--S", type=int, default=4096)
    p.add_argument("--SKV", type=int, default=8192)
    a = p.parse_args()
    main(S=a.S, SKV=a.SKV)
