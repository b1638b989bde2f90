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
* ``dkv="gather"`` (default): atomic-free and deterministic.  fp32 atomics run at ~1.2 TB/s
  chip-wide (they execute past the per-XCD L2s), and the scatter moves S*topk*576*4 bytes
  (19 GB at the reference shape: 16 ms).  Instead ``sparse_mla_bwd_dkv_contrib`` writes every
  (token, slot) partial row once, bf16, with plain coalesced stores (half the bytes, at HBM
  speed), the selected indices are sorted once (``torch.sort``: the inverse index, a CSR of
  the (token, slot) pairs that picked each KV row) and ``sparse_mla_bwd_dkv_reduce`` sums each
  KV row's partials in fp32 in a fixed order -- every dKV row written exactly once.
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
                    # the mask selects the exponent (exp2(-inf) = 0): no per-element branch
                    pv = T.exp2(T.if_then_else(ok, s[h, r] * scale - lse[h], -T.infinity(accum)))
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


@tilelang.jit(pass_configs=FAST_MATH)
def sparse_mla_bwd_dkv_contrib(B, S, H, D, DT, topk, block_I=32, num_stages=2, threads=256, dtype="bfloat16"):
    """Contrib[(b*S + s)*topk + k, :] = (dS^T Q + P^T dO)[k] of token s's k-th selected row, bf16.

    The MFMA work of ``sparse_mla_bwd_dkv`` with the scatter replaced by a coalesced tile store
    (the partial rows of one token are contiguous); ``Contrib`` has one extra row at the end,
    zeroed by the caller, that the reduction's tail entries point at."""
    NI = topk // block_I
    accum = "float"
    NP = B * S * topk

    @T.prim_func
    def main(Q: T.Tensor([B, S, H, D + DT], dtype), dO: T.Tensor([B, S, H, D], dtype),
             P: T.Tensor([B, S, H, topk], dtype), dS: T.Tensor([B, S, H, topk], dtype),
             Contrib: T.Tensor([NP + 1, D + DT], dtype)):
        with T.Kernel(S, B, threads=threads) as (bx, bz):
            Q_s = T.alloc_shared([H, D], dtype)
            Qt_s = T.alloc_shared([H, DT], dtype)
            dO_s = T.alloc_shared([H, D], dtype)
            p_s = T.alloc_shared([H, block_I], dtype)
            ds_s = T.alloc_shared([H, block_I], dtype)
            acc = T.alloc_fragment([block_I, D], accum)
            acct = T.alloc_fragment([block_I, DT], accum)
            acc_c = T.alloc_fragment([block_I, D], dtype)
            acct_c = T.alloc_fragment([block_I, DT], dtype)
            T.copy(Q[bz, bx, :, 0:D], Q_s)
            T.copy(Q[bz, bx, :, D:D + DT], Qt_s)
            T.copy(dO[bz, bx, :, :], dO_s)
            row0 = (bz * S + bx) * topk
            for i in T.Pipelined(NI, num_stages=num_stages):
                T.copy(P[bz, bx, :, i * block_I:(i + 1) * block_I], p_s)
                T.copy(dS[bz, bx, :, i * block_I:(i + 1) * block_I], ds_s)
                T.clear(acc)
                T.clear(acct)
                T.gemm(ds_s, Q_s, acc, transpose_A=True)
                T.gemm(p_s, dO_s, acc, transpose_A=True)
                T.gemm(ds_s, Qt_s, acct, transpose_A=True)
                T.copy(acc, acc_c)
                T.copy(acct, acct_c)
                T.copy(acc_c, Contrib[row0 + i * block_I:row0 + (i + 1) * block_I, 0:D])
                T.copy(acct_c, Contrib[row0 + i * block_I:row0 + (i + 1) * block_I, D:D + DT])

    return main


# the reduction's row ids come from Order / Offs built by inverse_index (every entry a valid
# Contrib row by construction): no per-element bounds selects, so the row loads vectorise
_NO_SAFE = {**FAST_MATH, tilelang.PassConfigKey.TL_DISABLE_SAFE_MEMORY_ACCESS: True}


@tilelang.jit(pass_configs=_NO_SAFE)
def sparse_mla_bwd_dkv_reduce(B, SKV, NP, D, DT, block_R=32, threads=256, dtype="bfloat16"):
    """dKV[b, j, 0, :] = sum of Contrib rows Order[Offs[key] : Offs[key + 1]], key = b*(SKV+1) + j,
    fp32, in index order (deterministic).  ``Order`` is padded with ``block_R`` entries equal to
    ``NP`` (Contrib's zero row), so a partial last tile reads zeros instead of branching.  The
    latent (D) and rope (DT) columns are separate register tiles (thread-divisible shapes)."""
    NK = B * (SKV + 1)

    @T.prim_func
    def main(Contrib: T.Tensor([NP + 1, D + DT], dtype), Order: T.Tensor([NP + block_R], "int32"),
             Offs: T.Tensor([NK + 1], "int32"), dKV: T.Tensor([B, SKV, 1, D + DT], "float32")):
        with T.Kernel(SKV, B, threads=threads) as (j, bz):
            pos = T.alloc_shared([block_R], "int32")
            acc = T.alloc_fragment([block_R, D], "float32")
            acct = T.alloc_fragment([block_R, DT], "float32")
            red = T.alloc_fragment([D], "float32")
            redt = T.alloc_fragment([DT], "float32")
            lo = T.alloc_var("int32")
            hi = T.alloc_var("int32")
            lo = Offs[bz * (SKV + 1) + j]
            hi = Offs[bz * (SKV + 1) + j + 1]
            T.clear(acc)
            T.clear(acct)
            for it in T.serial(T.ceildiv(hi - lo, block_R)):
                for r in T.Parallel(block_R):
                    pos[r] = T.if_then_else(lo + it * block_R + r < hi, Order[lo + it * block_R + r], NP)
                for r, c in T.Parallel(block_R, D, coalesced_width=8):
                    acc[r, c] += T.Cast("float32", Contrib[pos[r], c])
                for r, c in T.Parallel(block_R, DT, coalesced_width=8):
                    acct[r, c] += T.Cast("float32", Contrib[pos[r], D + c])
            T.reduce_sum(acc, red, dim=0)
            T.reduce_sum(acct, redt, dim=0)
            T.copy(red, dKV[bz, j, 0, 0:D])
            T.copy(redt, dKV[bz, j, 0, D:D + DT])

    return main


def inverse_index(indices, SKV, pad):
    """(Order, Offs) of ``indices`` [B, S, 1, topk]: the flat (token, slot) positions sorted by
    selected KV row (per batch), ``Offs`` the CSR row starts over keys ``b*(SKV+1) + row``
    (invalid / padding entries go to key ``b*(SKV+1) + SKV``, which is never reduced);
    ``Order`` padded with ``pad`` entries pointing at Contrib's zero row."""
    import torch
    B, S, _, topk = indices.shape
    idx = indices[:, :, 0, :].to(torch.int64)
    idx = torch.where((idx >= 0) & (idx < SKV), idx, torch.full_like(idx, SKV))
    keys = (idx + torch.arange(B, device=idx.device)[:, None, None] * (SKV + 1)).reshape(-1)
    _, order = torch.sort(keys, stable=True)
    counts = torch.bincount(keys, minlength=B * (SKV + 1))
    offs = torch.zeros(B * (SKV + 1) + 1, dtype=torch.int64, device=idx.device)
    offs[1:] = torch.cumsum(counts, 0)
    np_ = B * S * topk
    order = torch.cat([order, torch.full((pad, ), np_, dtype=torch.int64, device=idx.device)])
    return order.to(torch.int32), offs.to(torch.int32)


_KERNELS = {}


GATHER_BUDGET_BYTES = 4 << 30        # host (CPU target) budget
GATHER_BUDGET_FREE_FRACTION = 0.25   # on the GPU: a quarter of the free HBM (288 GB per MI355X)


def _gather_budget(dev):
    import torch
    if dev.type != "cuda":
        return GATHER_BUDGET_BYTES
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free * GATHER_BUDGET_FREE_FRACTION)


def sparse_mla_bwd(q, kv, o, do, indices, lse, sm_scale=None, target=None, dkv="gather",
                   gather_budget_bytes=None):
    """(dQ, dKV fp32) for the sparse MLA forward (tilelang.ops.dsa.sparse_mla_fwd).
    ``dkv``: "gather" (bf16 partial rows + sorted-index reduction, deterministic) or "atomic"
    (fp32 atomic scatter).

    The gather path holds one bf16 partial row per (token, slot): B*S*topk*576*2 bytes (4.8 GB
    at S=4096, topk=2048) plus a sort of B*S*topk keys.  Past ``gather_budget_bytes`` (default: a
    quarter of the device's free memory; a fixed 4 GiB had sent the reference shape to the atomic
    path, 9.3 -> 19.9 ms) it falls back to the atomic path, whose footprint is the O(SKV*576) fp32
    dKV alone.  Numerics: each partial row is rounded to bf16 before the fp32 sum (the atomic path
    adds fp32 partials), an extra ~2^-9 relative error per partial that averages out over the rows
    a KV row collects;
    tests/test_examples_cpu.py and test_gpu_examples_misc.py check both paths against fp32."""
    import torch
    B, S, H, DQK = q.shape
    SKV = kv.shape[1]
    D = o.shape[-1]
    DT = DQK - D
    topk = indices.shape[-1]
    tgt = target or ("cpu" if q.device.type == "cpu" else "hip")

    def k_(impl, *args, **kw):
        key = (id(impl), args, tuple(sorted(kw.items())), tgt)
        if key not in _KERNELS:  # building + hashing the program costs ms of host time per call
            _KERNELS[key] = tilelang.compile(impl.get_tir(*args, **kw), out_idx=impl.out_idx, target=tgt,
                                             pass_configs=getattr(impl, "pass_configs", None))
        return _KERNELS[key]

    delta = k_(sparse_mla_bwd_preprocess, B, S, H, D, dtype=_dt(q))(o, do)
    dq, p, ds = k_(sparse_mla_bwd_dq, B, S, SKV, H, D, DT, topk, sm_scale, dtype=_dt(q))(q, kv, do, indices, lse,
                                                                                      delta)
    if gather_budget_bytes is None:
        gather_budget_bytes = _gather_budget(q.device)
    if dkv == "gather" and B * S * topk * DQK * q.element_size() > gather_budget_bytes:
        dkv = "atomic"
    if dkv == "atomic":
        dkv_ = torch.zeros(B, SKV, 1, DQK, dtype=torch.float32, device=q.device)
        k_(sparse_mla_bwd_dkv, B, S, SKV, H, D, DT, topk, dtype=_dt(q))(q, do, indices, p, ds, dkv_)
        return dq, dkv_
    NP, R = B * S * topk, 32
    contrib = torch.empty(NP + 1, DQK, dtype=q.dtype, device=q.device)
    contrib[NP].zero_()
    k_(sparse_mla_bwd_dkv_contrib, B, S, H, D, DT, topk, dtype=_dt(q))(q, do, p, ds, contrib)
    order, offs = inverse_index(indices, SKV, R)
    dkv_ = torch.empty(B, SKV, 1, DQK, dtype=torch.float32, device=q.device)
    k_(sparse_mla_bwd_dkv_reduce, B, SKV, NP, D, DT, R, dtype=_dt(q))(contrib, order, offs, dkv_)
    return dq, dkv_


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
    ga = sparse_mla_bwd(qs, kvs, os_, dos, ids, ls, dkv="atomic")[1]
    torch.testing.assert_close(gkv, ga, rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    flop = 2 * S * H * topk * (512 + 576 + 576 + 576 + 512)
    for mode in ("gather", "atomic"):
        ms = do_bench(lambda: sparse_mla_bwd(q, kv, o, do, idx, lse, dkv=mode))
        print(f"sparse MLA bwd B{B} S{S} SKV{SKV} H{H} topk{topk} dkv={mode}: {ms:.3f} ms, "
              f"{flop / ms * 1e-9:.1f} TFLOPS", flush=True)


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--S", type=int, default=4096)
    p.add_argument("--SKV", type=int, default=8192)
    a = p.parse_args()
    main(S=a.S, SKV=a.SKV)
