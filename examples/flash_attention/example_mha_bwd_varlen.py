"""Variable-length (packed) FlashAttention backward (reference: examples/flash_attention/
example_gqa_bwd_tma_reduce_varlen.py).  Layout as example_mha_fwd_varlen.py: Q/O/dO
[total_q, H, D], K/V [total_k, H/G, D], prefix offsets ``cu_seqlens_q/k`` [B+1], causal masking
bottom-right aligned.

Kernels (same split as the dense backward, example_mha_bwd.py):
  flashattn_varlen_fwd_lse   forward + base-2 LSE [H, total_q]
  varlen_bwd_preprocess      Delta = rowsum(O * dO) [H, total_q]
  varlen_bwd_dkv             one workgroup per (KV tile, KV head, sequence); K/V resident in LDS,
                             the Q/dO tiles of all G query heads of the group stream through the
                             LDS-DMA pipeline: dK/dV accumulate in registers (no atomics)
  varlen_bwd_dq              one workgroup per (query tile, head, sequence): dQ = dS K in registers
Tiles that run past a sequence read the next sequence's rows (masked out) or zeros past the
tensor; stores are row-guarded so a tile never writes another sequence's gradients.
"""
import argparse

import tilelang
import tilelang.language as T

from example_mha_fwd_varlen import FAST_MATH, LOG2E, make_varlen


@tilelang.jit(out_idx=[5, 6], pass_configs=FAST_MATH)
def flashattn_varlen_fwd_lse(batch, heads, total_q, total_k, max_seqlen_q, dim, is_causal=True, groups=1,
                             block_M=128, block_N=64, threads=256, num_stages=2, dtype="bfloat16"):
    scale = (1.0 / dim)**0.5 * LOG2E
    head_kv = heads // groups
    accum = "float"

    @T.prim_func
    def main(Q: T.Tensor([total_q, heads, dim], dtype), K: T.Tensor([total_k, head_kv, dim], dtype),
             V: T.Tensor([total_k, head_kv, dim], dtype), cu_q: T.Tensor([batch + 1], "int32"),
             cu_k: T.Tensor([batch + 1], "int32"), Output: T.Tensor([total_q, heads, dim], dtype),
             LSE: T.Tensor([heads, total_q], "float32")):
        with T.Kernel(T.ceildiv(max_seqlen_q, block_M), heads, batch, threads=threads) as (bx, by, bz):
            Q_s = T.alloc_shared([block_M, dim], dtype)
            K_s = T.alloc_shared([block_N, dim], dtype)
            V_s = T.alloc_shared([block_N, dim], dtype)
            acc_s = T.alloc_fragment([block_M, block_N], accum)
            acc_s_cast = T.alloc_fragment([block_M, block_N], dtype)
            acc_o = T.alloc_fragment([block_M, dim], accum)
            m = T.alloc_fragment([block_M], accum)
            m_prev = T.alloc_fragment([block_M], accum)
            alpha = T.alloc_fragment([block_M], accum)
            l_sum = T.alloc_fragment([block_M], accum)
            r_sum = T.alloc_fragment([block_M], accum)
            o_cast = T.alloc_fragment([block_M, dim], dtype)
            q0 = cu_q[bz]
            k0 = cu_k[bz]
            q_len = cu_q[bz + 1] - q0
            k_len = cu_k[bz + 1] - k0
            off = k_len - q_len
            if bx * block_M < q_len:
                T.copy(Q[q0 + bx * block_M:q0 + (bx + 1) * block_M, by, :], Q_s)
                T.fill(acc_o, 0)
                T.fill(l_sum, 0)
                T.fill(m, -(2.0**30))
                n_kv = T.ceildiv(T.min(k_len, (bx + 1) * block_M + off), block_N) if is_causal else \
                    T.ceildiv(k_len, block_N)
                for k in T.Pipelined(n_kv, num_stages=num_stages):
                    T.copy(K[k0 + k * block_N:k0 + (k + 1) * block_N, by // groups, :], K_s)
                    T.copy(V[k0 + k * block_N:k0 + (k + 1) * block_N, by // groups, :], V_s)
                    for i, j in T.Parallel(block_M, block_N):
                        ok = k * block_N + j < k_len
                        if is_causal:
                            ok = ok & (bx * block_M + i + off >= k * block_N + j)
                        acc_s[i, j] = T.if_then_else(ok, 0, -T.infinity(accum))
                    T.gemm(Q_s, K_s, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                    T.copy(m, m_prev)
                    T.reduce_max(acc_s, m, dim=1, clear=False)
                    for i in T.Parallel(block_M):
                        alpha[i] = T.exp2((m_prev[i] - m[i]) * scale)
                    for i, j in T.Parallel(block_M, dim):
                        acc_o[i, j] *= alpha[i]
                    for i, j in T.Parallel(block_M, block_N):
                        acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m[i] * scale)
                    T.reduce_sum(acc_s, r_sum, dim=1)
                    for i in T.Parallel(block_M):
                        l_sum[i] = l_sum[i] * alpha[i] + r_sum[i]
                    T.copy(acc_s, acc_s_cast)
                    T.gemm(acc_s_cast, V_s, acc_o, policy=T.GemmWarpPolicy.FullRow)
                for i, j in T.Parallel(block_M, dim):
                    o_cast[i, j] = acc_o[i, j] / T.max(l_sum[i], 1e-30)
                for i, j in T.Parallel(block_M, dim):
                    if bx * block_M + i < q_len:
                        Output[q0 + bx * block_M + i, by, j] = o_cast[i, j]
                for i in T.Parallel(block_M):
                    if bx * block_M + i < q_len:
                        LSE[by, q0 + bx * block_M + i] = T.if_then_else(l_sum[i] > 0, m[i] * scale +
                                                                        T.log2(l_sum[i]), T.infinity("float32"))

    return main


@tilelang.jit(out_idx=[2])
def varlen_bwd_preprocess(heads, total_q, dim, blk=32, dtype="bfloat16"):

    @T.prim_func
    def main(O: T.Tensor([total_q, heads, dim], dtype), dO: T.Tensor([total_q, heads, dim], dtype),
             Delta: T.Tensor([heads, total_q], "float32")):
        with T.Kernel(heads, T.ceildiv(total_q, blk), threads=256) as (bx, by):
            acc = T.alloc_fragment([blk, dim], "float32")
            dsum = T.alloc_fragment([blk], "float32")
            for i, d in T.Parallel(blk, dim):
                r = by * blk + i
                acc[i, d] = T.if_then_else(r < total_q,
                                           T.cast(O[r, bx, d], "float32") * T.cast(dO[r, bx, d], "float32"), 0.0)
            T.reduce_sum(acc, dsum, dim=1)
            for i in T.Parallel(blk):
                if by * blk + i < total_q:
                    Delta[bx, by * blk + i] = dsum[i]

    return main


@tilelang.jit(out_idx=[8, 9], pass_configs=FAST_MATH)
def varlen_bwd_dkv(batch, heads, total_q, total_k, max_seqlen_k, dim, is_causal=True, groups=1, block_M=128,
                   block_N=64, threads=512, num_stages=2, dtype="bfloat16"):
    sm_scale = (1.0 / dim)**0.5
    scale = sm_scale * LOG2E
    head_kv = heads // groups
    accum = "float"

    @T.prim_func
    def main(Q: T.Tensor([total_q, heads, dim], dtype), K: T.Tensor([total_k, head_kv, dim], dtype),
             V: T.Tensor([total_k, head_kv, dim], dtype), dO: T.Tensor([total_q, heads, dim], dtype),
             LSE: T.Tensor([heads, total_q], "float32"), Delta: T.Tensor([heads, total_q], "float32"),
             cu_q: T.Tensor([batch + 1], "int32"), cu_k: T.Tensor([batch + 1], "int32"),
             dK: T.Tensor([total_k, head_kv, dim], dtype),
             dV: T.Tensor([total_k, head_kv, dim], dtype)):
        with T.Kernel(T.ceildiv(max_seqlen_k, block_M), head_kv, batch, threads=threads) as (by, bx, bz):
            K_s = T.alloc_shared([block_M, dim], dtype)
            V_s = T.alloc_shared([block_M, dim], dtype)
            q = T.alloc_shared([block_N, dim], dtype)
            do = T.alloc_shared([block_N, dim], dtype)
            lse_s = T.alloc_shared([block_N], accum)
            delta_s = T.alloc_shared([block_N], accum)
            qkT = T.alloc_fragment([block_M, block_N], accum)
            dsT = T.alloc_fragment([block_M, block_N], accum)
            qkT_cast = T.alloc_fragment([block_M, block_N], dtype)
            dsT_cast = T.alloc_fragment([block_M, block_N], dtype)
            dv = T.alloc_fragment([block_M, dim], accum)
            dk = T.alloc_fragment([block_M, dim], accum)
            q0 = cu_q[bz]
            k0 = cu_k[bz]
            q_len = cu_q[bz + 1] - q0
            k_len = cu_k[bz + 1] - k0
            off = k_len - q_len
            if by * block_M < k_len:
                T.copy(K[k0 + by * block_M:k0 + (by + 1) * block_M, bx, :], K_s)
                T.copy(V[k0 + by * block_M:k0 + (by + 1) * block_M, bx, :], V_s)
                T.clear(dv)
                T.clear(dk)
                # query tiles that can see this KV tile: query row i sees key j when i + off >= j
                loop_st = T.max(by * block_M - off, 0) // block_N if is_causal else 0
                n_q = T.max(T.ceildiv(q_len, block_N) - loop_st, 0)
                for it in T.Pipelined(n_q * groups, num_stages=num_stages):
                    # head clamped into range so the bounds prover keeps the Q / dO tiles LDS-DMA (the
                    # row offset may run past the sequence: buffer-resource DMA zero-fills past the tensor)
                    hq = T.max(T.min(bx * groups + it // n_q, heads - 1), 0)
                    kq = loop_st + it % n_q
                    T.copy(Q[q0 + kq * block_N:q0 + (kq + 1) * block_N, hq, :], q)
                    T.copy(dO[q0 + kq * block_N:q0 + (kq + 1) * block_N, hq, :], do)
                    # pipelined copies (issued a stage ahead; rows past total_q are guarded to 0 and
                    # masked below) instead of synchronous per-iteration loads
                    T.copy(LSE[hq, q0 + kq * block_N:q0 + (kq + 1) * block_N], lse_s)
                    T.copy(Delta[hq, q0 + kq * block_N:q0 + (kq + 1) * block_N], delta_s)
                    T.clear(qkT)
                    T.gemm(K_s, q, qkT, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                    # interior tiles (every query valid and, causal, past the diagonal) skip the mask
                    inner = ((kq + 1) * block_N <= q_len) & ((by + 1) * block_M <= k_len)
                    if is_causal:
                        inner = inner & (kq * block_N + off >= (by + 1) * block_M - 1)
                    if inner:
                        for i, j in T.Parallel(block_M, block_N):
                            qkT[i, j] = T.exp2(qkT[i, j] * scale - lse_s[j])
                    else:
                        for i, j in T.Parallel(block_M, block_N):
                            ok = (kq * block_N + j < q_len) & (by * block_M + i < k_len)
                            if is_causal:
                                ok = ok & (kq * block_N + j + off >= by * block_M + i)
                            qkT[i, j] = T.exp2(T.if_then_else(ok, qkT[i, j] * scale - lse_s[j], -T.infinity("float32")))
                    T.clear(dsT)
                    T.gemm(V_s, do, dsT, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                    T.copy(qkT, qkT_cast)
                    T.gemm(qkT_cast, do, dv, policy=T.GemmWarpPolicy.FullRow)
                    for i, j in T.Parallel(block_M, block_N):
                        dsT_cast[i, j] = qkT[i, j] * (dsT[i, j] - delta_s[j]) * sm_scale
                    T.gemm(dsT_cast, q, dk, policy=T.GemmWarpPolicy.FullRow)
                for i, d in T.Parallel(block_M, dim):
                    if by * block_M + i < k_len:
                        dK[k0 + by * block_M + i, bx, d] = dk[i, d]
                        dV[k0 + by * block_M + i, bx, d] = dv[i, d]

    return main


@tilelang.jit(out_idx=[8], pass_configs=FAST_MATH)
def varlen_bwd_dq(batch, heads, total_q, total_k, max_seqlen_q, dim, is_causal=True, groups=1, block_M=128,
                  block_N=64, threads=256, num_stages=2, dtype="bfloat16"):
    sm_scale = (1.0 / dim)**0.5
    scale = sm_scale * LOG2E
    head_kv = heads // groups
    accum = "float"

    @T.prim_func
    def main(Q: T.Tensor([total_q, heads, dim], dtype), K: T.Tensor([total_k, head_kv, dim], dtype),
             V: T.Tensor([total_k, head_kv, dim], dtype), dO: T.Tensor([total_q, heads, dim], dtype),
             LSE: T.Tensor([heads, total_q], "float32"), Delta: T.Tensor([heads, total_q], "float32"),
             cu_q: T.Tensor([batch + 1], "int32"), cu_k: T.Tensor([batch + 1], "int32"),
             dQ: T.Tensor([total_q, heads, dim], dtype)):
        n_qt = (max_seqlen_q + block_M - 1) // block_M
        with T.Kernel(heads, n_qt, batch, threads=threads) as (by, bx_raw, bz):
            bx = (n_qt - 1 - bx_raw) if is_causal else bx_raw  # causal: longest dQ rows first
            q = T.alloc_shared([block_M, dim], dtype)
            do = T.alloc_shared([block_M, dim], dtype)
            K_s = T.alloc_shared([block_N, dim], dtype)
            V_s = T.alloc_shared([block_N, dim], dtype)
            lse_s = T.alloc_shared([block_M], accum)
            delta_s = T.alloc_shared([block_M], accum)
            s = T.alloc_fragment([block_M, block_N], accum)
            dp = T.alloc_fragment([block_M, block_N], accum)
            ds_cast = T.alloc_fragment([block_M, block_N], dtype)
            dq = T.alloc_fragment([block_M, dim], accum)
            q0 = cu_q[bz]
            k0 = cu_k[bz]
            q_len = cu_q[bz + 1] - q0
            k_len = cu_k[bz + 1] - k0
            off = k_len - q_len
            if bx * block_M < q_len:
                T.copy(Q[q0 + bx * block_M:q0 + (bx + 1) * block_M, by, :], q)
                T.copy(dO[q0 + bx * block_M:q0 + (bx + 1) * block_M, by, :], do)
                for i in T.Parallel(block_M):
                    r = T.min(q0 + bx * block_M + i, total_q - 1)
                    lse_s[i] = LSE[by, r]
                    delta_s[i] = Delta[by, r]
                T.clear(dq)
                n_kv = T.ceildiv(T.min(k_len, (bx + 1) * block_M + off), block_N) if is_causal else \
                    T.ceildiv(k_len, block_N)
                for k in T.Pipelined(n_kv, num_stages=num_stages):
                    T.copy(K[k0 + k * block_N:k0 + (k + 1) * block_N, by // groups, :], K_s)
                    T.copy(V[k0 + k * block_N:k0 + (k + 1) * block_N, by // groups, :], V_s)
                    T.clear(s)
                    T.gemm(q, K_s, s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                    T.clear(dp)
                    T.gemm(do, V_s, dp, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                    inner = ((k + 1) * block_N <= k_len) & ((bx + 1) * block_M <= q_len)
                    if is_causal:
                        inner = inner & (bx * block_M + off >= (k + 1) * block_N - 1)
                    if inner:
                        for i, j in T.Parallel(block_M, block_N):
                            ds_cast[i, j] = T.exp2(s[i, j] * scale - lse_s[i]) * (dp[i, j] - delta_s[i]) * sm_scale
                    else:
                        for i, j in T.Parallel(block_M, block_N):
                            ok = (k * block_N + j < k_len) & (bx * block_M + i < q_len)
                            if is_causal:
                                ok = ok & (bx * block_M + i + off >= k * block_N + j)
                            pe = T.exp2(T.if_then_else(ok, s[i, j] * scale - lse_s[i], -T.infinity("float32")))
                            ds_cast[i, j] = pe * (dp[i, j] - delta_s[i]) * sm_scale
                    T.gemm(ds_cast, K_s, dq, policy=T.GemmWarpPolicy.FullRow)
                for i, d in T.Parallel(block_M, dim):
                    if bx * block_M + i < q_len:
                        dQ[q0 + bx * block_M + i, by, d] = dq[i, d]

    return main


def varlen_attention_bwd(q, k, v, o, lse, do, cu_q, cu_k, max_q, max_k, is_causal=True):
    H, HKV, D = q.shape[1], k.shape[1], q.shape[2]
    B = cu_q.numel() - 1
    G = H // HKV
    dt = str(q.dtype).replace("torch.", "")
    delta = varlen_bwd_preprocess(H, q.shape[0], D, dtype=dt)(o, do)
    dk, dv = varlen_bwd_dkv(B, H, q.shape[0], k.shape[0], max_k, D, is_causal, G, dtype=dt)(q, k, v, do, lse, delta,
                                                                                              cu_q, cu_k)
    dq = varlen_bwd_dq(B, H, q.shape[0], k.shape[0], max_q, D, is_causal, G, dtype=dt)(q, k, v, do, lse, delta,
                                                                                         cu_q, cu_k)
    return dq, dk, dv


class VarlenAttention:
    """``VarlenAttention.apply(q, k, v, cu_q, cu_k, max_q, max_k, causal)`` -> o, differentiable."""

    @staticmethod
    def apply(q, k, v, cu_q, cu_k, max_q, max_k, is_causal=True):
        import torch

        class _Fn(torch.autograd.Function):

            @staticmethod
            def forward(ctx, q, k, v):
                H, HKV, D = q.shape[1], k.shape[1], q.shape[2]
                dt = str(q.dtype).replace("torch.", "")
                fwd = flashattn_varlen_fwd_lse(cu_q.numel() - 1, H, q.shape[0], k.shape[0], max_q, D, is_causal,
                                               H // HKV, dtype=dt)
                o, lse = fwd(q, k, v, cu_q, cu_k)
                ctx.save_for_backward(q, k, v, o, lse)
                return o

            @staticmethod
            def backward(ctx, do):
                q, k, v, o, lse = ctx.saved_tensors
                return varlen_attention_bwd(q, k, v, o, lse, do.contiguous().to(q.dtype), cu_q, cu_k, max_q, max_k,
                                            is_causal)

        return _Fn.apply(q, k, v)


def reference_grads(q, k, v, cu_q, cu_k, do, is_causal=True):
    qr, kr, vr = (x.float().cpu().requires_grad_(True) for x in (q, k, v))
    o = _ref_fp32(qr, kr, vr, cu_q.cpu(), cu_k.cpu(), is_causal)
    o.backward(do.float().cpu())
    return o, qr.grad, kr.grad, vr.grad


def _ref_fp32(q, k, v, cu_q, cu_k, is_causal):
    import torch
    H = q.shape[1]
    G = H // k.shape[1]
    outs = []
    for b in range(len(cu_q) - 1):
        qs, qe, ks, ke = int(cu_q[b]), int(cu_q[b + 1]), int(cu_k[b]), int(cu_k[b + 1])
        qq = q[qs:qe].transpose(0, 1)
        kk = k[ks:ke].repeat_interleave(G, 1).transpose(0, 1)
        vv = v[ks:ke].repeat_interleave(G, 1).transpose(0, 1)
        s = qq @ kk.transpose(-1, -2) * q.shape[-1]**-0.5
        if is_causal:
            lq, lk = qe - qs, ke - ks
            mask = torch.arange(lq)[:, None] + (lk - lq) >= torch.arange(lk)[None, :]
            s = s.masked_fill(~mask, float("-inf"))
        outs.append((torch.softmax(s, -1).nan_to_num(0.0) @ vv).transpose(0, 1))
    return torch.cat(outs, 0)


def main(B=8, max_len=4096, H=32, G=4, D=128):
    import torch
    g = torch.Generator().manual_seed(0)
    lens = torch.randint(max_len // 4, max_len + 1, (B, ), generator=g).tolist()
    q, k, v, cu_q, cu_k = make_varlen(lens, lens, H, H // G, D, "cuda")
    fwd = flashattn_varlen_fwd_lse(B, H, q.shape[0], k.shape[0], max(lens), D, True, G)
    o, lse = fwd(q, k, v, cu_q, cu_k)
    do = torch.randn_like(o)
    from tilelang.profiler import do_bench
    varlen_attention_bwd(q, k, v, o, lse, do, cu_q, cu_k, max(lens), max(lens))
    lat = do_bench(lambda: varlen_attention_bwd(q, k, v, o, lse, do, cu_q, cu_k, max(lens), max(lens)))
    flops = sum(2.5 * 2 * 2.0 * H * L * L * D * 0.5 for L in lens)
    print(f"varlen causal attention bwd B{B} lens {min(lens)}..{max(lens)} H{H} G{G}: {lat:.3f} ms, "
          f"{flops / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--max_len", type=int, default=4096)
    a = p.parse_args()
    main(a.batch, a.max_len)
