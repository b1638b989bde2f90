"""GQA attention with a learned per-head sink, causal, optional sliding window (bhsd layout)
(reference: examples/attention_sink/example_gqa_sink_fwd_bhsd_wgmma_pipelined.py, the gpt-oss
attention; the reference's headline attention number -- 497 TFLOPS on H800 for b1 h64 kvh8
s4096 d128 -- is this kernel).

softmax is taken over [scores, sink]: the sink adds exp(sink - max) to each row's normaliser
and contributes nothing to the output.  MI355X schedule:

* one block per (head, 256-query tile, batch), 8 waves (FullRow: each wave owns 32 query rows
  of S = Q K^T, so row max/sum are in-wave shuffles and P feeds the P V MFMA from registers);
* K/V tiles stream through the 2-stage LDS-DMA ring;
* causal masking is applied only on the diagonal tiles: the KV loop is split into an unmasked
  main loop and a short masked tail, so the main loop has no per-element selects;
* query tiles are issued longest-first across ALL heads (grid = (heads, q-tiles) with the
  tile index reversed; the q-tile axis slowest -- across batches too -- when there are <= 4),
  so the tail of the grid is the cheap tiles (causal work is
  triangular; measured 0.75 -> see docs/RESULTS.md).
"""
import argparse
from typing import Optional

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(out_idx=[3], pass_configs=FAST_MATH)
def flashattn_sink(batch, heads, seq_q, seq_kv, dim, groups=1, window_size=None, sm_scale=None, block_M=256,
                   block_N=64, num_stages=2, threads=512, dtype="bfloat16", causal=True, lazy_rescale=True,
                   impl="staged", fold=True):
    """``lazy_rescale``: rows keep their running max until a score exceeds it by 2^8 (O is
    rescaled only then, per wave), see example_mha_fwd.py.

    Without a sliding window the kernel is the staged FA of
    examples/flash_attention/example_mha_fwd_pipelined.py with its ``sink`` term (Q in registers,
    QK^T(t) next to PV(t-1), softmax row sums on the matrix cores, diagonal-only masks); the
    windowed form keeps the split-loop schedule below.  ``fold``: the staged kernel's ``fold_max``
    schedule (running max as the QK^T accumulator init) with ``skip_masked`` (diagonal-tile waves
    that see no key skip their MFMAs)."""
    if window_size is None and seq_kv % block_N == 0 and impl == "staged":
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "flash_attention"))
        from example_mha_fwd_pipelined import flashattn_pipelined
        return flashattn_pipelined.get_tir(batch, heads, seq_q, dim, causal, groups, block_M, block_N, threads,
                                           num_stages, dtype, lazy_rescale, True, seq_kv=seq_kv, layout="bhsd",
                                           sum_mfma=True, sink=True, sm_scale=sm_scale, fold_max=fold,
                                           skip_masked=fold)
    if window_size is not None:
        assert window_size % block_N == 0, "window_size must be divisible by block_N"
    if sm_scale is None:
        sm_scale = (1.0 / dim)**0.5
    scale = sm_scale * LOG2E
    head_kv = heads // groups
    q_shape = [batch, heads, seq_q, dim]
    kv_shape = [batch, head_kv, seq_kv, dim]
    accum_dtype = "float"
    past_len = seq_kv - seq_q
    assert past_len >= 0
    n_qt = (seq_q + block_M - 1) // block_M

    @T.macro
    def step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, scores_max, scores_max_prev,
             scores_scale, scores_sum, logsum, k, qt, by, bz, masked):
        T.copy(K[bz, by // groups, k * block_N:(k + 1) * block_N, :], K_shared)
        if masked:
            for i, j in T.Parallel(block_M, block_N):
                q_idx = qt * block_M + i + past_len
                k_idx = k * block_N + j
                if window_size is not None:
                    acc_s[i, j] = T.if_then_else((q_idx >= k_idx) & (q_idx < k_idx + window_size), 0,
                                                 -T.infinity(accum_dtype))
                else:
                    acc_s[i, j] = T.if_then_else(((q_idx >= k_idx) | (not causal)) & (k_idx < seq_kv), 0,
                                                 -T.infinity(accum_dtype))
        else:
            T.clear(acc_s)
        T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
        T.copy(V[bz, by // groups, k * block_N:(k + 1) * block_N, :], V_shared)
        T.copy(scores_max, scores_max_prev)
        if lazy_rescale:
            # running max starts finite (-2^30), so fully masked rows never see inf - inf
            T.reduce_max(acc_s, scores_max_prev, dim=1, clear=False)
            rescale = T.alloc_var("int32")
            rescale = 0
            for i in T.Parallel(block_M):
                if (scores_max_prev[i] - scores_max[i]) * scale > 8.0:
                    scores_scale[i] = T.exp2((scores_max[i] - scores_max_prev[i]) * scale)
                    scores_max[i] = scores_max_prev[i]
                    rescale = 1
                else:
                    scores_scale[i] = 1.0
            if rescale != 0:
                for i, j in T.Parallel(block_M, dim):
                    acc_o[i, j] *= scores_scale[i]
        else:
            T.reduce_max(acc_s, scores_max, dim=1, clear=False)
            if masked:
                # a row whose keys are all masked so far keeps a finite (0) running max: exp2 of
                # -inf - 0 is 0, never inf - inf (softmax is shift invariant)
                for i in T.Parallel(block_M):
                    scores_max[i] = T.if_then_else(scores_max[i] == -T.infinity(accum_dtype), 0, scores_max[i])
            for i in T.Parallel(block_M):
                scores_scale[i] = T.exp2(scores_max_prev[i] * scale - scores_max[i] * scale)
            for i, j in T.Parallel(block_M, dim):
                acc_o[i, j] *= scores_scale[i]
        for i, j in T.Parallel(block_M, block_N):
            acc_s[i, j] = T.exp2(acc_s[i, j] * scale - scores_max[i] * scale)
        T.reduce_sum(acc_s, scores_sum, dim=1)
        for i in T.Parallel(block_M):
            logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
        T.copy(acc_s, acc_s_cast)
        T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)

    @T.prim_func
    def main(Q: T.Tensor(q_shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(kv_shape, dtype),
             Output: T.Tensor(q_shape, dtype), Sinks: T.Tensor([heads], dtype)):
        # heads on the fastest grid axis: every head's heaviest (last) query tile is dispatched
        # before any lighter one -- global longest-first order for the triangular causal work; with
        # few query tiles (<= 4) across batches too (the tile axis slowest), with more the batch
        # stays slowest for L2 reuse of K/V (the measured split of example_mha_fwd_pipelined)
        lpt = n_qt <= 4
        with T.Kernel(heads, *((batch, n_qt) if lpt else (n_qt, batch)), threads=threads) as (by, g1, g2):
            bx, bz = (g2, g1) if lpt else (g1, g2)
            Q_shared = T.alloc_shared([block_M, dim], dtype)
            K_shared = T.alloc_shared([block_N, dim], dtype)
            V_shared = T.alloc_shared([block_N, dim], dtype)
            acc_s = T.alloc_fragment([block_M, block_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([block_M, block_N], dtype)
            acc_o = T.alloc_fragment([block_M, dim], accum_dtype)
            scores_max = T.alloc_fragment([block_M], accum_dtype)
            scores_max_prev = T.alloc_fragment([block_M], accum_dtype)
            scores_scale = T.alloc_fragment([block_M], accum_dtype)
            scores_sum = T.alloc_fragment([block_M], accum_dtype)
            logsum = T.alloc_fragment([block_M], accum_dtype)
            o_cast = T.alloc_fragment([block_M, dim], dtype)
            qt = n_qt - 1 - bx  # heaviest causal tiles first

            T.copy(Q[bz, by, qt * block_M:(qt + 1) * block_M, :], Q_shared)
            T.fill(acc_o, 0)
            T.fill(logsum, 0)
            T.fill(scores_max, -(2.0**30) if lazy_rescale else -T.infinity(accum_dtype))
            # KV tiles [start, full_end) lie entirely below the diagonal (and inside the window's
            # far edge when windowed); [full_end, end) need the mask
            if causal:
                end = T.min(T.ceildiv(seq_kv, block_N), T.ceildiv((qt + 1) * block_M + past_len, block_N))
                full_end = T.max(T.min((qt * block_M + past_len + 1) // block_N, end), 0)
            else:
                end = T.ceildiv(seq_kv, block_N)
                full_end = seq_kv // block_N
            if window_size is not None:
                start = T.max(0, (qt * block_M + past_len - window_size) // block_N)
                for k in T.Pipelined(start, end, num_stages=num_stages):
                    step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, scores_max, scores_max_prev,
                         scores_scale, scores_sum, logsum, k, qt, by, bz, True)
            else:
                for k in T.Pipelined(full_end, num_stages=num_stages):
                    step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, scores_max, scores_max_prev,
                         scores_scale, scores_sum, logsum, k, qt, by, bz, False)
                for k in T.Pipelined(full_end, end, num_stages=num_stages):
                    step(K, V, Q_shared, K_shared, V_shared, acc_s, acc_s_cast, acc_o, scores_max, scores_max_prev,
                         scores_scale, scores_sum, logsum, k, qt, by, bz, True)
            for i in T.Parallel(block_M):
                logsum[i] += T.exp2(T.Cast(accum_dtype, Sinks[by]) * LOG2E - scores_max[i] * scale)
            for i, j in T.Parallel(block_M, dim):
                o_cast[i, j] = acc_o[i, j] / logsum[i]
            T.copy(o_cast, Output[bz, by, qt * block_M:(qt + 1) * block_M, :])

    return main


def ref_program(query, key, value, sinks, sliding_window: Optional[int] = None):
    """query [b,h,sq,d], key/value [b,hkv,skv,d], sinks [h] (gpt-oss reference semantics)."""
    import torch
    b, h, sq, d = query.shape
    hkv, skv = key.shape[1], key.shape[2]
    g = h // hkv
    k = key.float().repeat_interleave(g, dim=1)
    v = value.float().repeat_interleave(g, dim=1)
    logits = torch.einsum("bhqd,bhkd->bhqk", query.float(), k) / d**0.5
    pos_k = torch.arange(skv, device=query.device)
    pos_q = torch.arange(sq, device=query.device) + (skv - sq)
    mask = pos_k[None, :] > pos_q[:, None]
    if sliding_window:
        mask |= pos_k[None, :] < (pos_q[:, None] - sliding_window + 1)
    logits = logits.masked_fill(mask, float("-inf"))
    s = sinks.float().view(1, h, 1, 1)
    mx = torch.maximum(logits.max(dim=-1, keepdim=True).values, s)
    p = torch.exp(logits - mx)
    p = p / (p.sum(-1, keepdim=True) + torch.exp(s - mx))
    return torch.einsum("bhqk,bhkd->bhqd", p, v).to(query.dtype)


def flops(batch, heads, seq_q, seq_kv, dim, window_size=None):
    """The reference's count (benchmark_gqa_sink_fwd.py:142-147): causal = half the square."""
    if window_size is not None:
        return 2 * 2.0 * batch * heads * min(window_size, seq_kv // 2) * seq_q * dim
    return 2 * 2.0 * batch * heads * seq_q * seq_kv * dim * 0.5


def main(batch=1, heads=64, seq_q=4096, seq_kv=4096, dim=128, groups=8, window_size=None, dtype="bfloat16"):
    import torch
    tdt = getattr(torch, dtype)
    kernel = flashattn_sink(batch, heads, seq_q, seq_kv, dim, groups, window_size, dtype=dtype)
    q = torch.randn(batch, heads, seq_q, dim, device="cuda", dtype=tdt)
    k = torch.randn(batch, heads // groups, seq_kv, dim, device="cuda", dtype=tdt)
    v = torch.randn_like(k)
    sinks = torch.randn(heads, device="cuda", dtype=tdt)
    o = kernel(q, k, v, sinks)
    torch.testing.assert_close(o.float(), ref_program(q, k, v, sinks, window_size).float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v, sinks))
    print(f"gqa+sink fwd b{batch} h{heads} kvh{heads // groups} s{seq_q} d{dim}: {lat:.3f} ms, "
          f"{flops(batch, heads, seq_q, seq_kv, dim, window_size) / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=1)
    p.add_argument("--heads", type=int, default=64)
    p.add_argument("--seq_q", type=int, default=4096)
    p.add_argument("--seq_kv", type=int, default=4096)
    p.add_argument("--dim", type=int, default=128)
    p.add_argument("--groups", type=int, default=8)
    p.add_argument("--window_size", type=int, default=None)
    a = p.parse_args()
    main(a.batch, a.heads, a.seq_q, a.seq_kv, a.dim, a.groups, a.window_size)
