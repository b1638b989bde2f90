"""DeepSeek MLA decode over an fp8 (OCP e4m3) latent KV cache
(reference: examples/deepseek_mla/experimental/example_mla_decode_kv_fp8.py:1-95).

The reference keeps the latent cache in fp8, copies each tile to fp16 in shared memory and runs
both GEMMs in fp16.  On gfx950 the score GEMM consumes the fp8 cache directly:

  * S_nope = Q KV^T runs on ``v_mfma_scale_f32_16x16x128_f8f6f4`` (OCP e4m3 x e4m3, K = 512 in four
    128-wide MFMA steps).  Q is quantised once per block in the prologue, one fp32 scale per head
    row (``qs = amax / 448``); the cache carries one per-tensor fp32 scale ``kv_scale``.  The row
    factor ``qs[h] * kv_scale`` is applied to the raw fp8 scores before the rope part
    ``Q_pe K_pe^T`` (bf16 MFMA, K_pe stays bf16 as in the reference) accumulates on top.
  * O = P V needs the latent tile transposed (``ds_read_b64_tr_b16``), which the 8-bit MFMA path
    cannot feed, so the tile is widened once in LDS (fp8 -> bf16, packed conversions) and the PV
    GEMM is the bf16 wide schedule of ``example_mla_decode.py``; ``kv_scale`` is folded into the
    final 1 / logsum.

``qk_fp8=False`` keeps Q in bf16 and runs both GEMMs on the widened tile (the reference's
numerics; fp8 Q costs ~1-3 % relative error on the output at unit-variance inputs).

The cache tile moves HBM -> LDS by LDS-DMA at half the bytes of the bf16 kernel; split-KV plus the
LSE combine of ``example_mla_decode.py`` fills the chip at small batch.

``pv_fp8`` (default): P V on the fp8 MFMA as well -- P in e4m3 (bounded by 2^8 by the lazy rescale),
V straight from the fp8 tile through ``ds_read_b64_tr_b8`` transposed reads, and with block_N = 128
keys the PV GEMM is a 128-deep scaled MFMA step.  b128 h128 kv8192 (same process, round-robin,
profiles/r6/mla_fp8_ab.log): 945 TFLOPS against 636 for the bf16 kernel (1.49x) and 472 for the
widened-tile path; output error vs fp32 over the dequantised cache 2.8 % (relative norm, random
data) against 2.6 % with bf16 P V -- the fp8 Q dominates it.
"""
import argparse

import tilelang
import tilelang.language as T

FP8 = "float8_e4m3fn"
FP8_MAX = 448.0


@tilelang.jit(out_idx=[7], pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def mla_decode_kv_fp8(batch, heads, seqlen_kv, dim, pe_dim, block_N=128, block_H=64, num_split=2, threads=512,
                      num_stages=1, dtype="bfloat16", qk_fp8=True, pv_fp8=None, sum_mfma=True):
    """``qk_fp8``: scores on the fp8 MFMA with Q quantised per head row (default); False keeps Q in
    ``dtype`` and runs both GEMMs on the widened tile (the reference's numerics).
    ``pv_fp8`` (default: with ``qk_fp8``): O += P V on the fp8 MFMA too -- P in e4m3 (the lazy
    rescale bounds it by 2^8, inside e4m3's range, so no scale is needed; 3 mantissa bits per
    probability), V read straight from the fp8 cache tile with ds_read_b64_tr_b8: no widened copy
    of the tile, half the LDS bytes per PV operand.
    ``sum_mfma``: the softmax row sums are P x ones on the MFMA (P as P V consumes it: e4m3 with
    ``pv_fp8``), rescaled with O, instead of a per-tile cross-wave reduction (example_mla_decode.py)."""
    if pv_fp8 is None:
        pv_fp8 = qk_fp8
    scale = (1.0 / (dim + pe_dim))**0.5 * 1.44269504  # softmax in base 2
    accum_dtype = "float"
    VALID_BLOCK_H = min(block_H, heads)
    assert dim % 128 == 0, "the fp8 score GEMM steps K in 128-wide MFMA blocks"
    assert seqlen_kv % (num_split * block_N) == 0
    split_len = seqlen_kv // num_split
    policy = T.GemmWarpPolicy.Square

    @T.macro
    def attention_split(Q, Q_pe, KV, K_pe, kv_scale, glse, Output_partial):
        with T.Kernel(batch, heads // VALID_BLOCK_H, num_split, threads=threads) as (bx, by, bz):
            if qk_fp8:
                Q_f = T.alloc_fragment([block_H, dim], accum_dtype)
                q_amax = T.alloc_fragment([block_H], accum_dtype)
                Q8_shared = T.alloc_shared([block_H, dim], FP8)
                qs_shared = T.alloc_shared([block_H], accum_dtype)
            else:
                Q_local = T.alloc_fragment([block_H, dim], dtype)
            Q_pe_local = T.alloc_fragment([block_H, pe_dim], dtype)
            KV8_shared = T.alloc_shared([block_N, dim], FP8)
            if not pv_fp8:
                V_shared = T.alloc_shared([block_N, dim], dtype)
            K_pe_shared = T.alloc_shared([block_N, pe_dim], dtype)
            acc_s = T.alloc_fragment([block_H, block_N], accum_dtype)
            P_shared = T.alloc_shared([block_H, block_N], FP8 if pv_fp8 else dtype)
            sc_shared = T.alloc_shared([block_H], accum_dtype)
            any_s = T.alloc_shared([2], "int32")
            acc_o = T.alloc_fragment([block_H, dim], accum_dtype)
            scores_max = T.alloc_fragment([block_H], accum_dtype)
            scores_max_prev = T.alloc_fragment([block_H], accum_dtype)
            scores_scale = T.alloc_fragment([block_H], accum_dtype)
            scores_sum = T.alloc_fragment([block_H], accum_dtype)
            logsum = T.alloc_fragment([block_H], accum_dtype)

            if qk_fp8:
                # Q -> fp8, one scale per head row (folded with the cache scale)
                T.copy(Q[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, :], Q_f)
                T.reduce_absmax(Q_f, q_amax, dim=1)
                for i in T.Parallel(block_H):
                    q_amax[i] = T.max(q_amax[i], 1e-6) / FP8_MAX
                for i, j in T.Parallel(block_H, dim):
                    Q8_shared[i, j] = T.clamp(Q_f[i, j] / q_amax[i], -FP8_MAX, FP8_MAX)
                for i in T.Parallel(block_H):
                    qs_shared[i] = q_amax[i] * kv_scale
            else:
                T.copy(Q[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, :], Q_local)
            T.copy(Q_pe[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, :], Q_pe_local)
            if sum_mfma:
                ones_s = T.alloc_shared([block_N, 32], FP8 if pv_fp8 else dtype)
                acc_l = T.alloc_fragment([block_H, 32], accum_dtype)
                T.fill(ones_s, 1.0)
                T.clear(acc_l)
            T.fill(acc_o, 0)
            T.fill(logsum, 0)
            # lazy rescale: a row keeps its max until a score beats it by 2^8 (P <= 256); the O
            # accumulator (split over the latent columns) is rescaled only when some row moved
            T.fill(scores_max, -(2.0**30))

            # lazy-rescale flag, double-buffered by iteration parity: iteration t resets the slot
            # of t + 1 (ordered by the stage barrier against t - 1's readers and t + 1's setters)
            for z in T.Parallel(2):
                any_s[z] = 0
            for k in T.Pipelined(split_len // block_N, num_stages=num_stages):
                kv_start = split_len * bz + k * block_N
                T.copy(KV[bx, kv_start:kv_start + block_N, 0, :], KV8_shared)
                T.copy(K_pe[bx, kv_start:kv_start + block_N, 0, :], K_pe_shared)
                if qk_fp8:
                    T.gemm(Q8_shared, KV8_shared, acc_s, transpose_B=True, clear_accum=True, policy=policy)
                    for i, j in T.Parallel(block_H, block_N):
                        acc_s[i, j] *= qs_shared[i]
                    T.gemm(Q_pe_local, K_pe_shared, acc_s, transpose_B=True, policy=policy)
                    if not pv_fp8:
                        T.copy(KV8_shared, V_shared)
                else:
                    T.copy(KV8_shared, V_shared)
                    T.gemm(Q_local, V_shared, acc_s, transpose_B=True, clear_accum=True, policy=policy)
                    for i, j in T.Parallel(block_H, block_N):
                        acc_s[i, j] *= kv_scale
                    T.gemm(Q_pe_local, K_pe_shared, acc_s, transpose_B=True, policy=policy)
                for z in T.Parallel(1):  # previous tile's readers are past the stage barrier
                    any_s[z + (k + 1) % 2] = 0
                T.copy(scores_max, scores_max_prev)
                T.reduce_max(acc_s, scores_max_prev, dim=1, clear=False)  # candidate max
                for i in T.Parallel(block_H):
                    if (scores_max_prev[i] - scores_max[i]) * scale > 8.0:
                        scores_scale[i] = T.exp2((scores_max[i] - scores_max_prev[i]) * scale)
                        scores_max[i] = scores_max_prev[i]
                        any_s[k % 2] = 1
                    else:
                        scores_scale[i] = 1.0
                for i, j in T.Parallel(block_H, block_N):
                    acc_s[i, j] = T.exp2(acc_s[i, j] * scale - scores_max[i] * scale)
                if not sum_mfma:
                    T.reduce_sum(acc_s, scores_sum, dim=1)
                    for i in T.Parallel(block_H):
                        logsum[i] = logsum[i] * scores_scale[i] + scores_sum[i]
                T.copy(scores_scale, sc_shared)
                T.copy(acc_s, P_shared)
                if any_s[k % 2] != 0:
                    for i, j in T.Parallel(block_H, dim):
                        acc_o[i, j] *= sc_shared[i]
                    if sum_mfma:
                        for i, j in T.Parallel(block_H, 32):
                            acc_l[i, j] *= sc_shared[i]
                if pv_fp8:
                    T.gemm(P_shared, KV8_shared, acc_o)  # e4m3 x e4m3, B [keys, dim]: transposed reads
                else:
                    T.gemm(P_shared, V_shared, acc_o)
                if sum_mfma:
                    T.gemm(P_shared, ones_s, acc_l)
            if sum_mfma:
                for i, j in T.Parallel(block_H, 32):  # every column of P x ones is the row sum
                    if j == 0:
                        sc_shared[i] = acc_l[i, j]
                for i in T.Parallel(block_H):
                    logsum[i] = sc_shared[i]
            for i in T.Parallel(block_H):
                sc_shared[i] = kv_scale / logsum[i]
            for i, j in T.Parallel(block_H, dim):
                acc_o[i, j] *= sc_shared[i]
            for i in T.Parallel(block_H):
                logsum[i] = T.log2(logsum[i]) + scores_max[i] * scale
            T.copy(logsum, glse[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, bz])
            T.copy(acc_o, Output_partial[bx, by * VALID_BLOCK_H:(by + 1) * VALID_BLOCK_H, bz, :])

    @T.macro
    def combine(glse, Output_partial, Output):
        with T.Kernel(heads, batch, threads=128) as (hy, bz):
            o_acc = T.alloc_fragment([dim], accum_dtype)
            lse_max = T.alloc_local([1], accum_dtype)
            lse_sum = T.alloc_local([1], accum_dtype)
            sc = T.alloc_local([1], accum_dtype)
            T.clear(o_acc)
            lse_max[0] = -T.infinity(accum_dtype)
            for k in T.serial(num_split):
                lse_max[0] = T.max(lse_max[0], glse[bz, hy, k])
            lse_sum[0] = 0.0
            for k in T.serial(num_split):
                lse_sum[0] += T.exp2(glse[bz, hy, k] - lse_max[0])
            lse_sum[0] = T.log2(lse_sum[0]) + lse_max[0]
            for k in T.serial(num_split):
                sc[0] = T.exp2(glse[bz, hy, k] - lse_sum[0])
                for i in T.Parallel(dim):
                    o_acc[i] += Output_partial[bz, hy, k, i] * sc[0]
            for i in T.Parallel(dim):
                Output[bz, hy, i] = o_acc[i]

    @T.prim_func
    def main(
            Q: T.Tensor([batch, heads, dim], dtype),
            Q_pe: T.Tensor([batch, heads, pe_dim], dtype),
            KV: T.Tensor([batch, seqlen_kv, 1, dim], FP8),
            K_pe: T.Tensor([batch, seqlen_kv, 1, pe_dim], dtype),
            kv_scale: T.float32,
            glse: T.Tensor([batch, heads, num_split], accum_dtype),
            Output_partial: T.Tensor([batch, heads, num_split, dim], accum_dtype),
            Output: T.Tensor([batch, heads, dim], dtype),
    ):
        attention_split(Q, Q_pe, KV, K_pe, kv_scale, glse, Output_partial)
        combine(glse, Output_partial, Output)

    return main


def quantize_kv(kv):
    """bf16/fp32 latent cache -> (OCP e4m3 cache, per-tensor fp32 scale)."""
    import torch
    s = float(kv.float().abs().amax().clamp_min(1e-6)) / FP8_MAX
    return (kv.float() / s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn), s


def quantize_q_rows(q):
    """The kernel's Q quantisation (qk_fp8): e4m3 with one scale per head row, dequantised."""
    import torch
    s = q.float().abs().amax(-1, keepdim=True).clamp_min(1e-6) / FP8_MAX
    return (q.float() / s).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).float() * s


def ref_program(q, q_pe, kv8, kv_scale, k_pe, quant_q=False):
    """fp32 attention over the dequantised cache (``quant_q``: with the kernel's fp8 Q)."""
    import torch
    dim, pe_dim = q.shape[-1], q_pe.shape[-1]
    kv = kv8[:, :, 0].float() * kv_scale
    if quant_q:
        q = quantize_q_rows(q)
    s = (torch.einsum("bhd,bsd->bhs", q.float(), kv) +
         torch.einsum("bhd,bsd->bhs", q_pe.float(), k_pe[:, :, 0].float())) / (dim + pe_dim)**0.5
    return torch.einsum("bhs,bsd->bhd", torch.softmax(s, dim=-1), kv)


def flops(batch, heads, seqlen_kv, dim, pe_dim):
    return 2 * batch * heads * seqlen_kv * (dim + pe_dim) + 2 * batch * heads * seqlen_kv * dim


def main(batch=128, heads=128, kv_ctx=8192, dim=512, pe_dim=64, num_split=None, qk_fp8=True, pv_fp8=None,
         block_N=128, num_stages=1):
    import torch
    from example_mla_decode import auto_split
    num_split = num_split or auto_split(batch, heads)
    kernel = mla_decode_kv_fp8(batch, heads, kv_ctx, dim, pe_dim, num_split=num_split, qk_fp8=qk_fp8, pv_fp8=pv_fp8,
                               block_N=block_N, num_stages=num_stages)
    q = torch.randn(batch, heads, dim, device="cuda", dtype=torch.bfloat16)
    q_pe = torch.randn(batch, heads, pe_dim, device="cuda", dtype=torch.bfloat16)
    kv8, s = quantize_kv(torch.randn(batch, kv_ctx, 1, dim, device="cuda"))
    k_pe = torch.randn(batch, kv_ctx, 1, pe_dim, device="cuda", dtype=torch.bfloat16)
    glse = torch.empty(batch, heads, num_split, device="cuda")
    part = torch.empty(batch, heads, num_split, dim, device="cuda")
    out = kernel(q, q_pe, kv8, k_pe, s, glse, part)
    torch.testing.assert_close(out.float(), ref_program(q, q_pe, kv8, s, k_pe, qk_fp8), rtol=2e-2, atol=2e-2)
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, q_pe, kv8, k_pe, s, glse, part))
    pv = qk_fp8 if pv_fp8 is None else pv_fp8
    print(f"MLA decode fp8-KV ({'fp8' if qk_fp8 else 'bf16'} QK, {'fp8' if pv else 'bf16'} PV, block_N {block_N}, "
          f"{num_stages} stage(s)) b{batch} h{heads} kv{kv_ctx} split{num_split}: "
          f"{lat:.3f} ms, "
          f"{flops(batch, heads, kv_ctx, dim, pe_dim) / lat * 1e-9:.1f} TFLOPS")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=128)
    p.add_argument("--heads", type=int, default=128)
    p.add_argument("--kv_ctx", type=int, default=8192)
    p.add_argument("--num_split", type=int, default=None)
    p.add_argument("--bf16_qk", action="store_true", help="scores in bf16 on the widened tile")
    p.add_argument("--bf16_pv", action="store_true", help="P V in bf16 on the widened tile")
    p.add_argument("--block_N", type=int, default=128)
    p.add_argument("--num_stages", type=int, default=1)
    a = p.parse_args()
    main(a.batch, a.heads, a.kv_ctx, 512, 64, a.num_split, not a.bf16_qk, False if a.bf16_pv else None, a.block_N,
         a.num_stages)
