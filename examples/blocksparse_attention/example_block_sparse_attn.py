"""Block-sparse attention forward (reference: examples/blocksparse_attention/
example_tilelang_block_sparse_attn.py, examples/seer_attention/block_sparse_attn_tilelang.py).

``BlockMask[b, h, qi, kj]`` enables the (64-row query block, 64-row key block) pairs.  The
reference walks every key block and branches on the mask; here the mask is first compacted
(on the GPU, by torch) into per-query-block lists of active key blocks + counts, so the kernel's
KV loop has a data-dependent trip count and no branch: its K/V copies stay LDS-DMA producers of
``T.Pipelined`` and skipped blocks cost nothing.  Causal masking applies inside the diagonal
block.  Layout BHSD, one workgroup per (query block, head, batch), 4 waves x 16 rows (FullRow).
"""
import argparse

import tilelang
import tilelang.language as T

# exp/exp2 on the hardware transcendental unit (v_exp_f32): differs from the precise
# OCML expansion only for results below 2^-126, which softmax/decay terms never need
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}

LOG2E = 1.44269504


@tilelang.jit(out_idx=[-1], pass_configs=FAST_MATH)
def blocksparse_attn(batch, heads, seq_len, dim, is_causal=True, block=64, threads=256, num_stages=2,
                     dtype="bfloat16"):
    scale = (1.0 / dim)**0.5 * LOG2E
    nblk = seq_len // block
    B_M = B_N = block
    accum_dtype = "float"
    shape = [batch, heads, seq_len, dim]

    @T.prim_func
    def main(Q: T.Tensor(shape, dtype), K: T.Tensor(shape, dtype), V: T.Tensor(shape, dtype),
             BlockIdx: T.Tensor([batch, heads, nblk, nblk], "int32"), Counts: T.Tensor([batch, heads, nblk], "int32"),
             Output: T.Tensor(shape, dtype)):
        with T.Kernel(nblk, heads, batch, threads=threads) as (bx, by, bz):
            Q_shared = T.alloc_shared([B_M, dim], dtype)
            K_shared = T.alloc_shared([B_N, dim], dtype)
            V_shared = T.alloc_shared([B_N, dim], dtype)
            acc_s = T.alloc_fragment([B_M, B_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([B_M, B_N], dtype)
            acc_o = T.alloc_fragment([B_M, dim], accum_dtype)
            o_cast = T.alloc_fragment([B_M, dim], dtype)
            m = T.alloc_fragment([B_M], accum_dtype)
            m_prev = T.alloc_fragment([B_M], accum_dtype)
            alpha = T.alloc_fragment([B_M], accum_dtype)
            l_sum = T.alloc_fragment([B_M], accum_dtype)
            r_sum = T.alloc_fragment([B_M], accum_dtype)
            T.copy(Q[bz, by, bx * B_M:(bx + 1) * B_M, :], Q_shared)
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            for i in T.Pipelined(Counts[bz, by, bx], num_stages=num_stages):
                kb = T.min(T.max(BlockIdx[bz, by, bx, i], 0), nblk - 1)
                T.copy(K[bz, by, kb * B_N:(kb + 1) * B_N, :], K_shared)
                T.copy(V[bz, by, kb * B_N:(kb + 1) * B_N, :], V_shared)
                if is_causal:
                    for r, c in T.Parallel(B_M, B_N):
                        acc_s[r, c] = T.if_then_else(bx * B_M + r >= kb * B_N + c, 0, -T.infinity(accum_dtype))
                else:
                    T.clear(acc_s)
                T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                # lazy rescale: a row keeps its max until a score beats it by 2^8 (P <= 256); the
                # O rescale runs only on the blocks where one of the thread's rows moved
                T.copy(m, m_prev)
                T.reduce_max(acc_s, m_prev, dim=1, clear=False)  # candidate max
                rescale = T.alloc_var("int32")
                rescale = 0
                for r in T.Parallel(B_M):
                    if (m_prev[r] - m[r]) * scale > 8.0:
                        alpha[r] = T.exp2((m[r] - m_prev[r]) * scale)
                        m[r] = m_prev[r]
                        rescale = 1
                    else:
                        alpha[r] = 1.0
                for r, c in T.Parallel(B_M, B_N):
                    acc_s[r, c] = T.exp2(acc_s[r, c] * scale - m[r] * scale)
                T.reduce_sum(acc_s, r_sum, dim=1)
                for r in T.Parallel(B_M):
                    l_sum[r] = l_sum[r] * alpha[r] + r_sum[r]
                if rescale != 0:
                    for r, d in T.Parallel(B_M, dim):
                        acc_o[r, d] *= alpha[r]
                T.copy(acc_s, acc_s_cast)
                T.gemm(acc_s_cast, V_shared, acc_o, policy=T.GemmWarpPolicy.FullRow)
            for r, d in T.Parallel(B_M, dim):
                o_cast[r, d] = acc_o[r, d] / T.max(l_sum[r], 1e-30)
            T.copy(o_cast, Output[bz, by, bx * B_M:(bx + 1) * B_M, :])

    return main


def compact_mask(mask):
    """bool [B, H, nq, nk] -> (int32 active key-block lists, active first, [B, H, nq, nk]; counts [B, H, nq])."""
    import torch
    order = torch.argsort((~mask).to(torch.int8), dim=-1, stable=True)
    return order.int().contiguous(), mask.sum(-1).int().contiguous()


def random_block_mask(B, H, nblk, density, causal=True, device="cpu", seed=0):
    import torch
    g = torch.Generator(device=device).manual_seed(seed)
    m = torch.rand(B, H, nblk, nblk, generator=g, device=device) < density
    m |= torch.eye(nblk, dtype=torch.bool, device=device)  # every query block sees its diagonal
    if causal:
        m = m.tril()
    return m


def ref_program(q, k, v, mask, block=64, causal=True):
    import torch
    S = q.shape[2]
    full = mask.repeat_interleave(block, 2).repeat_interleave(block, 3)[:, :, :S, :S]
    if causal:
        full = full & torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
    s = (q.float() @ k.float().transpose(-1, -2)) * q.shape[-1]**-0.5
    s = s.masked_fill(~full, float("-inf"))
    return (torch.softmax(s, -1) @ v.float()).to(q.dtype)


def main(B=1, H=32, S=8192, D=128, density=0.25):
    import torch
    kernel = blocksparse_attn(B, H, S, D)
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16) for _ in range(3))
    mask = random_block_mask(B, H, S // 64, density, True, "cuda")
    idx, cnt = compact_mask(mask)
    o = kernel(q, k, v, idx, cnt)
    ref = ref_program(q[:, :2], k[:, :2], v[:, :2], mask[:, :2])
    torch.testing.assert_close(o[:, :2].float(), ref.float(), rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    lat = kernel.get_profiler().do_bench(lambda: kernel(q, k, v, idx, cnt))
    flops = 4 * D * 64 * 64 * int(cnt.sum())  # cnt sums over batch and heads
    print(f"block-sparse attn B{B} H{H} S{S} D{D} density {float(cnt.sum()) / mask.numel():.3f}: {lat:.3f} ms, "
          f"{flops / lat * 1e-9:.1f} TFLOPS (active blocks)")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--seq", type=int, default=8192)
    p.add_argument("--density", type=float, default=0.25)
    a = p.parse_args()
    main(S=a.seq, density=a.density)
