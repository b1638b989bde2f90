"""SeerAttention-style block-sparse attention forward (reference:
``examples/seer_attention/block_sparse_attn_tilelang.py``).

Input is the raw int8 block gate ``BlockSparseMask[b, h, qblk, kblk]`` produced by top-k or a
threshold over a downsampled attention map (``get_sparse_attn_mask_from_topk`` /
``..._from_threshold``).  The reference walks every key block and branches on the gate.  Here each
workgroup first compacts its gate row into an LDS list of active key blocks (a parallel gate
pass, an LDS scan and a scatter), so the KV loop has a data-dependent
trip count, no branch, and its K/V copies stay LDS-DMA producers of ``T.Pipelined``.

Queries may be a suffix of the keys (``seq_q <= seq_kv``, e.g. chunked prefill over a cache):
query block ``bx`` is gated by mask row ``bx + (seq_kv - seq_q) / block`` and masked causally
against absolute key positions.
"""
import argparse
import math

import torch
import torch.nn.functional as F

import tilelang
import tilelang.language as T

LOG2E = 1.44269504


def get_sparse_attn_mask_from_topk(x, topk, use_dense_for_last_block=False):
    bsz, num_head, downsample_len, _ = x.shape
    sparse_index = torch.topk(x, topk, dim=-1).indices
    dense_mask = torch.zeros([bsz, num_head, downsample_len, downsample_len], dtype=torch.bool, device=x.device)
    dense_mask.scatter_(-1, sparse_index, True)
    if use_dense_for_last_block:
        dense_mask[:, :, -2:, :] = True
    return dense_mask.tril_()


def get_sparse_attn_mask_from_threshold(x, threshold, use_dense_for_last_block=False):
    dense_mask = x > threshold
    if use_dense_for_last_block:
        dense_mask[:, :, -2:, :] = True
    return dense_mask.tril_()


@tilelang.jit(out_idx=[4], pass_configs={tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True})
def blocksparse_flashattn(batch, heads, seq_q, seq_kv, dim, downsample_len, is_causal, block=64, threads=256,
                          num_stages=2, dtype="float16"):
    assert seq_q <= seq_kv and (seq_kv - seq_q) % block == 0, "queries are a block-aligned suffix of the keys"
    scale = (1.0 / dim)**0.5 * LOG2E
    past_len = seq_kv - seq_q
    past_blocks = past_len // block
    B_M = B_N = block
    n_kv = T.ceildiv(seq_kv, B_N)
    accum_dtype = "float"
    q_shape, kv_shape = [batch, heads, seq_q, dim], [batch, heads, seq_kv, dim]

    @T.prim_func
    def main(Q: T.Tensor(q_shape, dtype), K: T.Tensor(kv_shape, dtype), V: T.Tensor(kv_shape, dtype),
             BlockSparseMask: T.Tensor([batch, heads, downsample_len, downsample_len], "int8"),
             Output: T.Tensor(q_shape, dtype)):
        with T.Kernel(T.ceildiv(seq_q, B_M), heads, batch, threads=threads) as (bx, by, bz):
            Q_shared = T.alloc_shared([B_M, dim], dtype)
            K_shared = T.alloc_shared([B_N, dim], dtype)
            V_shared = T.alloc_shared([B_N, dim], dtype)
            gate = T.alloc_shared([downsample_len], "int32")
            pos = T.alloc_shared([downsample_len], "int32")
            blocks = T.alloc_shared([downsample_len], "int32")
            acc_s = T.alloc_fragment([B_M, B_N], accum_dtype)
            acc_s_cast = T.alloc_fragment([B_M, B_N], dtype)
            acc_o = T.alloc_fragment([B_M, dim], accum_dtype)
            o_cast = T.alloc_fragment([B_M, dim], dtype)
            m = T.alloc_fragment([B_M], accum_dtype)
            m_prev = T.alloc_fragment([B_M], accum_dtype)
            alpha = T.alloc_fragment([B_M], accum_dtype)
            l_sum = T.alloc_fragment([B_M], accum_dtype)
            r_sum = T.alloc_fragment([B_M], accum_dtype)
            row = T.min(bx + past_blocks, downsample_len - 1)
            T.copy(Q[bz, by, bx * B_M:(bx + 1) * B_M, :], Q_shared)
            # compact the gate row into an LDS list of active key blocks (scan + scatter)
            for j in T.Parallel(downsample_len):
                gate[j] = T.if_then_else((BlockSparseMask[bz, by, row, j] != 0) & (j < n_kv), 1, 0)
            T.cumsum(gate, pos)
            for j in T.Parallel(downsample_len):
                if gate[j] != 0:
                    blocks[pos[j] - 1] = j
            T.fill(acc_o, 0)
            T.fill(l_sum, 0)
            T.fill(m, -(2.0**30))
            for i in T.Pipelined(pos[downsample_len - 1], num_stages=num_stages):
                kb = blocks[i]
                T.copy(K[bz, by, kb * B_N:(kb + 1) * B_N, :], K_shared)
                T.copy(V[bz, by, kb * B_N:(kb + 1) * B_N, :], V_shared)
                if is_causal:
                    for r, c in T.Parallel(B_M, B_N):
                        acc_s[r, c] = T.if_then_else(bx * B_M + r + past_len >= kb * B_N + c, 0,
                                                     -T.infinity(accum_dtype))
                else:
                    for r, c in T.Parallel(B_M, B_N):
                        acc_s[r, c] = T.if_then_else(kb * B_N + c < seq_kv, 0, -T.infinity(accum_dtype))
                T.gemm(Q_shared, K_shared, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
                # lazy rescale: O is rescaled only when a row's max moves by more than 2^8
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


def ref_program(q, k, v, block_mask, block=64, is_causal=True):
    Q_LEN, K_LEN = q.shape[2], k.shape[2]
    past_len = K_LEN - Q_LEN
    full = torch.kron(block_mask.float(), torch.ones(block, block, device=q.device)).bool()[..., :K_LEN, :K_LEN]
    eff = full[..., past_len:K_LEN, :]
    if is_causal:
        i = torch.arange(past_len, K_LEN, device=q.device).unsqueeze(1)
        j = torch.arange(K_LEN, device=q.device).unsqueeze(0)
        eff = eff & (j <= i)
    attn = torch.einsum("bhsd,bhtd->bhst", q.float(), k.float()) * q.shape[-1]**-0.5
    attn = attn.masked_fill(~eff, float("-inf"))
    return torch.einsum("bhst,bhtd->bhsd", F.softmax(attn, dim=-1), v.float()).to(q.dtype)


def run(BATCH, N_HEADS, Q_LEN, K_LEN, D_HEAD, TOPK, BLOCK=64, device="cuda", target=None, seed=0):
    torch.manual_seed(seed)
    q = torch.randn(BATCH, N_HEADS, Q_LEN, D_HEAD, device=device, dtype=torch.float16)
    k = torch.randn(BATCH, N_HEADS, K_LEN, D_HEAD, device=device, dtype=torch.float16)
    v = torch.randn(BATCH, N_HEADS, K_LEN, D_HEAD, device=device, dtype=torch.float16)
    downsample_len = math.ceil(K_LEN / BLOCK)
    x_ds = torch.randn(BATCH, N_HEADS, downsample_len, downsample_len, device=device, dtype=torch.float16)
    x_ds[:, :, :, 0] = 100
    block_mask = get_sparse_attn_mask_from_topk(x_ds, topk=TOPK)
    if target is None:
        kernel = blocksparse_flashattn(BATCH, N_HEADS, Q_LEN, K_LEN, D_HEAD, downsample_len, is_causal=True)
    else:
        kernel = tilelang.compile(
            blocksparse_flashattn.get_tir(BATCH, N_HEADS, Q_LEN, K_LEN, D_HEAD, downsample_len, is_causal=True,
                                          threads=256), out_idx=[4], target=target)
    out = kernel(q, k, v, block_mask.to(torch.int8))
    torch.testing.assert_close(out.float(), ref_program(q, k, v, block_mask, BLOCK).float(), atol=1e-2, rtol=1e-2)
    return kernel, (q, k, v, block_mask.to(torch.int8))


def test_topk_sparse_attention(device="cuda", target=None):
    run(4, 2, 256, 256, 64, TOPK=2, device=device, target=target)


def test_topk_sparse_attention_qlen_lt_klen(device="cuda", target=None):
    run(1, 1, 128, 256, 64, TOPK=1, device=device, target=target)


def main(bench=True):
    test_topk_sparse_attention()
    test_topk_sparse_attention_qlen_lt_klen()
    print("Pass topk sparse attention tests (qlen == klen, qlen < klen)")
    if bench:
        B, H, S, D = 1, 32, 8192, 128
        nblk = S // 64
        kernel, args = run(B, H, S, S, D, TOPK=nblk // 4, seed=1)
        from tilelang.profiler import do_bench
        ms = do_bench(lambda: kernel(*args))
        active = int(args[3].sum())
        print(f"seer block-sparse attn B{B} H{H} S{S} D{D} top-{nblk // 4}: {ms:.3f} ms, "
              f"{4 * D * 64 * 64 * active / ms * 1e-9:.1f} TFLOPS on active blocks (incl. in-kernel gate compaction)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-bench", action="store_true")
    main(not ap.parse_args().no_bench)
