"""MInference vertical-slash sparse attention (reference: examples/minference/
example_vertical_slash_sparse_attn.py).

Each head keeps a few *slash* lines (key = query - s) and *vertical* lines (key = v) of the
causal attention matrix.  Per query block of ``block_M`` rows the pattern becomes
  * ``block_offset``: the ``block_N``-aligned key blocks any slash line crosses (dense tiles),
  * ``column_index``: the vertical columns not already inside those blocks (gathered rows),
computed on the device by a tilelang kernel (``vs_convert``: LDS bitmap + prefix-sum compaction,
no host synchronisation; the reference ships a CUDA extension for this).  The attention kernel (one workgroup per query
block, head, batch) runs the online softmax over the dense key blocks (K/V tiles at data-dependent
offsets through the LDS-DMA ring) and then over the column chunks (``T.gather_rows``: per-lane row
addresses, LDS-DMA), causal-masked in both phases.
Parity with the reference's block boundaries is unpinned (the reference covers each slash with
unaligned key ranges, this version with aligned blocks); the test compares against a dense PyTorch
softmax over exactly the keys this conversion selects.
"""
import argparse

import tilelang
import tilelang.language as T

LOG2E = 1.44269504
FAST_MATH = {tilelang.PassConfigKey.TL_ENABLE_FAST_MATH: True}


@tilelang.jit(out_idx=[2, 3, 4, 5])
def vs_convert(batch, heads, seq_len, nv, ns, block_M=64, block_N=64, threads=256):
    """The index conversion on the device (the reference ships a CUDA extension for it), one
    workgroup per (query block, head, batch): the key blocks any slash line crosses are marked in an
    LDS bitmap and compacted in ascending order by a prefix sum; the vertical columns outside those
    blocks (and not past the block's last query) are compacted in input order the same way.  Output
    shapes are the static bounds (a 64-row segment of a slash crosses at most
    ceil((block_M - 1) / block_N) + 1 key blocks), so there is no host synchronisation."""
    NQ = (seq_len + block_M - 1) // block_M
    NK = (seq_len + block_N - 1) // block_N
    span = (block_M - 1) // block_N + 2
    MAXB = max(1, min(NK, span * ns))
    MAXC = max(block_N, (nv + block_N - 1) // block_N * block_N)

    @T.prim_func
    def main(Vidx: T.Tensor([batch, heads, nv], "int32"), Sidx: T.Tensor([batch, heads, ns], "int32"),
             BlockCount: T.Tensor([batch, heads, NQ], "int32"),
             BlockOffset: T.Tensor([batch, heads, NQ, MAXB], "int32"),
             ColumnCount: T.Tensor([batch, heads, NQ], "int32"),
             ColumnIndex: T.Tensor([batch, heads, NQ, MAXC], "int32")):
        with T.Kernel(NQ, heads, batch, threads=threads) as (bx, by, bz):
            cover = T.alloc_shared([NK], "int32")
            csum = T.alloc_shared([NK], "int32")
            vflag = T.alloc_shared([MAXC], "int32")
            vpos = T.alloc_shared([MAXC], "int32")
            m0 = bx * block_M
            m1 = T.min(m0 + block_M - 1, seq_len - 1)
            for j in T.Parallel(NK):
                cover[j] = 0
            for t in T.Parallel(ns):
                sv = Sidx[bz, by, t]
                lo = T.max(m0 - sv, 0)
                hi = T.min(m0 + block_M - 1 - sv, m1)
                for d in T.serial(span):
                    if (hi >= lo) & (lo // block_N + d <= hi // block_N):
                        cover[lo // block_N + d] = 1
            for j in T.Parallel(NK):
                csum[j] = cover[j]
            T.cumsum(csum, dim=0)
            for j in T.Parallel(NK):
                if cover[j] != 0:
                    BlockOffset[bz, by, bx, csum[j] - 1] = j * block_N
            for i in T.Parallel(MAXB):
                if i >= csum[NK - 1]:
                    BlockOffset[bz, by, bx, i] = -1
            for t in T.Parallel(MAXC):
                vv = T.if_then_else(t < nv, Vidx[bz, by, T.min(t, nv - 1)], -1)
                ok = (vv >= 0) & (vv <= m1)
                vflag[t] = T.if_then_else(ok, 1 - cover[T.max(T.min(vv, seq_len - 1), 0) // block_N], 0)
                vpos[t] = vflag[t]
            T.cumsum(vpos, dim=0)
            for t in T.Parallel(MAXC):
                if vflag[t] != 0:
                    ColumnIndex[bz, by, bx, vpos[t] - 1] = Vidx[bz, by, T.min(t, nv - 1)]
            for i in T.Parallel(MAXC):
                if i >= vpos[MAXC - 1]:
                    ColumnIndex[bz, by, bx, i] = -1
            for z in T.Parallel(1):
                BlockCount[bz, by, bx] = csum[NK - 1] + z
                ColumnCount[bz, by, bx] = vpos[MAXC - 1] + z

    return main


@tilelang.jit(out_idx=[2, 3, 4, 5])
def vs_convert_merged(batch, heads, seq_len, nv, ns, block_M=64, block_N=64, threads=256):
    """Index conversion with unaligned dense ranges (the reference's block semantics): ``Sidx`` sorted
    descending per head, so in every query block the slash ranges ``[m0 - s, m0 + block_M - 1 - s]``
    (clamped) arrive with ascending ends; ranges closer than ``block_N`` merge into segments (prefix
    sums over start flags), each segment is covered by ``ceil(len / block_N)`` key blocks starting at
    its first key (a block never reaches the next segment: the gap is at least ``block_N``), and the
    block list is emitted by a binary search over the segments' block prefix sums.  Vertical columns
    inside an emitted block are dropped (binary search over the segment starts).  Compared with
    ``block_N``-aligned blocks this attends up to 2x fewer keys per slash."""
    NQ = (seq_len + block_M - 1) // block_M
    NK = (seq_len + block_N - 1) // block_N
    per_range = (block_M + block_N - 1) // block_N + 1
    MAXB = max(1, min(NK + ns, ns * per_range))
    MAXC = max(block_N, (nv + block_N - 1) // block_N * block_N)
    LOGS = max(1, (ns + 1).bit_length() + 1)

    @T.prim_func
    def main(Vidx: T.Tensor([batch, heads, nv], "int32"), Sidx: T.Tensor([batch, heads, ns], "int32"),
             BlockCount: T.Tensor([batch, heads, NQ], "int32"),
             BlockOffset: T.Tensor([batch, heads, NQ, MAXB], "int32"),
             ColumnCount: T.Tensor([batch, heads, NQ], "int32"),
             ColumnIndex: T.Tensor([batch, heads, NQ, MAXC], "int32")):
        with T.Kernel(NQ, heads, batch, threads=threads) as (bx, by, bz):
            lo_s = T.alloc_shared([ns], "int32")
            hi_s = T.alloc_shared([ns], "int32")
            segid = T.alloc_shared([ns], "int32")
            seg_lo = T.alloc_shared([ns], "int32")
            seg_hi = T.alloc_shared([ns], "int32")
            bpos = T.alloc_shared([ns], "int32")
            vflag = T.alloc_shared([MAXC], "int32")
            vpos = T.alloc_shared([MAXC], "int32")
            m0 = bx * block_M
            m1 = T.min(m0 + block_M - 1, seq_len - 1)
            for t in T.Parallel(ns):
                sv = Sidx[bz, by, t]
                lo_s[t] = T.max(m0 - sv, 0)
                hi_s[t] = T.min(m0 + block_M - 1 - sv, m1)
            for t in T.Parallel(ns):  # a valid range starting a new segment (invalid ranges: a prefix)
                prev_ok = (t > 0) & (hi_s[T.max(t - 1, 0)] >= lo_s[T.max(t - 1, 0)])
                new_seg = T.if_then_else(prev_ok, lo_s[t] > hi_s[T.max(t - 1, 0)] + block_N, True)
                segid[t] = T.if_then_else((hi_s[t] >= lo_s[t]) & new_seg, 1, 0)
            for t in T.Parallel(ns):
                bpos[t] = segid[t]
            T.cumsum(segid, dim=0)
            for t in T.Parallel(ns):  # segment bounds: its first range's start, its last range's end
                if hi_s[t] >= lo_s[t]:
                    if bpos[t] != 0:
                        seg_lo[segid[t] - 1] = lo_s[t]
                    if (t == ns - 1) | (segid[T.min(t + 1, ns - 1)] != segid[t]):
                        seg_hi[segid[t] - 1] = hi_s[t]
            for k in T.Parallel(ns):  # blocks per segment (0 past the last segment)
                bpos[k] = T.if_then_else(k < segid[ns - 1], (seg_hi[k] - seg_lo[k] + block_N) // block_N, 0)
            T.cumsum(bpos, dim=0)
            for i in T.Parallel(MAXB):
                if i < bpos[ns - 1]:
                    a = T.alloc_var("int32")
                    b = T.alloc_var("int32")
                    a = 0
                    b = ns - 1  # first k with bpos[k] > i lies in [a, b]
                    for _ in T.serial(LOGS):
                        if a < b:
                            mid = (a + b) // 2
                            if bpos[mid] > i:
                                b = mid
                            else:
                                a = mid + 1
                    first = T.if_then_else(a > 0, bpos[T.max(a - 1, 0)], 0)
                    BlockOffset[bz, by, bx, i] = seg_lo[a] + (i - first) * block_N
                else:
                    BlockOffset[bz, by, bx, i] = -1
            for t in T.Parallel(MAXC):
                vv = T.if_then_else(t < nv, Vidx[bz, by, T.min(t, nv - 1)], -1)
                a2 = T.alloc_var("int32")
                b2 = T.alloc_var("int32")
                a2 = 0
                b2 = segid[ns - 1]  # last segment with seg_lo <= vv: a2 - 1 after the search
                for _ in T.serial(LOGS):
                    if a2 < b2:
                        mid2 = (a2 + b2) // 2
                        if seg_lo[mid2] <= vv:
                            a2 = mid2 + 1
                        else:
                            b2 = mid2
                kk = T.max(a2 - 1, 0)
                nb_k = bpos[kk] - T.if_then_else(kk > 0, bpos[T.max(kk - 1, 0)], 0)
                inside = (a2 > 0) & (vv < seg_lo[kk] + nb_k * block_N)
                vflag[t] = T.if_then_else((vv >= 0) & (vv <= m1) & (inside == False), 1, 0)  # noqa: E712
                vpos[t] = vflag[t]
            T.cumsum(vpos, dim=0)
            for t in T.Parallel(MAXC):
                if vflag[t] != 0:
                    ColumnIndex[bz, by, bx, vpos[t] - 1] = Vidx[bz, by, T.min(t, nv - 1)]
            for i in T.Parallel(MAXC):
                if i >= vpos[MAXC - 1]:
                    ColumnIndex[bz, by, bx, i] = -1
            for z in T.Parallel(1):
                BlockCount[bz, by, bx] = bpos[ns - 1] + z
                ColumnCount[bz, by, bx] = vpos[MAXC - 1] + z

    return main


def convert_vertical_slash_merged_py(v_idx, s_idx, seq_len, block_M=64, block_N=64):
    """Python reference of ``vs_convert_merged`` (per query block): (block_offsets, columns) lists."""
    out = []
    NQ = (seq_len + block_M - 1) // block_M
    for b in range(v_idx.shape[0]):
        for h in range(v_idx.shape[1]):
            ss = sorted(s_idx[b, h].tolist(), reverse=True)
            for qb in range(NQ):
                m0, m1 = qb * block_M, min(qb * block_M + block_M - 1, seq_len - 1)
                segs = []
                for sv in ss:
                    lo, hi = max(m0 - sv, 0), min(m0 + block_M - 1 - sv, m1)
                    if hi < lo:
                        continue
                    if segs and lo <= segs[-1][1] + block_N:
                        segs[-1][1] = max(segs[-1][1], hi)
                    else:
                        segs.append([lo, hi])
                offs, cov = [], []
                for lo, hi in segs:
                    n = (hi - lo + block_N) // block_N
                    offs += [lo + u * block_N for u in range(n)]
                    cov.append((lo, lo + n * block_N))
                cols = [v for v in v_idx[b, h].tolist() if 0 <= v <= m1 and not any(a <= v < e for a, e in cov)]
                out.append((b, h, qb, offs, cols))
    return out


def convert_vertical_slash_indexes(v_idx, s_idx, seq_len, block_M=64, block_N=64, merged=None):
    """(block_count, block_offset, column_count, column_index) int32 from a device kernel: ``merged``
    (default past 16K keys) unaligned dense ranges over merged slash segments (``vs_convert_merged``),
    else ``block_N``-aligned key blocks (``vs_convert``); block offsets ascending, columns in input
    order, unused slots -1."""
    import torch
    B, H, NV = v_idx.shape
    if merged is None:
        merged = seq_len > 16384
    if merged:
        k = vs_convert_merged(B, H, seq_len, NV, s_idx.shape[-1], block_M, block_N)
        return k(v_idx.int().contiguous(), torch.sort(s_idx.int(), dim=-1, descending=True).values.contiguous())
    k = vs_convert(B, H, seq_len, NV, s_idx.shape[-1], block_M, block_N)
    return k(v_idx.int().contiguous(), s_idx.int().contiguous())


def convert_vertical_slash_indexes_torch(v_idx, s_idx, seq_len, block_M=64, block_N=64):
    """Vectorised-PyTorch form of the conversion (the test's reference): v_idx [B, H, NV], s_idx
    [B, H, NS] -> (block_count [B,H,NQ], block_offset [B,H,NQ,MAXB], column_count [B,H,NQ],
    column_index [B,H,NQ,MAXC]) int32; unused slots are -1, columns sorted."""
    import torch
    dev = v_idx.device
    B, H, _ = v_idx.shape
    NQ = (seq_len + block_M - 1) // block_M
    NK = (seq_len + block_N - 1) // block_N
    m0 = torch.arange(NQ, device=dev) * block_M                      # query block starts
    s = s_idx.long()[:, :, None, :]                                   # [B,H,1,NS]
    lo = (m0[None, None, :, None] - s).clamp(min=0)                   # first key of the slash segment
    hi = torch.minimum(m0[None, None, :, None] + block_M - 1 - s,
                       (m0 + block_M - 1).clamp(max=seq_len - 1)[None, None, :, None])
    valid = hi >= lo
    kb = torch.arange(NK, device=dev)
    blk_lo, blk_hi = lo // block_N, hi // block_N
    cover = ((kb[None, None, None, None, :] >= blk_lo[..., None]) & (kb[None, None, None, None, :] <= blk_hi[..., None])
             & valid[..., None]).any(3)                               # [B,H,NQ,NK]
    cover &= kb[None, None, None, :] * block_N <= (m0 + block_M - 1)[None, None, :, None]
    block_count = cover.sum(-1).int()
    maxb = max(1, int(block_count.max()))
    order = torch.where(cover, kb, NK + kb).argsort(-1)[..., :maxb]
    block_offset = torch.where(torch.gather(cover, -1, order), order * block_N, torch.full_like(order, -1)).int()
    v = v_idx.long()[:, :, None, :]                                   # [B,H,1,NV]
    vcover = torch.gather(cover, -1, (v // block_N).clamp(max=NK - 1).expand(B, H, NQ, -1))
    vok = (v <= (m0 + block_M - 1)[None, None, :, None]) & ~vcover & (v < seq_len)
    column_count = vok.sum(-1).int()
    maxc = max(block_N, int((column_count.max() + block_N - 1) // block_N * block_N))
    vsorted = torch.where(vok, v.expand_as(vok), seq_len + v.expand_as(vok)).sort(-1).values[..., :maxc]
    if vsorted.shape[-1] < maxc:
        vsorted = torch.nn.functional.pad(vsorted, (0, maxc - vsorted.shape[-1]), value=2 * seq_len)
    column_index = torch.where(vsorted < seq_len, vsorted, torch.full_like(vsorted, -1)).int()
    return block_count.contiguous(), block_offset.contiguous(), column_count.contiguous(), column_index.contiguous()


@tilelang.jit(out_idx=[-1], pass_configs=FAST_MATH)
def vs_sparse_flashattn(batch, heads, seq_len, dim, max_blocks, max_cols, block_M=64, block_N=64, threads=256,
                        num_stages=2, dtype="float16", num_split=1):
    """``num_split`` > 1: each query block's key work (dense blocks, then column chunks) is divided
    over ``num_split`` workgroups, which write fp32 partial outputs and base-2 LSEs; a second kernel
    of the program combines them (short / lightly populated sequences at B1 H1 otherwise leave most
    CUs idle: 64 workgroups at 8K)."""
    scale = dim**-0.5 * LOG2E
    NQ = (seq_len + block_M - 1) // block_M
    NC = max_cols // block_N
    accum = "float"

    @T.macro
    def softmax_step(acc_s, acc_s_cast, acc_o, m, m_prev, alpha, l_sum, r_sum, V_s):
        # lazy rescale: O is rescaled only when one of the thread's rows moved its max by > 2^8
        T.copy(m, m_prev)
        T.reduce_max(acc_s, m_prev, dim=1, clear=False)  # candidate max
        rescale = T.alloc_var("int32")
        rescale = 0
        for i in T.Parallel(block_M):
            if (m_prev[i] - m[i]) * scale > 8.0:
                alpha[i] = T.exp2((m[i] - m_prev[i]) * scale)
                m[i] = m_prev[i]
                rescale = 1
            else:
                alpha[i] = 1.0
        if rescale != 0:
            for i, d in T.Parallel(block_M, dim):
                acc_o[i, d] *= alpha[i]
        for i, j in T.Parallel(block_M, block_N):
            acc_s[i, j] = T.exp2(acc_s[i, j] * scale - m[i] * scale)
        T.reduce_sum(acc_s, r_sum, dim=1)
        for i in T.Parallel(block_M):
            l_sum[i] = l_sum[i] * alpha[i] + r_sum[i]
        T.copy(acc_s, acc_s_cast)
        T.gemm(acc_s_cast, V_s, acc_o, policy=T.GemmWarpPolicy.FullRow)

    P = num_split

    @T.macro
    def attend(Q, K, V, BlockCount, BlockOffset, ColumnCount, ColumnIndex, bx, by, bz, sp, acc_o, m, l_sum):
        Q_s = T.alloc_shared([block_M, dim], dtype)
        K_s = T.alloc_shared([block_N, dim], dtype)
        V_s = T.alloc_shared([block_N, dim], dtype)
        cidx = T.alloc_shared([block_N], "int32")
        acc_s = T.alloc_fragment([block_M, block_N], accum)
        acc_s_cast = T.alloc_fragment([block_M, block_N], dtype)
        m_prev = T.alloc_fragment([block_M], accum)
        alpha = T.alloc_fragment([block_M], accum)
        r_sum = T.alloc_fragment([block_M], accum)
        T.copy(Q[bz, by, bx * block_M:(bx + 1) * block_M, :], Q_s)
        T.fill(acc_o, 0)
        T.fill(l_sum, 0)
        T.fill(m, -(2.0**30))
        nb_all = BlockCount[bz, by, bx]
        nb0 = nb_all * sp // P
        nb1 = nb_all * (sp + 1) // P
        for i in T.Pipelined(nb1 - nb0, num_stages=num_stages):
            k0 = T.max(BlockOffset[bz, by, bx, nb0 + i], 0)
            T.copy(K[bz, by, k0:k0 + block_N, :], K_s)
            T.copy(V[bz, by, k0:k0 + block_N, :], V_s)
            for r, c in T.Parallel(block_M, block_N):
                acc_s[r, c] = T.if_then_else((k0 + c <= bx * block_M + r) & (k0 + c < seq_len), 0,
                                             -T.infinity(accum))
            T.gemm(Q_s, K_s, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
            softmax_step(acc_s, acc_s_cast, acc_o, m, m_prev, alpha, l_sum, r_sum, V_s)
        nc_all = T.ceildiv(ColumnCount[bz, by, bx], block_N)
        nc0 = nc_all * sp // P
        nc1 = nc_all * (sp + 1) // P
        for j in T.Pipelined(nc1 - nc0, num_stages=num_stages):
            T.gather_rows(K[bz, by, :, :], ColumnIndex[bz, by, bx, (nc0 + j) * block_N:(nc0 + j + 1) * block_N], K_s)
            T.gather_rows(V[bz, by, :, :], ColumnIndex[bz, by, bx, (nc0 + j) * block_N:(nc0 + j + 1) * block_N], V_s)
            T.copy(ColumnIndex[bz, by, bx, (nc0 + j) * block_N:(nc0 + j + 1) * block_N], cidx)
            for r, c in T.Parallel(block_M, block_N):
                acc_s[r, c] = T.if_then_else((cidx[c] >= 0) & (cidx[c] <= bx * block_M + r), 0,
                                             -T.infinity(accum))
            T.gemm(Q_s, K_s, acc_s, transpose_B=True, policy=T.GemmWarpPolicy.FullRow)
            softmax_step(acc_s, acc_s_cast, acc_o, m, m_prev, alpha, l_sum, r_sum, V_s)

    if P == 1:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, seq_len, dim], dtype), K: T.Tensor([batch, heads, seq_len, dim], dtype),
                 V: T.Tensor([batch, heads, seq_len, dim], dtype), BlockCount: T.Tensor([batch, heads, NQ], "int32"),
                 BlockOffset: T.Tensor([batch, heads, NQ, max_blocks], "int32"),
                 ColumnCount: T.Tensor([batch, heads, NQ], "int32"),
                 ColumnIndex: T.Tensor([batch, heads, NQ, max_cols], "int32"),
                 Output: T.Tensor([batch, heads, seq_len, dim], dtype)):
            with T.Kernel(NQ, heads, batch, threads=threads) as (bx, by, bz):
                acc_o = T.alloc_fragment([block_M, dim], accum)
                m = T.alloc_fragment([block_M], accum)
                l_sum = T.alloc_fragment([block_M], accum)
                attend(Q, K, V, BlockCount, BlockOffset, ColumnCount, ColumnIndex, bx, by, bz, 0, acc_o, m, l_sum)
                for i, d in T.Parallel(block_M, dim):
                    acc_o[i, d] /= T.max(l_sum[i], 1e-30)
                T.copy(acc_o, Output[bz, by, bx * block_M:(bx + 1) * block_M, :])
    else:

        @T.prim_func
        def main(Q: T.Tensor([batch, heads, seq_len, dim], dtype), K: T.Tensor([batch, heads, seq_len, dim], dtype),
                 V: T.Tensor([batch, heads, seq_len, dim], dtype), BlockCount: T.Tensor([batch, heads, NQ], "int32"),
                 BlockOffset: T.Tensor([batch, heads, NQ, max_blocks], "int32"),
                 ColumnCount: T.Tensor([batch, heads, NQ], "int32"),
                 ColumnIndex: T.Tensor([batch, heads, NQ, max_cols], "int32"),
                 Opart: T.Tensor([batch, heads, P, seq_len, dim], accum),
                 Lse: T.Tensor([batch, heads, P, seq_len], accum),
                 Output: T.Tensor([batch, heads, seq_len, dim], dtype)):
            with T.Kernel(NQ, heads, batch * P, threads=threads) as (bx, by, bzp):
                bz = bzp // P
                sp = bzp % P
                acc_o = T.alloc_fragment([block_M, dim], accum)
                m = T.alloc_fragment([block_M], accum)
                l_sum = T.alloc_fragment([block_M], accum)
                attend(Q, K, V, BlockCount, BlockOffset, ColumnCount, ColumnIndex, bx, by, bz, sp, acc_o, m, l_sum)
                for i, d in T.Parallel(block_M, dim):
                    acc_o[i, d] /= T.max(l_sum[i], 1e-30)
                for i in T.Parallel(block_M):  # base-2 LSE; an empty split gets -inf weight
                    l_sum[i] = T.if_then_else(l_sum[i] > 0, T.log2(l_sum[i]) + m[i] * scale, -T.infinity(accum))
                T.copy(acc_o, Opart[bz, by, sp, bx * block_M:(bx + 1) * block_M, :])
                T.copy(l_sum, Lse[bz, by, sp, bx * block_M:(bx + 1) * block_M])
            with T.Kernel(T.ceildiv(seq_len, 64), heads, batch, threads=256) as (rx, hy, bz):
                for r, d in T.Parallel(64, dim):
                    row = rx * 64 + r
                    if row < seq_len:
                        mx = T.alloc_var(accum)
                        mx = -T.infinity(accum)
                        for q in T.serial(P):
                            mx = T.max(mx, Lse[bz, hy, q, row])
                        num = T.alloc_var(accum)
                        den = T.alloc_var(accum)
                        num = 0.0
                        den = 0.0
                        for q in T.serial(P):
                            w = T.exp2(Lse[bz, hy, q, row] - mx)
                            num = num + w * Opart[bz, hy, q, row, d]
                            den = den + w
                        Output[bz, hy, row, d] = T.Cast(dtype, num / T.max(den, 1e-30))

    return main


def vertical_slash_sparse_attention(q, k, v, v_idx, s_idx, block_M=128, block_N=None, threads=512, num_stages=2,
                                    num_split=None):
    """q/k/v [B, H, S, D]; v_idx [B, H, NV]; s_idx [B, H, NS] -> output [B, H, S, D].
    Tiles from scripts/minference_sweep.py at the reference's B1 H1 D64 (profiles/r6/minference_sweep*.log):
    128-row query blocks over 8 waves; 128-key blocks up to 32K keys (fewer, fuller pipeline steps:
    8K 0.279 -> 0.167 ms against the 64x64 / 4-wave tile), 64-key blocks beyond (finer slash coverage:
    64K 2.00 -> 1.40 ms).  ``num_split`` (default: enough splits for ~512 workgroups, at most 8) divides
    each query block's key work over several workgroups (combined by LSE)."""
    import torch
    B, H, S, D = q.shape
    if block_N is None:
        block_N = 128 if S <= 32768 else 64
    NQ = (S + block_M - 1) // block_M
    if num_split is None:
        num_split = max(1, min(8, 512 // max(1, NQ * H * B)))
    # merged unaligned slash segments attend fewer keys, which pays past 16K keys (32K / 64K:
    # -6..-13 % end to end); below that nearly every key block is covered anyway and the aligned
    # conversion's two serial prefix sums (instead of four) are the cheaper index pass
    # (profiles/r6/minference_table_merged.md against minference_table_split.md)
    bc, bo, cc, ci = convert_vertical_slash_indexes(v_idx, s_idx, S, block_M, block_N)
    k_ = vs_sparse_flashattn(B, H, S, D, bo.shape[-1], ci.shape[-1], block_M, block_N, threads=threads,
                             num_stages=num_stages, dtype=str(q.dtype).replace("torch.", ""), num_split=num_split)
    if num_split == 1:
        return k_(q, k, v, bc, bo, cc, ci)
    opart = torch.empty(B, H, num_split, S, D, device=q.device, dtype=torch.float32)
    lse = torch.empty(B, H, num_split, S, device=q.device, dtype=torch.float32)
    return k_(q, k, v, bc, bo, cc, ci, opart, lse)


def ref_program(q, k, v, v_idx, s_idx, block_M=64, block_N=64, merged=None):
    """Dense fp32 softmax over exactly the keys selected by convert_vertical_slash_indexes."""
    import torch
    B, H, S, D = q.shape
    bc, bo, cc, ci = convert_vertical_slash_indexes(v_idx, s_idx, S, block_M, block_N, merged)
    allowed = torch.zeros(B, H, S, S, dtype=torch.bool, device=q.device)
    NQ = bo.shape[2]
    for qb in range(NQ):
        rows = slice(qb * block_M, min(S, (qb + 1) * block_M))
        for b in range(B):
            for h in range(H):
                for off in bo[b, h, qb].tolist():
                    if off >= 0:
                        allowed[b, h, rows, off:off + block_N] = True
                for c in ci[b, h, qb].tolist():
                    if c >= 0:
                        allowed[b, h, rows, c] = True
    allowed &= torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
    s = torch.einsum("bhqd,bhkd->bhqk", q.float(), k.float()) * D**-0.5
    p = torch.softmax(s.masked_fill(~allowed, float("-inf")), -1).nan_to_num(0.0)
    return torch.einsum("bhqk,bhkd->bhqd", p, v.float())


def main(B=1, H=8, S=8192, D=128, n_vertical=1000, n_slash=200):
    import torch
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.float16) for _ in range(3))
    g = torch.Generator(device="cuda").manual_seed(0)
    v_idx = torch.stack([torch.randperm(S, device="cuda", generator=g)[:n_vertical]
                         for _ in range(B * H)]).view(B, H, -1)
    s_idx = torch.stack([torch.randperm(S, device="cuda", generator=g)[:n_slash] for _ in range(B * H)]).view(B, H, -1)
    s_idx[..., 0] = 0  # the main diagonal
    o = vertical_slash_sparse_attention(q, k, v, v_idx, s_idx)
    sub = slice(S - 128, S)
    ref = ref_program(q[:, :1], k[:, :1], v[:, :1], v_idx[:, :1], s_idx[:, :1])
    torch.testing.assert_close(o[:, :1, sub].float(), ref[:, :, sub], rtol=2e-2, atol=2e-2)
    print("All checks pass.")
    from tilelang.profiler import do_bench
    lat = do_bench(lambda: vertical_slash_sparse_attention(q, k, v, v_idx, s_idx))
    print(f"vertical-slash sparse attention B{B} H{H} S{S}: {lat:.3f} ms (index conversion + kernel)")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--seq", type=int, default=8192)
    a = p.parse_args()
    main(S=a.seq)
