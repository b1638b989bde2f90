"""CDNA4 (gfx950) MFMA fragment layouts and operand LDS swizzles.

Reference counterparts (CDNA3 16x16x16 only): ``src/layout/gemm_layouts.cc:62-298``
(``makeGemmFragmentCCDNA``, ``makeGemmFragmentACDNA``) and
``tilelang/intrinsics/mfma_layout.py``.  gfx950 doubles K per instruction:

* ``v_mfma_f32_16x16x32_{f16,bf16}`` — lane ``l`` holds ``A[l&15][8(l>>4)+j]`` and
  ``B[8(l>>4)+j][l&15]`` (j<8); C/D: ``col = l&15, row = 4(l>>4)+v``.
* ``v_mfma_f32_32x32x16_{f16,bf16}`` — lane holds ``A[l&31][8(l>>5)+j]``; C/D:
  ``col = l&31, row = (v&3) + 8(v>>2) + 4(l>>5)``.

The emitter issues ``mfma(B_frag, A_frag, acc)`` (operands swapped), so every
lane holds a *row* segment of C: ``C[m = l&15][n = 4(l>>4)+v]``.  That makes the
accumulator directly usable as the A operand of a following GEMM with the
k-permutation ``k = 16h + 4(l>>4) + v`` (``kperm=1``), the B side of which is read
with ``ds_read_b64_tr_b16`` from the same rows (guide §3 "An accumulator tile as
the next MFMA's operand").  This is what keeps FlashAttention's P in registers.
"""
from __future__ import annotations

import functools
import itertools
from typing import List, Optional, Sequence, Tuple

from .fragment import Digit, Fragment
from .layout import SwizzleLayout
from ..analysis import lds_bank

WAVE = 64


def mfma_shape(dtype_bits: int, prefer_32: bool = False) -> Tuple[int, int, int]:
    """(m, n, k) of the MFMA instruction used for an input element width."""
    if dtype_bits == 16:
        return (32, 32, 16) if prefer_32 else (16, 16, 32)
    if dtype_bits == 8:
        return (32, 32, 16) if prefer_32 else (16, 16, 32)
    if dtype_bits == 32:
        return (16, 16, 4)
    raise ValueError(f"no MFMA for {dtype_bits}-bit inputs")


def compute_warp_partition(M: int, N: int, num_warps: int, policy: int = 0, mtile: int = 16,
                           ntile: int = 16, read_cost: Optional[Tuple[int, int]] = None) -> Tuple[int, int]:
    """Split ``num_warps`` waves into ``warp_m x warp_n`` (reference gemm.cc:144-354).

    policy: 0 = Square (balance per-wave tile), 1 = FullRow (waves along M), 2 = FullCol (along N).
    ``read_cost`` = (ds_read instructions per 16 rows of A, per 16 columns of B) per 32-deep K
    step (1 for a K-contiguous LDS operand read with ds_read_b128, 2 for an MN-contiguous one
    read with two ds_read_b64_tr_b16): among equally square tilings, the one issuing fewer LDS
    read instructions wins (256x256 over 8 waves with B [K][N]: 2x4 issues 16 reads per step,
    4x2 issues 20 -- +1-2 % on the fp16 GEMM, profiles/r3/gemm_prefetch_ab.log).
    """
    cands = []
    for wm in range(1, num_warps + 1):
        if num_warps % wm:
            continue
        wn = num_warps // wm
        if M % (wm * mtile) or N % (wn * ntile):
            continue
        cands.append((wm, wn))
    if not cands:
        raise ValueError(f"cannot partition a {M}x{N} GEMM tile over {num_warps} waves "
                         f"(needs M%(warp_m*{mtile})==0 and N%(warp_n*{ntile})==0)")
    if policy == 1:
        return max(cands, key=lambda c: (c[0], -c[1]))
    if policy == 2:
        return max(cands, key=lambda c: (c[1], -c[0]))

    def score(c):
        wm, wn = c
        tm, tn = M // wm, N // wn
        reads = 0 if read_cost is None else (tm // 16) * read_cost[0] + (tn // 16) * read_cost[1]
        # prefer square per-wave tiles, then fewer LDS read instructions, then more waves along M
        return (abs(tm - tn) / max(tm, tn), reads, -wm)

    return min(cands, key=score)


def mfma_c_fragment(M: int, N: int, warp_m: int, warp_n: int, mn: Tuple[int, int] = (16, 16)) -> Fragment:
    """Accumulator layout of a ``M x N`` tile computed by ``warp_m x warp_n`` waves (swapped operands)."""
    WM, WN = M // warp_m, N // warp_n
    if mn == (16, 16):
        m_rep, n_rep = WM // 16, WN // 16
        thread = [Digit(0, WM, warp_m), Digit(1, WN, warp_n), Digit(1, 4, 4), Digit(0, 1, 16)]
        local = [Digit(0, 16, m_rep), Digit(1, 16, n_rep), Digit(1, 1, 4)]
    elif mn == (32, 32):
        m_rep, n_rep = WM // 32, WN // 32
        thread = [Digit(0, WM, warp_m), Digit(1, WN, warp_n), Digit(1, 4, 2), Digit(0, 1, 32)]
        local = [Digit(0, 32, m_rep), Digit(1, 32, n_rep), Digit(1, 8, 4), Digit(1, 1, 4)]
    else:
        raise ValueError(mn)
    return Fragment([M, N], _drop_unit(thread), _drop_unit(local), f"mfma_c{mn[0]}")


def mfma_c_fragment_direct(M: int, N: int, warp_m: int, warp_n: int) -> Fragment:
    """Accumulator of a 16x16 MFMA issued with operands in natural order (``mfma(A, B)``): lane
    ``l`` holds ``C[4(l>>4) + v][l & 15]``.  Used by the 2:4 sparse GEMM, whose sparse operand
    must be the instruction's A source, so the swap trick of the dense path is unavailable."""
    WM, WN = M // warp_m, N // warp_n
    m_rep, n_rep = WM // 16, WN // 16
    thread = [Digit(0, WM, warp_m), Digit(1, WN, warp_n), Digit(0, 4, 4), Digit(1, 1, 16)]
    local = [Digit(0, 16, m_rep), Digit(1, 16, n_rep), Digit(0, 1, 4)]
    return Fragment([M, N], _drop_unit(thread), _drop_unit(local), "mfma_c16_direct")


def mfma_a_fragment(M: int, K: int, warp_m: int, warp_n: int, kperm: int = 0, mn=(16, 16),
                    trans: bool = False) -> Fragment:
    """A operand held in registers (gemm_rs).  Replicated over the ``warp_n`` waves.
    ``trans``: the tile is stored [K, M] (``T.gemm(transpose_A=True)``): same registers, dims swapped.

    kperm=0: natural  k = 32*kk + 8*g + j
    kperm=1: C-layout compatible  k = 32*kk + 16*h + 4*g + v   (local order kk, h, v)
    """
    if trans:
        return transpose_fragment(mfma_a_fragment(M, K, warp_m, warp_n, kperm, mn))
    WM = M // warp_m
    if mn == (32, 32):
        return _mfma_a_fragment32(M, K, warp_m, warp_n, kperm)
    if mn != (16, 16):
        raise NotImplementedError(f"register A operand for MFMA {mn}")
    m_rep = WM // 16
    kk = K // 32
    thread = [Digit(0, WM, warp_m), Digit(-1, 1, warp_n)]
    if kperm == 0:
        thread += [Digit(1, 8, 4), Digit(0, 1, 16)]
        local = [Digit(0, 16, m_rep), Digit(1, 32, kk), Digit(1, 1, 8)]
    else:
        thread += [Digit(1, 4, 4), Digit(0, 1, 16)]
        local = [Digit(0, 16, m_rep), Digit(1, 16, 2 * kk), Digit(1, 1, 4)]
    return Fragment([M, K], _drop_unit(thread), _drop_unit(local), f"mfma_a_kperm{kperm}")


def transpose_fragment(f: Fragment) -> Fragment:
    """The same thread/register distribution over the transposed 2-D tile (dims 0 and 1 swapped):
    a register A operand stored [K, M] (``transpose_A``) holds exactly the values, registers and
    lanes of its [M, K] layout, so the MFMA consumes it unchanged."""
    sw = {0: 1, 1: 0}

    def flip(ds):
        return [Digit(sw.get(d.dim, d.dim), d.stride, d.size) for d in ds]

    return Fragment([f.shape[1], f.shape[0]], flip(f.thread_digits), flip(f.local_digits), f.name + "_t",
                    f.thread_offset)


def _mfma_a_fragment32(M: int, K: int, warp_m: int, warp_n: int, kperm: int) -> Fragment:
    """Register A operand of ``v_mfma_f32_32x32x16_{f16,bf16}`` (lane: row ``l&31``, k-half ``h=l>>5``).

    kperm=0: natural  k = 16*kk + 8*h + j                       (local order kk, j)
    kperm=1: the k order of a 32x32 accumulator used as the next GEMM's A operand:
             k = 16*kk + 8*(j>>2) + 4*h + (j&3)                  (local order kk, j>>2, j&3)
             -- C holds n = 32*ni + 8*(v>>2) + 4*h + (v&3), so registers v = 8s..8s+7 of tile ni
             are exactly the 8 values of k step kk = 2*ni + s (no data movement).
    """
    WM = M // warp_m
    m_rep, kk = WM // 32, K // 16
    thread = [Digit(0, WM, warp_m), Digit(-1, 1, warp_n)]
    if kperm == 0:
        thread += [Digit(1, 8, 2), Digit(0, 1, 32)]
        local = [Digit(0, 32, m_rep), Digit(1, 16, kk), Digit(1, 1, 8)]
    else:
        thread += [Digit(1, 4, 2), Digit(0, 1, 32)]
        local = [Digit(0, 32, m_rep), Digit(1, 16, kk), Digit(1, 8, 2), Digit(1, 1, 4)]
    return Fragment([M, K], _drop_unit(thread), _drop_unit(local), f"mfma32_a_kperm{kperm}")


def _drop_unit(digs: List[Digit]) -> List[Digit]:
    return [d for d in digs if d.size > 1]


# ---------------------------------------------------------------------------
# LDS operand swizzles, searched against the gfx950 bank model
# ---------------------------------------------------------------------------


def _read_patterns(kind: str, rows: int, cols: int, elem_bytes: int, row_base_step: int = 16) -> List[List[tuple]]:
    """Per-instruction lists of 64 (row, col) lane addresses for an operand read pattern.

    kind:
      'k_rows'  : K-contiguous operand, each lane reads 8 consecutive k (16 B for 16-bit data,
                  8 B for 8-bit) of row (l&15) at k-chunk (l>>4)    -> ds_read_b128 / b64
      'tr'      : MN-contiguous operand read with ds_read_b64_tr_b16 (natural k order)
      'tr_kperm': same, C-layout compatible k order (16h + 4g + q)
    """
    pats = []
    if kind == "k_rows16":
        # packed-fp4 operand of the scaled 16x16x128 MFMA: 64 bytes per row per K step, 16
        # consecutive bytes (32 e2m1) per lane -> one b128 read
        for r0 in range(0, min(rows, 64), row_base_step):
            for k0 in range(0, cols, 64):
                pats.append([(r0 + (l & 15), k0 + (l >> 4) * 16) for l in range(64)])
        return pats
    if kind in ("k_rows_32", "k_rows_i8_32"):
        # 32x32 MFMA K-contiguous operand: lane l reads row l & 31, 16 bytes at k-chunk (l >> 5)
        epl = 16 // max(1, elem_bytes)
        for r0 in range(0, min(rows, 64), 32):
            for k0 in range(0, cols, 2 * epl):
                pats.append([(r0 + (l & 31), k0 + (l >> 5) * epl) for l in range(64)])
        return pats
    if kind in ("tr32", "tr32_kperm"):
        # 32x32x16 MN-contiguous operand via ds_read_b64_tr_b16: lane (g, i) supplies row
        # k0 + 8 (g >> 1) + 4 h + q (kperm: k0 + 4 (g >> 1) + 8 h + q), cols c0 + 16 (g & 1) + 4 p
        for c0 in range(0, min(cols, 64), 32):
            for k0 in range(0, rows, 16):
                for h in range(2):
                    p = []
                    for l in range(64):
                        g, i = l >> 4, l & 15
                        q, pp = i >> 2, i & 3
                        r = k0 + 8 * (g >> 1) + 4 * h + q if kind == "tr32" else k0 + 4 * (g >> 1) + 8 * h + q
                        p.append((r, c0 + 16 * (g & 1) + 4 * pp))
                    pats.append(p)
        return pats
    if kind == "k_rows32mx":
        # fp8 operand of the block-scaled 16x16x128 MFMA in hardware K order: two b128 reads per
        # lane at byte 16g and 64 + 16g of the 128-byte K step (see tl/gemm.h gemm_ss_mx)
        for r0 in range(0, min(rows, 64), row_base_step):
            for k0 in range(0, cols, 128):
                for half in range(2):
                    pats.append([(r0 + (l & 15), k0 + (l >> 4) * 16 + 64 * half) for l in range(64)])
        return pats
    if kind == "k_rows24mx":
        # packed-fp6 operand of the block-scaled 16x16x128 MFMA: 96 bytes per row per K step,
        # lane group g takes the 24 bytes (32 fp6) at 24 g: three 8-byte reads (tl/gemm.h)
        for r0 in range(0, min(rows, 64), row_base_step):
            for k0 in range(0, cols, 96):
                for j in range(3):
                    pats.append([(r0 + (l & 15), k0 + (l >> 4) * 24 + 8 * j) for l in range(64)])
        return pats
    if kind in ("tr8", "tr8_32"):
        # MN-contiguous 8-bit operand via ds_read_b64_tr_b8 (tl/gemm.h ld_tr8_b8): lane (g, i)
        # supplies row k0 + 8 g + (i >> 1) [tr8_32: k0 + 32 g + 8 t + (i >> 1)], cols c0 + 8 (i & 1)
        nt = 4 if kind == "tr8_32" else 1
        kst = 128 if kind == "tr8_32" else 32
        for c0 in range(0, min(cols, 64), 16):
            for k0 in range(0, rows, kst):
                for t in range(nt):
                    pats.append([(k0 + (32 if nt == 4 else 8) * (l >> 4) + 8 * t + ((l & 15) >> 1),
                                  c0 + 8 * (l & 1)) for l in range(64)])
        return pats
    if kind == "k_rows32":
        # 8-bit operand of the scaled 16x16x128 MFMA: 32 consecutive bytes per lane, two b128 reads
        for r0 in range(0, min(rows, 64), row_base_step):
            for k0 in range(0, cols, 128):
                for half in range(2):
                    pats.append([(r0 + (l & 15), k0 + (l >> 4) * 32 + 16 * half) for l in range(64)])
        return pats
    if kind == "k_rows":
        k_per_lane = 8
        kstep = 4 * k_per_lane
        for r0 in range(0, min(rows, 64), row_base_step):
            for k0 in range(0, cols, kstep):
                pats.append([(r0 + (l & 15), k0 + (l >> 4) * k_per_lane) for l in range(64)])
    elif kind in ("tr", "tr_kperm"):
        # rows are k, cols are m/n; 16 columns per MFMA tile
        for c0 in range(0, min(cols, 64), 16):
            for k0 in range(0, rows, 32):
                for h in range(2):
                    p = []
                    for l in range(64):
                        g, i = l >> 4, l & 15
                        q, pp = i >> 2, i & 3
                        if kind == "tr":
                            r = k0 + 8 * g + 4 * h + q
                        else:
                            r = k0 + 16 * h + 4 * g + q
                        p.append((r, c0 + 4 * pp))
                    pats.append(p)
    else:
        raise ValueError(kind)
    return pats


def _instr_for(kind: str, elem_bytes: int) -> str:
    if kind in ("k_rows32", "k_rows16", "k_rows32mx", "k_rows_32", "k_rows_i8_32"):
        return "ds_read_b128"
    if kind in ("tr32", "tr32_kperm"):
        return "ds_read_b64_tr_b16"
    if kind == "k_rows":
        return "ds_read_b128" if elem_bytes == 2 else "ds_read_b64"
    if kind == "k_rows24mx":
        return "ds_read_b64"
    return "ds_read_b64_tr_b16"


def _candidates(cpr: int, max_row_bit: int = 6):
    # only chunk bits below the 256-byte bank row (16 chunks) change the bank of an access
    nbits = min(4, max(0, cpr.bit_length() - 1))
    max_row_bit = min(max_row_bit, 5)
    choices = [None] + list(range(max_row_bit))
    for combo in itertools.product(choices, repeat=nbits):
        bits = [(rb, cb) for cb, rb in enumerate(combo) if rb is not None]
        yield bits


def _native_costs(kind: str, rows: int, cols: int, elem_bytes: int, cands):
    """Modelled cycles of every candidate swizzle for one read pattern (csrc/core/lds.cc)."""
    from .._native import core
    pats = _read_patterns(kind, rows, cols, elem_bytes)
    flat = [v for p in pats for rc in p for v in rc]
    return core().swizzle_costs(_instr_for(kind, elem_bytes), flat, len(pats), cols, elem_bytes,
                                [list(c) for c in cands])


@functools.lru_cache(maxsize=None)
def choose_swizzle(kind: str, rows: int, cols: int, elem_bytes: int) -> Tuple[Tuple[int, int], ...]:
    """Pick the chunk-XOR swizzle with the fewest modelled LDS cycles for this read pattern
    (exhaustive over row-bit -> chunk-bit assignments, scored with the gfx950 bank model)."""
    cpr = cols * elem_bytes // 16
    # XOR on chunk bits below the largest power of two dividing the row keeps every chunk in its
    # row (a 12-chunk fp6 row: bits 0-1 only)
    cpr &= -cpr
    if cpr <= 1:
        return ()
    cands = [tuple(b) for b in _candidates(cpr, max_row_bit=min(6, max(1, rows.bit_length() - 1)))]
    cost = _native_costs(kind, rows, cols, elem_bytes, cands)
    best = min(range(len(cands)), key=lambda i: (int(cost[i]), len(cands[i])))
    return cands[best]


def swizzle_report(kind: str, rows: int, cols: int, elem_bytes: int, bits) -> dict:
    pats = _read_patterns(kind, rows, cols, elem_bytes)
    instr = _instr_for(kind, elem_bytes)
    lay = SwizzleLayout([rows, cols], elem_bytes, list(bits))
    base = SwizzleLayout([rows, cols], elem_bytes, [])
    cyc = sum(lds_bank.instruction_cycles(instr, [lay.forward(r, c)[0] * elem_bytes for r, c in p]) for p in pats)
    cyc0 = sum(lds_bank.instruction_cycles(instr, [base.forward(r, c)[0] * elem_bytes for r, c in p]) for p in pats)
    ideal = len(pats) * len(lds_bank.INSTRUCTIONS[instr][0])
    return {"instruction": instr, "cycles": cyc, "cycles_unswizzled": cyc0, "conflict_free": ideal}


@functools.lru_cache(maxsize=None)
def choose_swizzle_multi(kinds: Tuple[str, ...], rows: int, cols: int, elem_bytes: int):
    """Best swizzle for a tile read with several patterns (e.g. MLA's KV tile, read row-wise by
    Q.KV^T and transposed by P.KV): minimise the summed modelled cycles."""
    if len(kinds) == 1:
        return choose_swizzle(kinds[0], rows, cols, elem_bytes)
    cpr = cols * elem_bytes // 16
    cpr &= -cpr
    if cpr <= 1:
        return ()
    cands = [tuple(b) for b in _candidates(cpr, max_row_bit=min(6, max(1, rows.bit_length() - 1)))]
    total = [0] * len(cands)
    for kind in kinds:
        for i, c in enumerate(_native_costs(kind, rows, cols, elem_bytes, cands)):
            total[i] += c
    best = min(range(len(cands)), key=lambda i: (int(total[i]), len(cands[i])))
    return cands[best]


def operand_swizzle_multi(kinds, shape: Sequence[int], elem_bytes: int) -> SwizzleLayout:
    rows, cols = int(shape[-2]), int(shape[-1])
    kinds = tuple(sorted(set(kinds)))
    bits = choose_swizzle_multi(kinds, rows, cols, elem_bytes)
    return SwizzleLayout(list(shape), elem_bytes, list(bits), name="swz_" + "+".join(kinds))


def operand_swizzle(kind: str, shape: Sequence[int], elem_bytes: int) -> SwizzleLayout:
    rows, cols = int(shape[-2]), int(shape[-1])
    bits = choose_swizzle(kind, rows, cols, elem_bytes)
    return SwizzleLayout(list(shape), elem_bytes, list(bits), name=f"swz_{kind}")


def default_operand_swizzle(shape, elem_bytes: int) -> SwizzleLayout:
    return operand_swizzle("k_rows", shape, elem_bytes)
