"""K-half split of pipelined GEMM main loops (gfx950 "phased" GEMM schedule, part 1).

A canonical tile-GEMM main loop

    for k in T.Pipelined(K / BK, num_stages=2):
        T.copy(A[.., k*BK : +BK], A_s)        # A_s [BM][BK]  (or [BK][BM])
        T.copy(B[k*BK : +BK, ..], B_s)        # B_s [BK][BN]  (or [BN][BK])
        T.gemm(A_s, B_s, C)

is rewritten into two K halves with their own LDS tiles

        T.copy(A[.., k*BK : +BK/2], A_s0);  T.copy(A[.., k*BK+BK/2 : +BK/2], A_s1)
        T.copy(B[k*BK : +BK/2, ..], B_s0);  T.copy(B[k*BK+BK/2 : +BK/2, ..], B_s1)
        T.gemm(A_s0, B_s0, C);  T.gemm(A_s1, B_s1, C)

which computes the same thing, but makes each K half a contiguous LDS region that the
LDS-DMA engine can refill on its own (``global_load_lds`` writes 1 KiB lane-linear pieces).
The software pipeline (``pipeline.py``, ``phased`` schedule) then refills the K-half that the
matrix cores have just finished with, so two half-tiles stay in flight across every barrier and
no ``s_waitcnt vmcnt(0)`` sits in the main loop (guide §5 "The 256^2 8-phase template",
"Pipelining across barriers").

Applied when the loop matches that shape, both operands are 16-bit, BK = 64 (two 32-deep MFMA
K steps), num_stages = 2, and ``tl.gemm_phased`` is not disabled.

The 256x256x64 NT tile on 512 threads (``tl.gemm_quad``, default on) is instead marked
``quad``: the pipeline pass replaces the whole loop with ``tl::gemm_quad_nt`` (tl/gemm_quad.h,
the guide's 8-phase quadrant schedule; +8-10 % over the K-half schedule at 4096^3 / 8192^3).
"""
from __future__ import annotations

from typing import Optional

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import IntImm, as_int, binop
from .utils import Mutator, flatten_seq


def _k_dims(op: O.GemmOp):
    """(dim of A_s holding K, dim of B_s holding K) for 2-D shared operands."""
    return (0 if op.trans_A else 1), (1 if op.trans_B else 0)


def _split_copy(cp: O.CopyOp, kdim_dst: int, half: int, new_dst: Buffer, which: int) -> Optional[O.CopyOp]:
    """Copy of K-half ``which`` into ``new_dst``; the source dim that lands on ``kdim_dst``."""
    src, dst = cp.src, cp.dst
    dshape = dst.buffer.static_shape()
    if dshape is None or len(dshape) != 2 or dst.static_extents() != dshape:
        return None
    sext = src.static_extents()
    if sext is None:
        return None
    nonunit = [d for d, e in enumerate(sext) if e != 1]
    if len(nonunit) != 2 or [sext[d] for d in nonunit] != dshape:
        return None
    sd = nonunit[kdim_dst]
    region = list(src.region)
    m, e = region[sd]
    region[sd] = (binop("+", m, IntImm(which * half)), half)
    new_src = BufferRegion(src.buffer, region)
    dreg = [(IntImm(0), n) for n in new_dst.static_shape()]
    return O.CopyOp(new_src, BufferRegion(new_dst, dreg), cp.coalesced_width, cp.disable_tma, cp.eviction_policy)


def _split_gather(gp: O.GatherRowsOp, kdim_dst: int, half: int, new_dst: Buffer, which: int):
    """K-half ``which`` of a row gather into ``new_dst``: the gathered rows are the tile's M dim,
    the source's column dim (its last non-row, non-unit dim) is K."""
    dshape = gp.dst.buffer.static_shape()
    if dshape is None or len(dshape) != 2 or kdim_dst != 1 or gp.dst.static_extents() != dshape:
        return None
    sext = gp.src.static_extents()
    if sext is None:
        return None
    cols = [d for d, e in enumerate(sext) if d != gp.row_dim and e != 1]
    if len(cols) != 1 or sext[cols[0]] != dshape[1]:
        return None
    region = list(gp.src.region)
    m, e = region[cols[0]]
    region[cols[0]] = (binop("+", m, IntImm(which * half)), half)
    dreg = [(IntImm(0), n) for n in new_dst.static_shape()]
    return O.GatherRowsOp(BufferRegion(gp.src.buffer, region), gp.idx, BufferRegion(new_dst, dreg), gp.row_dim)


def _plus_const(e, base, c) -> bool:
    """``e`` is ``base + c`` (structurally)."""
    from ..ir.expr import BinOp, as_int, structural_equal
    return isinstance(e, BinOp) and e.op == "+" and as_int(e.b) == c and structural_equal(e.a, base)


def _minus_const(e, base, c) -> bool:
    from ..ir.expr import BinOp, as_int, structural_equal
    return isinstance(e, BinOp) and e.op == "-" and as_int(e.b) == c and structural_equal(e.a, base)


def quad_k(dtype):
    """K of one quad-loop tile: 128 bytes of a row (64 fp16/bf16, 128 fp8)."""
    return 128 // max(1, dtype.bits // 8)


QUAD_DTYPES = ("float16", "bfloat16", "float8_e4m3fn", "float8_e5m2")


def quad_loop_ok(stmts, threads, target) -> bool:
    """The loop body is the 256x256 NT tile GEMM with 128-byte K tiles that ``tl::gemm_quad_nt_x``
    (tl/gemm_quad.h) implements: A_s [256][KE] (a plain copy or a row gather), B_s [256][KE]
    (transpose_B), KE = 64 fp16/bf16 or 128 fp8 (OCP e4m3 / e5m2, the scaled 16x16x128 MFMA),
    512 threads on a 4x2 wave grid, fp32 fragment accumulator; optionally T.gemm(valid_m=) and
    the MoE extension GEMM -- A_x [32][KE] (rows 256..287 of the same copy or gather), the same
    B_s, 1x8 waves (FullCol), valid_m = the main valid_m - 256."""
    from ..ir import dtypes as _dt
    from . import gemm_lower
    if threads != 512:
        return False
    gemms = [x.op for x in stmts if isinstance(x, S.TileOpStmt) and isinstance(x.op, O.GemmOp)]
    prods = [x.op for x in stmts if isinstance(x, S.TileOpStmt) and isinstance(x.op, (O.CopyOp, O.GatherRowsOp))]
    if len(gemms) + len(prods) != len(stmts) or len(gemms) not in (1, 2):
        return False
    main = [g for g in gemms if g.A.buffer.static_shape() == [256, quad_k(g.A.buffer.dtype)]]
    if len(main) != 1:
        return False
    g = main[0]
    ke = quad_k(g.A.buffer.dtype)
    ext = [x for x in gemms if x is not g]
    x = ext[0] if ext else None

    def plain(op):
        return not (op.trans_A or not op.trans_B or op.is_mx or op.is_sp or op.clear_accum not in (False, None, 0) or
                    getattr(op, "valid_m_min", None) is not None or op.C.buffer.dtype != _dt.float32 or
                    op.A.buffer.scope != "shared" or op.B.buffer.scope != "shared")

    def warps(op, wm, wn):
        try:
            plan = gemm_lower.gemm_plan(op, threads, target)
        except Exception:  # noqa: BLE001 -- not plannable: the generic path reports it
            return False
        return plan.get("warp_m") == wm and plan.get("warp_n") == wn and tuple(plan.get("mfma") or ()) == (16, 16, 32)

    A, B = g.A.buffer, g.B.buffer
    if not plain(g) or B.static_shape() != [256, ke] or A.dtype.name not in QUAD_DTYPES or B.dtype != A.dtype:
        return False
    if not warps(g, 4, 2):
        return False
    dsts = {A, B}
    if x is not None:
        if not plain(x) or x.B.buffer is not B or x.A.buffer.static_shape() != [32, ke] or x.A.buffer.dtype != A.dtype:
            return False
        if x.C.buffer.static_shape() != [32, 256] or not warps(x, 1, 8):
            return False
        vm, vx = getattr(g, "valid_m", None), getattr(x, "valid_m", None)
        if (vm is None) != (vx is None) or (vm is not None and not _minus_const(vx, vm, 256)):
            return False
        dsts.add(x.A.buffer)
    by_dst = {p.dst.buffer: p for p in prods}
    if set(by_dst) != dsts or len(by_dst) != len(prods) or any(p.src.buffer.scope != "global" for p in prods):
        return False
    if not isinstance(by_dst[B], O.CopyOp):
        return False
    pa = by_dst[A]
    if x is not None:
        px = by_dst[x.A.buffer]
        if type(px) is not type(pa) or px.src.buffer is not pa.src.buffer:
            return False
        if isinstance(pa, O.GatherRowsOp):
            (mm, em), (mx, ex) = pa.idx.region[-1], px.idx.region[-1]
            if pa.row_dim != 0 or px.row_dim != 0 or as_int(em) != 256 or as_int(ex) != 32 or \
                    not _plus_const(mx, mm, 256):
                return False
        else:
            if not _plus_const(px.src.region[0][0], pa.src.region[0][0], 256):
                return False
    elif isinstance(pa, O.GatherRowsOp) and (pa.row_dim != 0 or as_int(pa.idx.region[-1][1]) != 256):
        return False
    return True


class _QuadMark(Mutator):
    """Marks the T.Pipelined loops ``quad_loop_ok`` accepts (``quad`` annotation): the pipeline
    pass replaces them with ``tl::gemm_quad_nt_x`` (pipeline.py _quad_schedule), ksplit skips them."""

    def __init__(self, threads, target):
        self.threads, self.target = threads, target
        self.count = 0

    def visit_ForStmt(self, s: S.ForStmt):
        body = self.stmt(s.body)
        ann = dict(s.annotations)
        if s.kind == "pipelined" and int(ann.get("num_stages", 0)) == 2 and not ann.get("order") and \
                not ann.get("stage") and quad_loop_ok(flatten_seq(body), self.threads, self.target):
            ann["quad"] = True
            self.count += 1
        return S.ForStmt(s.var, s.min, s.extent, s.kind, body, ann)

    def visit_AllocStmt(self, s):
        return s


def mark_quad_loops(kernel: S.KernelStmt, threads: int, target) -> S.KernelStmt:
    qm = _QuadMark(threads, target)
    k = qm.stmt(kernel)
    return k if qm.count else kernel


class _KSplit(Mutator):

    def __init__(self, mode=True):
        self.mode = mode
        self.new_allocs = {}  # old buffer -> (half0, half1)
        self.pairs = {}       # A tile <-> B tile of one split GEMM
        self.applied = 0

    def visit_ForStmt(self, s: S.ForStmt):
        body = self.stmt(s.body)
        loop = S.ForStmt(s.var, s.min, s.extent, s.kind, body, s.annotations)
        if s.kind != "pipelined" or int(s.annotations.get("num_stages", 0)) != 2:
            return loop
        if s.annotations.get("order") or s.annotations.get("stage") or s.annotations.get("quad"):
            return loop
        stmts = flatten_seq(body)
        gemms = [x for x in stmts if isinstance(x, S.TileOpStmt) and isinstance(x.op, O.GemmOp)]
        copies = [x for x in stmts if isinstance(x, S.TileOpStmt) and isinstance(x.op, (O.CopyOp, O.GatherRowsOp))]
        if len(gemms) != 1 or len(copies) != 2 or len(stmts) != 3:
            return loop
        g = gemms[0].op
        if g.is_mx or g.is_sp:
            return loop
        A, B = g.A.buffer, g.B.buffer
        if A.scope != "shared" or B.scope != "shared" or A.dtype.bits != 16 or B.dtype != A.dtype:
            return loop
        if g.C.buffer.scope != "fragment":
            return loop
        cps = {c.op.dst.buffer: c.op for c in copies}
        if set(cps) != {A, B} or any(c.op.src.buffer.scope != "global" for c in copies):
            return loop
        ka, kb = _k_dims(g)
        sa, sb = A.static_shape(), B.static_shape()
        if sa is None or sb is None or len(sa) != 2 or len(sb) != 2 or sa[ka] != 64 or sb[kb] != 64:
            return loop
        if g.A.static_extents() != sa or g.B.static_extents() != sb:
            return loop
        half = 32
        parts = {}
        for buf, kd in ((A, ka), (B, kb)):
            shp = list(buf.static_shape())
            shp[kd] = half
            if buf in self.new_allocs:  # a second phased loop over the same operand tile reuses its halves
                h0, h1 = self.new_allocs[buf]
            else:
                h0 = Buffer(buf.name + "_k0", shp, buf.dtype, "shared")
                h1 = Buffer(buf.name + "_k1", shp, buf.dtype, "shared")
            split = _split_gather if isinstance(cps[buf], O.GatherRowsOp) else _split_copy
            c0 = split(cps[buf], kd, half, h0, 0)
            c1 = split(cps[buf], kd, half, h1, 1)
            if c0 is None or c1 is None:
                return loop
            c0.khalf, c1.khalf = 0, 1
            parts[buf] = (h0, h1, c0, c1)
        new = []
        for buf in (A, B):
            h0, h1, c0, c1 = parts[buf]
            new += [S.TileOpStmt(c0), S.TileOpStmt(c1)]
        for i in range(2):
            gi = O.GemmOp(BufferRegion(parts[A][i], [(IntImm(0), n) for n in parts[A][i].static_shape()]),
                          BufferRegion(parts[B][i], [(IntImm(0), n) for n in parts[B][i].static_shape()]),
                          g.C, g.trans_A, g.trans_B, g.policy, g.clear_accum if i == 0 else False, g.k_pack,
                          g.wg_wait)
            gi.mfma_shape = g.mfma_shape
            gi.valid_m = getattr(g, "valid_m", None)
            gi.khalf = i
            new.append(S.TileOpStmt(gi))
        for buf in (A, B):
            self.new_allocs[buf] = parts[buf][:2]
        self.pairs[A], self.pairs[B] = B, A
        self.applied += 1
        ann = dict(s.annotations)
        ann["phased"] = self.mode
        return S.ForStmt(s.var, s.min, s.extent, s.kind, S.SeqStmt(new), ann)

    def visit_AllocStmt(self, s):
        return s


class _AllocSplit(Mutator):
    """Allocates the halves as A_k0, B_k0, A_k1, B_k1 at the first of the two tiles' allocations:
    the LDS arena follows allocation order, so the A and B tiles one phase reads sit within
    64 KiB of each other and every ds_read of the phase addresses them from one base register
    with the 16-bit immediate offset (A_k1 and B_k1 64 KiB apart cost 2 VALU per read pair)."""

    def __init__(self, new_allocs, used, pairs):
        self.new_allocs = new_allocs
        self.used = used
        self.pairs = pairs
        self.done = set()

    def visit_AllocStmt(self, s):
        if s.buffer in self.new_allocs:
            keep = [s] if s.buffer in self.used else []
            if s.buffer in self.done:
                return S.seq(*keep) if keep else S.SeqStmt([])
            other = self.pairs.get(s.buffer)
            first = [s.buffer] + ([other] if other is not None and other in self.new_allocs and other not in self.done
                                  else [])
            order = [self.new_allocs[b][0] for b in first] + [self.new_allocs[b][1] for b in first]
            self.done.update(first)
            return S.seq(*(keep + [S.AllocStmt(h) for h in order]))
        return s


def split_gemm_k_halves(kernel: S.KernelStmt, mode=True) -> S.KernelStmt:
    """``mode``: True, or "prio" to also raise the wave priority around each MFMA cluster.
    Loops marked ``quad`` (mark_quad_loops) are left whole."""
    ks = _KSplit(mode)
    k = ks.stmt(kernel)
    if not ks.applied:
        return kernel
    from .pipeline import _referenced_buffers
    used = _referenced_buffers(k)
    return _AllocSplit(ks.new_allocs, used, ks.pairs).stmt(k)
