"""Software pipelining of ``T.Pipelined`` loops (tile level).

Reference: ``src/transform/pipeline_planning.cc`` (derives stage/order from
``num_stages``; async stages when the target has async copy) and
``inject_pipeline.cc`` (prologue/body/epilogue, multi-versioned buffers).

MI355X design (guide §5 "Pipelining across barriers", T3/T4):
  * every global->shared ``T.copy`` in the loop body is a *producer*; its shared
    buffer is multi-versioned ``num_stages`` deep (one LDS arena slot per stage);
  * producers that are eligible become **LDS-DMA** (``global_load_lds_dwordx4``)
    issued ``num_stages-1`` iterations ahead; the loop waits with a *counted*
    ``s_waitcnt vmcnt(N)`` and a raw ``s_barrier`` (no ``vmcnt(0)`` drain), so
    ``num_stages-2`` tiles stay in flight across every barrier;
  * other producers are **register staged** (T14 "issue-early / write-late"): the
    global loads of tile k+1 are issued before the compute of tile k and written
    to LDS after it;
  * one barrier per iteration orders both the RAW hazard on tile k and the WAR
    hazard on the slot being refilled.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir import lowered as L
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import PrimExpr, Var, IntImm, as_int, binop, convert, divisible_by, free_vars, substitute
from ..ir import dtypes as _dt
from ..layout.layout import Layout, LinearLayout, SwizzleLayout
from .utils import BufferReplacer, Mutator, bound, flatten_seq


import logging as _logging

_log = _logging.getLogger("tilelang.pipeline")

class AsyncCopyOp(O.TileOp):
    """Global->LDS DMA copy (lowered to ``tl::glds16``)."""
    kind = "async_copy"

    def __init__(self, src: BufferRegion, dst: BufferRegion, plan: dict, idx: Optional[BufferRegion] = None,
                 key: Optional[int] = None):
        # gathers: ``idx`` = the row indices; ``key`` names the register array they were
        # prefetched into (GatherIndexOp, one pipeline step earlier), None = load at issue
        self.src, self.dst, self.plan, self.idx, self.key = src, dst, plan, idx, key

    def regions(self):
        return [self.src, self.dst] + ([self.idx] if self.idx is not None else [])

    def reads(self):
        return [self.src] + ([self.idx] if self.idx is not None else [])

    def writes(self):
        return [self.dst]


class QuadGemmLoopOp(O.TileOp):
    """A whole 256x256x64 NT GEMM main loop as ``tl::gemm_quad_nt_x`` (tl/gemm_quad.h): ``a`` / ``b``
    are the global tiles of the first K step (``a_rdim`` / ``b_rdim`` their row dims); ``idx`` the
    row list of a gathered A (None: dense); ``lds_a`` / ``lds_b`` / ``lds_x`` the 2-stage LDS rings;
    ``n`` the K-step count; ``C`` (and the extension's ``Cx``) keep their GEMMs' fragment layouts;
    ``m_limit`` the main GEMM's valid_m (None: all rows)."""
    kind = "gemm_quad_loop"

    def __init__(self, a: BufferRegion, a_rdim: int, idx: Optional[BufferRegion], b: BufferRegion, b_rdim: int,
                 lds_a: Buffer, lds_b: Buffer, lds_x: Optional[Buffer], C: BufferRegion, Cx: Optional[BufferRegion],
                 n, m_limit=None, row_mode=False, b_row_mode=False, k_len=None):
        # row_mode: dense A whose row range is not provable -- rows from the tile's first row,
        # range-checked against the tensor (tl::gemm_quad_nt_x GATHER with a null row list);
        # b_row_mode: the same for B's rows (ragged N); k_len: the tensors' K when the last K
        # tile runs past it (its chunks at or past k_len read zeros)
        self.row_mode, self.b_row_mode, self.k_len = row_mode, b_row_mode, k_len
        self.a, self.a_rdim, self.idx, self.b, self.b_rdim = a, a_rdim, idx, b, b_rdim
        self.lds_a, self.lds_b, self.lds_x, self.C, self.Cx, self.n, self.m_limit = \
            lds_a, lds_b, lds_x, C, Cx, n, m_limit

    def regions(self):
        return [r for r in (self.a, self.idx, self.b, self.C, self.Cx) if r is not None]

    def reads(self):
        return [r for r in (self.a, self.idx, self.b, self.C, self.Cx) if r is not None]

    def writes(self):
        return [r for r in (self.C, self.Cx) if r is not None]


class GatherIndexOp(O.TileOp):
    """Prefetch of a gather's row indices into registers (one per LDS-DMA instruction and lane),
    issued a step ahead of the DMA that consumes them, so the index load latency never sits
    between the barrier and the DMA issue."""
    kind = "gather_index"

    def __init__(self, idx: BufferRegion, plan: dict, key: int):
        self.idx, self.plan, self.key = idx, plan, key

    def regions(self):
        return [self.idx]

    def reads(self):
        return [self.idx]


class StagedCopyOp(O.TileOp):
    """Register-staged copy split in two phases sharing a staging register array."""
    kind = "staged_copy"

    def __init__(self, src: BufferRegion, dst: BufferRegion, phase: str, key: int):
        self.src, self.dst, self.phase, self.key = src, dst, phase, key

    def regions(self):
        return [self.src, self.dst]

    def reads(self):
        return [self.src] if self.phase == "load" else []

    def writes(self):
        return [self.dst] if self.phase == "store" else []


def stage_layout(layout: Optional[Layout], shape: List[int], stages: int) -> Layout:
    if layout is None:
        return LinearLayout([stages] + list(shape))
    if isinstance(layout, SwizzleLayout):
        return SwizzleLayout([stages] + list(layout.shape), layout.elem_bytes, layout.bits, layout.name)
    if isinstance(layout, LinearLayout):
        return LinearLayout([stages] + list(layout.shape))
    size = 1
    for s in (layout.output_shape or shape):
        size *= int(s)
    inner = layout

    def fwd(s, *idx):
        return [s * size + inner.offset(*idx)]

    return Layout([stages] + list(shape), fwd, None, [stages * size], name=f"stage_{layout.name}")


def _squeeze(ext):
    ext = list(ext)
    while len(ext) > 2 and ext[0] == 1:
        ext = ext[1:]
    return ext


def glds_plan(op: O.CopyOp, num_threads: int, ranges, target, k_tail: bool = False) -> Optional[dict]:
    """Decide whether a global->shared copy can be a lane-linear LDS-DMA; return its geometry.
    ``k_tail`` (the quad GEMM loop only): the innermost (contiguous) dim may also run past the
    tensor -- a ragged last K tile, zero-filled chunk by chunk by tl::gemm_quad_nt_x (``ktail``)."""
    if target is not None and getattr(target, "kind", "hip") != "hip":
        return None
    if getattr(target, "disable_glds", False):
        return None
    src, dst = op.src, op.dst
    sb, db = src.buffer, dst.buffer
    if sb.scope != "global" or db.scope != "shared" or sb.dtype != db.dtype:
        return None
    eb = sb.dtype.bytes
    dext = dst.static_extents()
    dshape = db.static_shape()
    if dext is None or dshape is None or dext != dshape or len(dshape) not in (1, 2):
        return None
    nw = num_threads // 64
    dw = nw
    if len(dshape) == 1 or (dshape[0] * dshape[1] * eb) % (1024 * nw):
        if getattr(target, "disable_small_dma", False):
            return None
        sp = _small_dma_plan(op, num_threads, ranges)
        nbytes = dshape[0] * dshape[1] * eb if len(dshape) == 2 else 0
        if sp is not None or len(dshape) == 1 or nbytes % 1024 or nw % (nbytes // 1024):
            return sp
        # whole 1 KiB wave pieces, fewer than the waves: the extra waves re-fetch a covered piece
        # (same bytes, same LDS address; uniform DMA count per wave for the counted waits)
        dw = nbytes // 1024
    R, C = dshape
    if (C * eb) % 16:
        return None
    lay = db.layout
    if lay is not None and not isinstance(lay, (SwizzleLayout, LinearLayout)):
        return None
    # map the two tile dims onto source dims (skip unit dims)
    sext = src.static_extents()
    if sext is None:
        return None
    nonunit = [d for d, e in enumerate(sext) if e != 1]
    if R == 1:
        if len(nonunit) != 1 or sext[nonunit[0]] != C:
            return None
        rdim, cdim = None, nonunit[0]
    else:
        if len(nonunit) != 2 or sext[nonunit[0]] != R or sext[nonunit[1]] != C:
            return None
        rdim, cdim = nonunit
    strides = sb.get_strides()
    if as_int(strides[cdim]) != 1:
        return None
    # 16-byte alignment of every source chunk: row stride and column start
    epc = 16 // eb
    if rdim is not None:
        rs = strides[rdim]
        if not divisible_by(convert(rs), epc):
            return None
    if not divisible_by(src.region[cdim][0], epc):
        return None
    # in-bounds proof for every dim.  A data-dependent offset along the OUTERMOST tensor dim
    # (MoE expert rows, expert ids) is still fine: leaving that dim leaves the tensor, so a
    # buffer-resource LDS-DMA (hardware zero fill past num_records) gives exactly the
    # zero-padded tile — no register staging needed.
    shape = sb.shape
    oob = False
    ktail = None
    last = len(src.region) - 1
    for d, (m, e) in enumerate(src.region):
        b = bound(m, ranges)
        s = as_int(shape[d])
        ev = as_int(e)
        if b is None or s is None or ev is None or b[0] < 0 or b[1] + ev > s:
            if d == 0 and ev is not None:
                oob = True
                continue
            if k_tail and d == last and d > 0 and s is not None and b is not None and b[0] >= 0 and \
                    (s * eb) % 16 == 0 and as_int(strides[d]) == 1:
                ktail = s  # chunks at or past column s read zeros (whole 16-byte chunks: s*eb % 16 == 0)
                continue
            return None
    nbytes = None
    if oob:
        numel = 1
        for s in shape:
            if as_int(s) is None:
                return None
            numel *= as_int(s)
        st0 = as_int(strides[0])
        if st0 is None or sb.strides is not None or numel * eb >= (1 << 31):
            return None
        nbytes = numel * eb
    n_chunks = R * C * eb // 16
    return dict(R=R, C=C, eb=eb, rdim=rdim, cdim=cdim, instrs=n_chunks // 64 // dw, nwaves=dw, cpr=C * eb // 16,
                oob_bytes=nbytes, dup=dw < nw, ktail=ktail)


def _small_dma_plan(op: O.CopyOp, num_threads: int, ranges) -> Optional[dict]:
    """LDS-DMA for a tile smaller than one 16-byte DMA per lane of the workgroup (MX scale tiles,
    per-row LSE / Delta vectors): every wave issues exactly ONE 4-byte buffer LDS-DMA
    (``tl::buffer_lds4``), lane chunk ``P = wave * 64 + lane``; lanes past the tile get an
    out-of-range offset (the hardware writes a zero and reads nothing) and land in padding of the
    stage slot, which is sized ``waves * 256`` bytes.  One instruction per wave keeps the counted
    ``vmcnt`` waits uniform; the alternative -- a register-staged copy -- needs its global load
    retired before its ds_write, and the compiler's conservative LDS-DMA alias wait in front of that
    ds_write is ``vmcnt(0)``, which drained the whole ring every iteration."""
    src, dst = op.src, op.dst
    sb, db = src.buffer, dst.buffer
    eb = sb.dtype.bytes
    dshape = db.static_shape()
    nw = num_threads // 64
    total = 1
    for d in dshape:
        total *= d
    if (total * eb) % 4 or total * eb > 256 * nw or eb > 4:
        return None
    lay = db.layout
    if lay is not None and not (isinstance(lay, LinearLayout) or (isinstance(lay, SwizzleLayout) and not lay.bits)):
        return None
    R, C = (1, dshape[0]) if len(dshape) == 1 else dshape
    if (C * eb) % 4:
        return None
    sext = src.static_extents()
    if sext is None:
        return None
    nonunit = [d for d, e in enumerate(sext) if e != 1]
    if R == 1:
        if len(nonunit) != 1 or sext[nonunit[0]] != C:
            return None
        rdim, cdim = None, nonunit[0]
    else:
        if len(nonunit) != 2 or sext[nonunit[0]] != R or sext[nonunit[1]] != C:
            return None
        rdim, cdim = nonunit
    strides = sb.get_strides()
    if as_int(strides[cdim]) != 1:
        return None
    epc = max(1, 4 // eb)  # elements per 4-byte chunk
    if rdim is not None and not divisible_by(convert(strides[rdim]), epc):
        return None
    if not divisible_by(src.region[cdim][0], epc):
        return None
    shape = sb.shape
    for d, (m, e) in enumerate(src.region):  # outer dim may leave the tensor (zero fill), others not
        b = bound(m, ranges)
        s_ = as_int(shape[d])
        ev = as_int(e)
        if b is None or s_ is None or ev is None or b[0] < 0 or b[1] + ev > s_:
            if d == 0 and ev is not None:
                continue
            return None
    numel = 1
    for s_ in shape:
        if as_int(s_) is None:
            return None
        numel *= as_int(s_)
    if sb.strides is not None or numel * eb >= (1 << 31):
        return None
    return dict(small=True, R=R, C=C, eb=eb, rdim=rdim, cdim=cdim, cpr=C * eb // 4, instrs=1, nwaves=nw,
                nchunks=total * eb // 4, oob_bytes=numel * eb, pad_elems=nw * 256 // eb)


def _padded_stage_layout(shape: List[int], stages: int, pad_elems: int) -> Layout:
    """Row-major stage slots of ``pad_elems`` elements each (small-tile DMA padding)."""
    strides = []
    acc = 1
    for d in reversed(shape):
        strides.append(acc)
        acc *= d
    strides = strides[::-1]

    def fwd(s, *idx):
        off = s * pad_elems
        for i, st in zip(idx, strides):
            off = off + i * st
        return [off]

    return Layout([stages] + list(shape), fwd, None, [stages * pad_elems], name="stage_padded")


def gather_plan(op: O.GatherRowsOp, num_threads: int, target) -> Optional[dict]:
    """LDS-DMA geometry of a row gather: every lane fetches one 16-byte chunk of the row its
    chunk belongs to, addressed through a buffer resource (out-of-range rows -> zeros)."""
    if target is not None and getattr(target, "kind", "hip") != "hip":
        return None
    if getattr(target, "disable_glds", False):
        return None
    src, dst = op.src, op.dst
    sb, db = src.buffer, dst.buffer
    if sb.scope != "global" or db.scope != "shared" or sb.dtype != db.dtype:
        return None
    eb = sb.dtype.bytes
    dext, dshape = dst.static_extents(), db.static_shape()
    if dext is None or dshape is None or dext != dshape or len(dshape) != 2:
        return None
    R, C = dshape
    nw = num_threads // 64
    if (C * eb) % 16:
        return None
    # a tile smaller than one 16-byte chunk per lane of the workgroup (e.g. a 32-row MoE
    # extension tile): the first ``dw`` waves' chunks cover it and every further wave re-fetches
    # the chunk of wave (w mod dw) -- identical bytes to the same LDS address -- so each wave still
    # issues the same number of DMA instructions per stage (the counted vmcnt waits stay uniform)
    dw = nw
    if (R * C * eb) % (1024 * nw):
        if (R * C * eb) % 1024 or nw % ((R * C * eb) // 1024):
            return None
        dw = (R * C * eb) // 1024
    lay = db.layout
    if lay is not None and not isinstance(lay, (SwizzleLayout, LinearLayout)):
        return None
    cpr = C * eb // 16
    if cpr % 64 and 64 % cpr:
        return None
    rdim = op.row_dim
    sext = src.static_extents()
    if sext is None:
        return None
    cols = [d for d, e in enumerate(sext) if d != rdim and e != 1]
    if len(cols) != 1 or sext[cols[0]] != C:
        return None
    cdim = cols[0]
    strides = sb.get_strides()
    epc = 16 // eb
    if as_int(strides[cdim]) != 1 or not divisible_by(convert(strides[rdim]), epc) or \
            not divisible_by(src.region[cdim][0], epc):
        return None
    iext = [as_int(e) for e in op.idx.extents]
    if None in iext or [e for e in iext if e != 1] not in ([R], []) or _prod_i(iext) != R:
        return None
    return dict(R=R, C=C, eb=eb, rdim=rdim, cdim=cdim, instrs=R * C * eb // 16 // 64 // dw, nwaves=dw, cpr=cpr,
                gather=True, dup=dw < nw)


def _prod_i(xs):
    r = 1
    for x in xs:
        r *= x
    return r


class _Ranges:

    def __init__(self):
        self.r: Dict[Var, tuple] = {}


def _var_ranges_for_kernel(k: S.KernelStmt) -> Dict[Var, tuple]:
    r = {}
    for v, g in zip(k.block_vars, k.grid):
        gv = as_int(g)
        if gv is not None:
            r[v] = (0, gv - 1)
    tot = k.num_threads
    for v, t in zip(k.thread_vars, k.threads):
        r[v] = (0, int(t) - 1)
    return r


class PipelineInjector(Mutator):

    def __init__(self, kernel: S.KernelStmt, num_threads: int, target):
        self.kernel = kernel
        self.T = num_threads
        self.target = target
        self.ranges = _var_ranges_for_kernel(kernel)
        self.key = 0

    def visit_ForStmt(self, s: S.ForStmt):
        mn, ext = as_int(s.min), as_int(s.extent)
        if mn is not None and ext is not None and ext > 0:
            self.ranges[s.var] = (mn, mn + ext - 1)
        body = self.stmt(s.body)
        if s.kind != "pipelined":
            return S.ForStmt(s.var, s.min, s.extent, s.kind, body, s.annotations)
        return self.pipeline(S.ForStmt(s.var, s.min, s.extent, s.kind, body, s.annotations))

    def visit_LetStmt(self, s):
        b = bound(s.value, self.ranges)  # clamped table lookups stay provably in bounds
        if b is not None:
            self.ranges[s.var] = b
        return s

    def pipeline(self, loop: S.ForStmt):
        nstages = int(loop.annotations.get("num_stages", 0))
        stmts = flatten_seq(loop.body)
        serial = S.ForStmt(loop.var, loop.min, loop.extent, "serial", loop.body,
                           {k: v for k, v in loop.annotations.items() if k != "num_stages"})
        if nstages < 2 or getattr(self.target, "kind", "hip") == "cpu":
            return serial
        k, n = loop.var, loop.extent
        lets: Dict[Var, PrimExpr] = {}
        producers = []
        written_elsewhere = set()
        for st in stmts:
            if isinstance(st, S.LetStmt):
                lets[st.var] = substitute(st.value, lets)
            elif isinstance(st, S.TileOpStmt) and isinstance(st.op, O.CopyOp) and \
                    st.op.src.buffer.scope == "global" and st.op.dst.buffer.scope == "shared":
                producers.append(st)
            elif isinstance(st, S.TileOpStmt) and isinstance(st.op, O.GatherRowsOp) and \
                    gather_plan(st.op, self.T, self.target) is not None:
                producers.append(st)  # gathers have no register-staged form: async or in-loop
            else:
                for w in S.walk(st):
                    if isinstance(w, S.TileOpStmt):
                        for r in w.op.writes():
                            written_elsewhere.add(r.buffer)
                    if isinstance(w, S.StoreStmt):
                        written_elsewhere.add(w.buffer)
        producers = [p for p in producers if p.op.dst.buffer not in written_elsewhere]
        if not producers:
            return serial
        allowed = set(free_vars_stmt_outer(self.kernel)) | {k}
        prods = []
        for p in producers:
            src = _subst_region(p.op.src, lets)
            fv = set()
            for m, e in src.region:
                fv |= {id(v) for v in free_vars(m)}
            loop_local = {id(v) for v in lets}  # unresolved lets would appear as themselves
            prods.append((p, src))
        # classify producers
        rng = dict(self.ranges)
        if as_int(loop.min) is not None and as_int(loop.extent) is not None:
            rng[k] = (as_int(loop.min), as_int(loop.min) + as_int(loop.extent) - 1)
        else:
            # data-dependent trip counts (causal / windowed attention): interval of the loop
            # var from the bounds of its start and end, so LDS-DMA stays provably in bounds
            # (only the start's lower bound and the end's upper bound matter: half-open intervals
            # such as max(0, data-dependent) starts still give a finite loop-var range)
            from .utils import _bound
            lo = _bound(loop.min, self.ranges)
            ext = loop.extent
            from ..ir.expr import BinOp, structural_equal
            if isinstance(ext, BinOp) and ext.op == "-" and structural_equal(ext.b, loop.min):
                hi = _bound(ext.a, self.ranges)  # T.Pipelined(start, end): extent = end - start
            else:
                hi = _bound(binop("+", loop.min, ext), self.ranges)
            inf = float("inf")
            if lo is not None and hi is not None and abs(lo[0]) != inf and abs(hi[1]) != inf:
                rng[k] = (int(lo[0]), int(max(lo[0], hi[1] - 1)))
        asyncs, staged = [], []
        for p, src in prods:
            if isinstance(p.op, O.GatherRowsOp):
                asyncs.append((p, src, gather_plan(p.op, self.T, self.target)))
                continue
            plan = glds_plan(O.CopyOp(src, p.op.dst), self.T, rng, self.target)
            if plan is None and loop.annotations.get("quad") and nstages == 2:
                # the quad GEMM loop zero-fills a ragged last K tile itself (tl/gemm_quad.h ktail)
                plan = glds_plan(O.CopyOp(src, p.op.dst), self.T, rng, self.target, k_tail=True)
            if plan is not None and plan.get("ktail") and not loop.annotations.get("quad"):
                plan = None
            if plan is not None:
                asyncs.append((p, src, plan))
            else:
                staged.append((p, src))
                _log.debug("register-staged pipeline copy %s -> %s (not provably in bounds / not DMA-shaped): %s",
                           src.buffer.name, p.op.dst.buffer.name,
                           [(str(m), bound(m, rng)) for m, _ in src.region])
        small_pad = {}
        for p, _, plan in asyncs:
            if plan.get("small"):
                small_pad[p.op.dst.buffer] = plan["pad_elems"]
        # multi-version the shared buffers
        mapping = {}
        newbufs = {}
        versions = getattr(self, "versions", None)
        if versions is None:
            versions = self.versions = {}
        for p, _ in prods:
            B = p.op.dst.buffer
            if B in newbufs:
                continue
            # several pipelined loops over the same tile (e.g. an unmasked main loop and a masked
            # tail) share one multi-versioned LDS ring per stage count
            pad = small_pad.get(B)
            NB = versions.get((B, nstages, pad))
            if NB is None:
                shp = B.static_shape()
                NB = Buffer(B.name, [nstages] + shp, B.dtype, "shared")
                # small-tile DMA: every wave writes a 256-byte window of the slot (padding)
                NB.layout = stage_layout(B.layout, shp, nstages) if pad is None else \
                    _padded_stage_layout(shp, nstages, pad)
                NB._auto_name = False
                NB.stages_of = B
                versions[(B, nstages, pad)] = NB
            newbufs[B] = NB
        kk = binop("-", k, loop.min)
        stage = binop("%", kk, nstages)
        for B, NB in newbufs.items():
            mapping[B] = (NB, [stage])
        L_instr = sum(pl["instrs"] for _, _, pl in asyncs)

        gkeys = {}
        for p, _, plan in asyncs:
            if plan.get("gather"):
                self.key += 1
                gkeys[id(p)] = self.key

        def gather_idx(j):
            out = []
            for p, src, plan in asyncs:
                if id(p) in gkeys:
                    idxj = _subst_region(_subst_region(p.op.idx, lets), {k: binop("+", loop.min, j)})
                    out.append(S.TileOpStmt(GatherIndexOp(idxj, plan, gkeys[id(p)])))
            return out

        def issue_async(j, stg):
            out = []
            for p, src, plan in asyncs:
                srcj = _subst_region(src, {k: binop("+", loop.min, j)})
                NB = newbufs[p.op.dst.buffer]
                dst = BufferRegion(NB, [(stg, 1)] + list(p.op.dst.region))
                idxj = None
                if isinstance(p.op, O.GatherRowsOp):
                    idxj = _subst_region(_subst_region(p.op.idx, lets), {k: binop("+", loop.min, j)})
                out.append(S.TileOpStmt(AsyncCopyOp(srcj, dst, plan, idxj, gkeys.get(id(p)))))
            return out

        keys = {}

        def staged_phase(j, stg, phase):
            out = []
            for p, src in staged:
                if id(p) not in keys:
                    self.key += 1
                    keys[id(p)] = self.key
                srcj = _subst_region(src, {k: binop("+", loop.min, j)})
                NB = newbufs[p.op.dst.buffer]
                dst = BufferRegion(NB, [(stg, 1)] + list(p.op.dst.region))
                out.append(S.TileOpStmt(StagedCopyOp(srcj, dst, phase, keys[id(p)])))
            return out

        prologue = []
        nv = as_int(n)

        def guarded(j, st):
            if nv is not None:
                return S.seq(*st) if j < nv else None
            return S.IfStmt(binop("<", j, n), S.seq(*st))

        if gkeys:
            prologue.append(guarded(0, gather_idx(0)))
        for j in range(nstages - 1):
            st = issue_async(j, j)
            if not st:
                break
            if nv is not None and j >= nv:
                break
            prologue.append(S.seq(*st) if nv is not None else S.IfStmt(binop("<", j, n), S.seq(*st)))
            if gkeys:
                prologue.append(guarded(j + 1, gather_idx(j + 1)))
        prologue = [x for x in prologue if x is not None]
        if staged:
            st = staged_phase(0, 0, "load") + staged_phase(0, 0, "store")
            prologue.append(S.seq(*st) if nv is not None and nv > 0 else S.IfStmt(binop("<", 0, n), S.seq(*st)))

        consumer_stmts = [st for st in stmts if not any(st is p for p, _ in prods)]
        if loop.annotations.get("quad") and nstages == 2 and not staged:
            q = _quad_schedule(self, loop, asyncs, consumer_stmts, newbufs, rng)
            if q is None and any(pl.get("ktail") for _, _, pl in asyncs):
                # a k-tail plan only the quad template can run: the generic pipeline again, without
                # the relaxed plans (those copies are register-staged)
                ann = {kk_: v for kk_, v in loop.annotations.items() if kk_ != "quad"}
                return self.pipeline(S.ForStmt(loop.var, loop.min, loop.extent, loop.kind, loop.body, ann))
            if q is not None:
                return q
            _log.debug("quad GEMM loop %s: falling back to the generic pipeline", loop.var)
        if loop.annotations.get("phased") and nstages == 2 and not staged and len(asyncs) == 4 and \
                all(getattr(p.op, "khalf", None) is not None for p, _, _ in asyncs):
            ph = _phased_schedule(self, loop, asyncs, issue_async, consumer_stmts, mapping, newbufs, kk, n, lets)
            if ph is not None:
                return ph
        consumers = BufferReplacer(mapping).stmt(S.SeqStmt(consumer_stmts))
        body = []
        if asyncs:
            if nstages > 2:
                body.append(S.IfStmt(binop("<", binop("+", kk, nstages - 2), n),
                                     L.CallStmt("tl::wait_vmcnt", [], [L_instr * (nstages - 2)]),
                                     L.CallStmt("tl::wait_vmcnt", [], [0])))
            else:
                body.append(L.CallStmt("tl::wait_vmcnt", [], [0]))
        body.append(L.CallStmt("tl::barrier_raw", []))
        if staged:
            # register-staged loads go out BEFORE this iteration's LDS-DMAs: vmcnt retires in issue
            # order, so the wait the compiler puts in front of their LDS store can leave the DMAs
            # in flight (vmcnt(#DMAs)); issued after them it had to be vmcnt(0), which drained the
            # whole ring every iteration (the MX GEMM's scale tiles: 63 % of wave cycles waiting)
            j1 = binop("+", kk, 1)
            body.append(S.IfStmt(binop("<", j1, n), S.seq(*staged_phase(j1, binop("%", j1, nstages), "load"))))
        if asyncs:
            j = binop("+", kk, nstages - 1)
            body.append(S.IfStmt(binop("<", j, n), S.seq(*issue_async(j, binop("%", j, nstages)))))
            if gkeys:
                j2 = binop("+", kk, nstages)
                body.append(S.IfStmt(binop("<", j2, n), S.seq(*gather_idx(j2))))
        body.append(consumers)
        if staged:
            j1 = binop("+", kk, 1)
            body.append(S.IfStmt(binop("<", j1, n), S.seq(*staged_phase(j1, binop("%", j1, nstages), "store"))))
        ann_new = {"pipelined": nstages, "_lets": lets}
        uf = loop.annotations.get("unroll_factor") or getattr(self.target, "pipeline_unroll", None)
        if uf and int(uf) > 1:
            ann_new["unroll_factor"] = int(uf)
        new_loop = S.ForStmt(k, loop.min, loop.extent, "serial", S.SeqStmt(body), ann_new)
        # allocations for the new multi-versioned buffers replace the old ones (done by caller)
        self.replaced = getattr(self, "replaced", {})
        for B, NB in newbufs.items():
            lst = self.replaced.setdefault(B, [])
            if NB not in lst:
                lst.append(NB)
        tail = [L.CallStmt("tl::barrier_raw", [])]
        return S.SeqStmt(prologue + [new_loop] + tail)


def _phased_schedule(self, loop, asyncs, issue_async, consumer_stmts, mapping, newbufs, kk, n, lets=None):
    """K-half phased GEMM schedule (after ``gemm_ksplit``): two 2-deep LDS rings, one per K half.
    Iteration t reads stage s = t % 2:

        wait(k0(t)) barrier | issue k1(t+1) | gemm(k0 half of s)
        wait(k1(t)) barrier | issue k0(t+2) | gemm(k1 half of s)

    A K half is refilled as soon as every wave has passed the barrier behind its last read, and
    each wait is counted (two half-tiles stay in flight), never vmcnt(0) in steady state."""
    k = loop.var
    halves = {0: [], 1: []}
    for p, src, plan in asyncs:
        halves[p.op.khalf].append((p, src, plan))
    h = sum(pl["instrs"] for _, _, pl in halves[0])
    if h != sum(pl["instrs"] for _, _, pl in halves[1]):
        return None

    # row gathers (MoE token rows): their indices must not depend on the K step; they are loaded
    # into registers once before the loop, so the counted vmcnt waits see only the DMAs
    idx_pre, idx_key = [], {}
    for p, src, plan in asyncs:
        if isinstance(p.op, O.GatherRowsOp):
            idx = _subst_region(p.op.idx, lets or {})
            if any(v is k for m, e in idx.region for v in free_vars(m)):
                return None
            self.key += 1
            idx_key[id(p)] = (self.key, idx)
            idx_pre.append(S.TileOpStmt(GatherIndexOp(idx, plan, self.key)))

    def issue(half, j, stg):
        out = []
        for p, src, plan in halves[half]:
            srcj = _subst_region(src, {k: binop("+", loop.min, j)})
            NB = newbufs[p.op.dst.buffer]
            dst = BufferRegion(NB, [(stg, 1)] + list(p.op.dst.region))
            key, idxj = idx_key.get(id(p), (None, None))
            out.append(S.TileOpStmt(AsyncCopyOp(srcj, dst, plan, idxj, key)))
        return S.seq(*out)

    nv = as_int(n)
    gemms = [st for st in consumer_stmts if isinstance(st, S.TileOpStmt) and isinstance(st.op, O.GemmOp)]
    others = [st for st in consumer_stmts if st not in gemms]
    if len(gemms) != 2 or others:
        return None
    g0 = BufferReplacer(mapping).stmt(gemms[0])
    g1 = BufferReplacer(mapping).stmt(gemms[1])
    if getattr(gemms[0].op, "khalf", 0) == 1:
        g0, g1 = g1, g0

    if loop.annotations.get("phased") == "prio":
        g0 = S.seq(L.CallStmt("tl::setprio", [], [1]), g0, L.CallStmt("tl::setprio", [], [0]))
        g1 = S.seq(L.CallStmt("tl::setprio", [], [1]), g1, L.CallStmt("tl::setprio", [], [0]))

    def wait(more, n_more, n_last):
        return S.IfStmt(more, L.CallStmt("tl::wait_vmcnt", [], [n_more]), L.CallStmt("tl::wait_vmcnt", [], [n_last]))

    if loop.annotations.get("phased") is True and getattr(self.target, "gemm_prefetch", None) is not False and \
            all(_prefetchable(g.op, self.target) for g in gemms):
        return _prefetch_schedule(self, loop, gemms, newbufs, issue, wait, idx_pre, h, kk, n, nv)

    prologue = idx_pre + [issue(0, IntImm(0), IntImm(0)), issue(1, IntImm(0), IntImm(0))]
    if nv is None or nv > 1:
        prologue.append(S.IfStmt(binop("<", IntImm(1), n), issue(0, IntImm(1), IntImm(1))) if nv is None
                        else issue(0, IntImm(1), IntImm(1)))
    t1 = binop("+", kk, 1)
    t2 = binop("+", kk, 2)
    more = binop("<", t1, n)
    body = [wait(more, 2 * h, h), L.CallStmt("tl::barrier_raw", []),
            S.IfStmt(more, issue(1, t1, binop("%", t1, 2))), g0,
            wait(more, 2 * h, 0), L.CallStmt("tl::barrier_raw", []),
            S.IfStmt(binop("<", t2, n), issue(0, t2, binop("%", kk, 2))), g1]
    new_loop = S.ForStmt(k, loop.min, loop.extent, "serial", S.SeqStmt(body), {"pipelined": 2, "phased": True})
    self.replaced = getattr(self, "replaced", {})
    for B, NB in newbufs.items():
        lst = self.replaced.setdefault(B, [])
        if NB not in lst:
            lst.append(NB)
    return S.SeqStmt(prologue + [new_loop, L.CallStmt("tl::barrier_raw", [])])


def _k_coeff(e, k) -> Optional[int]:
    """Coefficient of ``k`` in ``e`` if ``e`` is affine in ``k`` (other terms free), else None."""
    from ..ir.expr import BinOp
    if not any(v is k for v in free_vars(e)):
        return 0
    if e is k:
        return 1
    if isinstance(e, BinOp) and e.op in ("+", "-"):
        ca, cb = _k_coeff(e.a, k), _k_coeff(e.b, k)
        if ca is None or cb is None:
            return None
        return ca + cb if e.op == "+" else ca - cb
    if isinstance(e, BinOp) and e.op == "*":
        if as_int(e.b) is not None:
            c = _k_coeff(e.a, k)
            return None if c is None else c * as_int(e.b)
        if as_int(e.a) is not None:
            c = _k_coeff(e.b, k)
            return None if c is None else c * as_int(e.a)
    return None


def _in_bounds(src: BufferRegion, ranges) -> bool:
    """Every dim of ``src`` provably inside its buffer over ``ranges``."""
    for d, (m, e) in enumerate(src.region):
        b, s, ev = bound(m, ranges), as_int(src.buffer.shape[d]), as_int(e)
        if b is None or s is None or ev is None or b[0] < 0 or b[1] + ev > s:
            return False
    return True


def _quad_schedule(self, loop, asyncs, consumer_stmts, newbufs, ranges):
    """The whole loop as ``tl::gemm_quad_nt_x`` (loops marked ``quad`` by gemm_ksplit.mark_quad_loops):
    the operand tiles' K start advances by exactly one 128-byte tile (64 fp16 / 128 fp8) per step
    along the contiguous dim, plain
    copies are provably in bounds (gathers are range-checked by the buffer resource), and the
    GEMM (+ the MoE extension GEMM) are the only consumers.  None: the generic pipeline runs it."""
    gemms = [st.op for st in consumer_stmts if isinstance(st, S.TileOpStmt) and isinstance(st.op, O.GemmOp)]
    if len(gemms) != len(consumer_stmts) or len(gemms) not in (1, 2):
        return None
    from .gemm_ksplit import quad_k
    g = [x for x in gemms if x.A.buffer.static_shape() == [256, quad_k(x.A.buffer.dtype)]]
    if len(g) != 1:
        return None
    g = g[0]
    ke = quad_k(g.A.buffer.dtype)
    x = next((o for o in gemms if o is not g), None)
    k = loop.var
    tiles = {}
    ktail = set()
    for p, src, plan in asyncs:
        gather = isinstance(p.op, O.GatherRowsOp)
        if not gather and (plan.get("gather") or plan.get("rdim") is None):
            return None
        rdim = p.op.row_dim if gather else plan["rdim"]
        cdim = len(src.region) - 1
        kt = plan.get("ktail") if not gather else None
        if kt is not None:
            ktail.add(kt)
        if not gather and not _in_bounds(src, ranges):
            # the outermost (row) dim and / or a ragged last K tile unproven: rows past the tensor
            # read zeros, as the generic pipeline's out-of-range LDS-DMA (the template's
            # range-checked row mode), and so do K chunks past the row end (ktail)
            reg = list(src.region)
            row_oob = not _in_bounds(BufferRegion(src.buffer, reg[:cdim] + [(IntImm(0), reg[cdim][1])
                                                                              if kt is not None else reg[cdim]]),
                                     ranges)
            if row_oob and rdim != 0:
                return None
            probe = [(IntImm(0), reg[0][1]) if row_oob else reg[0]] + reg[1:cdim] + \
                [(IntImm(0), reg[cdim][1]) if kt is not None else reg[cdim]]
            if not _in_bounds(BufferRegion(src.buffer, probe), ranges):
                return None
            gather = "rows" if row_oob else False
        if as_int(src.buffer.get_strides()[cdim]) != 1:
            return None
        for d, (m, _) in enumerate(src.region):
            if _k_coeff(m, k) != (ke if d == cdim else 0):
                return None
        idx = _subst_region(p.op.idx, {k: loop.min}) if gather is True else None
        if idx is not None and any(v is k for m, _ in idx.region for v in free_vars(m)):
            return None
        tiles[p.op.dst.buffer] = (_subst_region(src, {k: loop.min}), rdim, idx, gather)
    A, B = g.A.buffer, g.B.buffer
    want = {A, B} | ({x.A.buffer} if x is not None else set())
    if set(tiles) != want or tiles[B][3] not in (False, "rows"):
        return None
    if len(ktail) > 1 or (ktail and x is not None):
        return None  # A and B must share the ragged K (the MoE extension GEMM: aligned K only)
    k_len = next(iter(ktail)) if ktail else None
    if k_len is not None and any(tiles[Bf][3] is True for Bf in tiles):
        return None  # gathered rows: aligned K only
    b_rows = tiles[B][3] == "rows"
    a_src, a_rdim, idx, a_mode = tiles[A]
    if x is not None and tiles[x.A.buffer][3] != a_mode:
        return None
    for Bf, checked in ((A, a_mode or k_len is not None), (B, b_rows or k_len is not None)):
        if not checked:
            continue
        # gathered / range-checked rows or K chunks: tl::gemm_quad_nt_x forms the byte offsets and
        # the buffer resource's range in 32 bits (tl/gemm_quad.h), as the dense DMA plan's own
        # numel * eb < 2^31 condition; a larger tensor runs the generic pipeline
        numel = 1
        for s_ in tiles[Bf][0].buffer.shape:
            if as_int(s_) is None:
                return None
            numel *= as_int(s_)
        if numel * tiles[Bf][0].buffer.dtype.bytes >= (1 << 31):
            return None
    if a_mode and a_rdim != 0:
        return None
    op = QuadGemmLoopOp(a_src, a_rdim, idx, tiles[B][0], tiles[B][1], newbufs[A], newbufs[B],
                        newbufs[x.A.buffer] if x is not None else None, g.C, x.C if x is not None else None,
                        loop.extent, getattr(g, "valid_m", None), row_mode=a_mode == "rows", b_row_mode=b_rows,
                        k_len=k_len)
    self.replaced = getattr(self, "replaced", {})
    for Bf in want:
        lst = self.replaced.setdefault(Bf, [])
        if newbufs[Bf] not in lst:
            lst.append(newbufs[Bf])
    # the barrier ahead: earlier readers of the LDS the DMAs overwrite are done
    return S.SeqStmt([L.CallStmt("tl::barrier_raw", []), S.TileOpStmt(op), L.CallStmt("tl::barrier_raw", [])])


def _prefetchable(op, target) -> bool:
    """A K-half GEMM whose fragments can be read one phase ahead (``tl::gemm_ss_load`` /
    ``gemm_ss_mma``): 16-bit operands, both in LDS, the 16x16x32 MFMA, nothing else fused."""
    from ..ir import dtypes as _dt
    if not isinstance(op, O.GemmOp) or op.is_mx or op.is_sp:
        return False
    if op.clear_accum not in (False, None, 0):
        return False
    if (getattr(op, "mfma_shape", None) or getattr(target, "mfma_shape", None)) == "32x32":
        return False
    A, B = op.A.buffer, op.B.buffer
    return A.scope == "shared" and B.scope == "shared" and A.dtype == B.dtype and \
        A.dtype in (_dt.float16, _dt.bfloat16)


def _prefetch_schedule(self, loop, gemms, newbufs, issue, wait, idx_pre, h, kk, n, nv):
    """Register-prefetched K-half schedule.  Half-tiles go to two LDS banks (even K halves in
    bank 0, odd in bank 1), each two stages deep; the fragments of a half are read from LDS in
    the phase BEFORE its MFMAs, while the previous half's MFMAs run:

        prologue: issue tiles 0, 1;  wait(0a) barrier;  F0 <- frags(bank0[0])
        iteration t (s = t % 2):
          wait(t.b)   barrier | issue (t+2).a -> bank0[s] | F1 <- frags(bank1[s])   | mma(F0)
          wait(t+1.a) barrier | issue (t+2).b -> bank1[s] | F0 <- frags(bank0[s^1]) | mma(F1)

    A phase refills the slot of its own bank that the previous phase read and reads the other
    bank, so the ds_reads provably miss the LDS-DMA just issued (no compiler vmcnt(0)); every
    wait is counted (two half-tiles in flight across each barrier).  Measured on gfx950:
    fp16 4096^3 1057 -> 1225 TF (profiles/r3/gemm_prefetch_ab.log)."""
    from ..ir.expr import Var
    from ..ir import dtypes as _dt
    import copy
    k = loop.var
    self.key += 1
    f0, f1 = Var(f"tl_frag{self.key}_0", _dt.handle), Var(f"tl_frag{self.key}_1", _dt.handle)

    def at(g, stage, mode, var, mma_var=None):
        st = BufferReplacer({B: (NB, [stage]) for B, NB in newbufs.items()}).stmt(g)
        op = copy.copy(st.op)
        op.frag = (mode, var) if mma_var is None else (mode, var, mma_var)
        return S.TileOpStmt(op)

    g0, g1 = gemms
    if getattr(g0.op, "khalf", 0) == 1:
        g0, g1 = g1, g0
    zero, one = IntImm(0), IntImm(1)
    prologue = idx_pre + [issue(0, zero, zero), issue(1, zero, zero)]
    if nv is None or nv > 1:
        two = S.seq(issue(0, one, one), issue(1, one, one))
        prologue.append(S.IfStmt(binop("<", one, n), two) if nv is None else two)
    prologue += [at(g0, zero, "decl", f0), at(g0, zero, "decl", f1)]
    prologue.append(wait(binop("<", one, n), 3 * h, h))
    prologue += [L.CallStmt("tl::barrier_raw", []), at(g0, zero, "load", f0)]
    t1, t2 = binop("+", kk, 1), binop("+", kk, 2)
    more, more2 = binop("<", t1, n), binop("<", t2, n)
    s_, s1 = binop("%", kk, 2), binop("%", t1, 2)
    odd_wait = S.IfStmt(more2, L.CallStmt("tl::wait_vmcnt", [], [2 * h]), wait(more, h, 0))
    body = [wait(more, 2 * h, 0), L.CallStmt("tl::barrier_raw", []),
            S.IfStmt(more2, issue(0, t2, s_)), at(g1, s_, "load_mma", f1, f0),
            odd_wait, L.CallStmt("tl::barrier_raw", []),
            S.IfStmt(more2, issue(1, t2, s_)), at(g0, s1, "load_mma", f0, f1)]
    new_loop = S.ForStmt(k, loop.min, loop.extent, "serial", S.SeqStmt(body), {"pipelined": 2, "phased": True})
    self.replaced = getattr(self, "replaced", {})
    for B, NB in newbufs.items():
        lst = self.replaced.setdefault(B, [])
        if NB not in lst:
            lst.append(NB)
    return S.SeqStmt(prologue + [new_loop, L.CallStmt("tl::barrier_raw", [])])


def free_vars_stmt_outer(kernel):
    return list(kernel.block_vars) + list(kernel.thread_vars)


def _subst_region(r: BufferRegion, vmap) -> BufferRegion:
    return BufferRegion(r.buffer, [(substitute(m, vmap), substitute(e, vmap) if isinstance(e, PrimExpr) else e)
                                   for m, e in r.region])


class _AllocReplacer(Mutator):

    def __init__(self, replaced):
        self.replaced = replaced

    def visit_AllocStmt(self, s):
        if s.buffer in self.replaced:
            nbs = self.replaced[s.buffer]
            keep = [s] if s.buffer in getattr(self, "still_used", ()) else []
            return S.seq(*(keep + [S.AllocStmt(nb) for nb in nbs]))
        return s


def _referenced_buffers(stmt) -> set:
    """Buffers a (pre-lowering) statement reads or writes: tile-op regions, loads, stores."""
    from ..ir.expr import post_order, BufferLoad
    out = set()
    for x in S.walk(stmt):
        exprs = []
        if isinstance(x, S.TileOpStmt):
            for r in x.op.regions():
                if hasattr(r, "buffer"):
                    out.add(r.buffer)
        elif isinstance(x, S.StoreStmt):
            out.add(x.buffer)
            exprs = [x.value] + list(x.indices)
        elif isinstance(x, S.LetStmt):
            exprs = [x.value]
        elif isinstance(x, S.EvaluateStmt):
            exprs = [x.expr]
        elif isinstance(x, (S.IfStmt, S.WhileStmt)):
            exprs = [x.cond]
        for e in exprs:
            if hasattr(e, "dtype"):
                for n in post_order(e):
                    if isinstance(n, BufferLoad):
                        out.add(n.buffer)
    return out


def inject_software_pipeline(kernel: S.KernelStmt, num_threads: int, target) -> S.KernelStmt:
    pi = PipelineInjector(kernel, num_threads, target)
    new = pi.stmt(kernel)
    replaced = getattr(pi, "replaced", {})
    if replaced:
        ar = _AllocReplacer(replaced)
        # a tile also used outside the pipelined loops (e.g. a stream-K partial loop next to a
        # pipelined data-parallel loop) keeps its single-buffer allocation as well
        used = _referenced_buffers(new)
        ar.still_used = {b for b in replaced if b in used}
        new = ar.stmt(new)
    return new
