"""Lower tile operators and ``T.Parallel`` nests into per-thread (SIMT) code.

Reference: ``src/transform/lower_tile_op.cc`` (calls each op's ``Lower``),
``src/op/parallel.cc`` + ``loop_partition.cc`` + ``loop_vectorize.cc`` (partition
a parallel nest over threads using the fragment layout and vectorise it),
``src/op/copy.cc`` (SIMT copy), ``src/op/reduce.cc`` (thread-local reduce +
``tl::AllReduce``), ``src/op/fill.cc``.

After this pass:
  * fragments are per-thread ``local`` arrays indexed by compile-time register numbers
    (register index of logical element = Fragment.forward_index, proven uniform over
    the block's threads by enumeration — so nothing is indexed at run time and the
    arrays stay in VGPRs/AGPRs);
  * every buffer access is flat (global: strides applied; shared: swizzled physical
    offset inside the buffer's LDS slot);
  * contiguous accesses are vectorised up to 16 B per lane.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir import lowered as L
from ..ir import dtypes as _dt
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import (BinOp, BufferLoad, Call, IntImm, PrimExpr, Var, as_int, binop, call, cast, compile_py, const,
                       convert, divisible_by, free_vars, logical_and, logical_not, select, substitute, transform,
                       post_order, modular)
from ..layout.fragment import Digit, Fragment
from ..layout.layout import LinearLayout, SwizzleLayout
from .layout_inference import ParallelNest
from .pipeline import AsyncCopyOp, GatherIndexOp, StagedCopyOp
from .utils import Mutator, Substituter, bound
from . import gemm_lower


class LoweringError(Exception):
    pass


_REDUCE_OPS = {
    "sum": ("tl::SumOp", "+"),
    "abssum": ("tl::SumOp", "+"),
    "max": ("tl::MaxOp", "max"),
    "absmax": ("tl::MaxOp", "max"),
    "min": ("tl::MinOp", "min"),
    "bitand": ("tl::BitAndOp", "&"),
    "bitor": ("tl::BitOrOp", "|"),
    "bitxor": ("tl::BitXorOp", "^"),
}


def _reduce_init(kind, dtype):
    if kind in ("sum", "abssum", "bitor", "bitxor"):
        return const(0, dtype)
    if kind in ("max", "absmax"):
        return const(-float("inf") if dtype.is_float else _dt.min_value(dtype), dtype) if kind == "max" \
            else const(0, dtype)
    if kind == "min":
        return const(float("inf") if dtype.is_float else _dt.max_value(dtype), dtype)
    if kind == "bitand":
        return const(-1, dtype)
    raise ValueError(kind)


def _combine(kind, a, b):
    if kind in ("sum", "abssum"):
        return a + b
    if kind in ("max", "absmax"):
        return binop("max", a, b)
    if kind == "min":
        return binop("min", a, b)
    if kind == "bitand":
        return a & b
    if kind == "bitor":
        return a | b
    if kind == "bitxor":
        return a ^ b
    raise ValueError(kind)


def _tree_combine(kind, xs):
    """Balanced reduction tree: log-depth dependency chains (ILP) and shallow expressions.
    max / min trees are ternary, max(max(a, b), c) per node, which the backend emits as one
    v_max3 / v_min3: (n-1)/2 instructions instead of n-1 on the VALU (FA's row max)."""
    xs = list(xs)
    if kind in ("max", "absmax", "min"):
        while len(xs) > 1:
            nxt = []
            i = 0
            while i < len(xs):
                grp = xs[i:i + 3]
                acc = grp[0]
                for g in grp[1:]:
                    acc = _combine(kind, acc, g)
                nxt.append(acc)
                i += 3
            xs = nxt
        return xs[0]
    while len(xs) > 1:
        nxt = [_combine(kind, xs[i], xs[i + 1]) for i in range(0, len(xs) - 1, 2)]
        if len(xs) % 2:
            nxt.append(xs[-1])
        xs = nxt
    return xs[0]


def _prod(xs):
    n = 1
    for x in xs:
        n *= x
    return n


class LowerCtx:

    def __init__(self, kernel: S.KernelStmt, target, pass_cfg=None):
        self.kernel = kernel
        self.T = kernel.num_threads
        self.target = target
        self.is_cpu = kernel.is_cpu or getattr(target, "kind", "hip") == "cpu"
        self.tid = Var("tid")
        self.tid.nonneg = True
        self.lane = Var("lane")
        self.wave = Var("wave")
        self.frag_local: Dict[Buffer, Buffer] = {}
        self.flat: Dict[Buffer, Buffer] = {}
        self.extra_allocs: List[Buffer] = []
        self.staging: Dict[int, Buffer] = {}
        self.pass_cfg = pass_cfg or {}
        self.narrow_index = set()  # global buffers addressed with 32-bit offsets
        self.no_vectorize = bool(self.pass_cfg.get("tir.disable_vectorize", False))
        # tl.dynamic_alignment: dynamic extents are multiples of this (enables vector accesses)
        self.dynamic_alignment = int(self.pass_cfg.get("tl.dynamic_alignment", 0) or 0)
        self.uses_grid_sync = False
        self.thread_range = None  # (lo, hi): inside ``if lo <= tx < hi`` (thread-range partitioning)
        # ThreadSync is off (tl.disable_thread_storage_sync): the workspace exchanges this pass
        # emits carry their own leading / trailing barriers instead of relying on it
        self.self_sync = bool(self.pass_cfg.get("tl.disable_thread_storage_sync", False))
        self.dynamic_vars = set()
        if self.dynamic_alignment > 1:
            from .pipeline import _referenced_buffers
            for b in _referenced_buffers(kernel):
                for d in b.shape:
                    if isinstance(d, Var):
                        self.dynamic_vars.add(d)
        self.known_div: Dict[Var, tuple] = {}
        self.ranges = {}
        for v, g in zip(kernel.block_vars, kernel.grid):
            gv = as_int(g)
            if gv is not None:
                self.ranges[v] = (0, gv - 1)
        self.ranges[self.tid] = (0, self.T - 1)
        self.uses_lane = False
        self.uses_wave = False
        self.ws_counter = 0

    # -- buffers ---------------------------------------------------------------------
    def flat_of(self, b: Buffer) -> Buffer:
        if b.scope == "fragment":
            return self.local_of(b)
        fb = self.flat.get(b)
        if fb is None:
            if b.alias_of is not None:
                base = self.flat_of(b.alias_of[0])
                if b.dtype != base.dtype:
                    # T.view(..., dtype=): the same bytes read as another type
                    if base.scope != "global":
                        raise LoweringError(f"T.view({b.alias_of[0].name}, dtype={b.dtype.name}): a dtype view of a "
                                            f"{base.scope} buffer is not supported; view the global tensor")
                    fb = Buffer(b.name, [b.numel()], b.dtype, base.scope)
                    fb.reinterpret = base
                    fb.param_index = base.param_index
                    fb._auto_name = False
                    self.flat[b] = fb
                    return fb
                self.flat[b] = base
                return base
            size = None
            if b.scope == "shared":
                from ..layout.layout import physical_size
                size = physical_size(b.layout, b.shape)
            fb = Buffer(b.name, [size] if size is not None else [b.numel()], b.dtype, b.scope)
            fb.orig = b
            fb.param_index = b.param_index
            fb.nontemporal = getattr(b, "nontemporal", False)
            fb._auto_name = False
            self.flat[b] = fb
        return fb

    def local_of(self, b: Buffer) -> Buffer:
        lb = self.frag_local.get(b)
        a = getattr(b, "alias_of", None)
        if lb is None and a is not None and a[0].scope == "fragment":
            if a[0].dtype != b.dtype:
                raise LoweringError(f"T.view of fragment {a[0].name} with another dtype is not supported")
            lb = self.local_of(a[0])  # a reshaped view shares the base's registers
            self.frag_local[b] = lb
            return lb
        if lb is None:
            lay = b.layout
            if not isinstance(lay, Fragment):
                raise LoweringError(f"fragment {b.name} has no inferred layout")
            lb = Buffer(b.name, [lay.local_size], b.dtype, "local")
            lb.orig = b
            lb._auto_name = False
            self.frag_local[b] = lb
        return lb

    def legal_index(self, b: Buffer, indices):
        """LegalizeNegativeIndex (reference ``src/transform/legalize_negative_index.cc``): an
        index that is provably negative counts from the end of its dimension (``A[-i - 1]`` for
        ``i`` in [0, 4) is ``A[n - 1 - i]``); an index of unknown sign is left alone."""
        out = []
        for i, s in zip(indices, b.shape):
            bd = bound(i, self.ranges)
            out.append(binop("+", i, s) if bd is not None and bd[1] < 0 else i)
        return out

    def flat_index(self, b: Buffer, indices) -> PrimExpr:
        indices = self.legal_index(b, indices)
        if b.scope == "shared":
            lay = b.layout
            if lay is None:
                return b.offset_of(indices)
            return convert(lay.offset(*indices))
        if b.scope in ("local", "var"):
            return b.offset_of(indices)
        if b.scope == "global":
            return b.offset_of(indices, wide=self.wide_index(b))
        raise LoweringError(f"cannot flatten access to {b.scope} buffer {b.name}")

    def wide_index(self, b: Buffer) -> bool:
        """int64 offsets for a global buffer: ``tl.config_index_bitwidth`` (32/64) decides; by
        default a statically sized tensor of >= 2^31 elements gets int64, everything else int32
        and the launcher refuses tensors that would overflow it (``narrow_index`` params)."""
        bits = int(self.pass_cfg.get("tl.config_index_bitwidth", 0) or 0)
        if bits == 64:
            return True
        n = b.static_numel()
        if bits != 32 and n is not None and n >= (1 << 31):
            return True
        if bits != 32 and any(isinstance(d, PrimExpr) and d.dtype.is_int and d.dtype.bits >= 64 for d in b.shape):
            return True  # an int64 symbolic extent (T.symbolic("n", "int64")): sized past 2^31
        if bits == 32 and n is not None and n >= (1 << 31):
            raise LoweringError(f"{b.name} has {n} elements but tl.config_index_bitwidth=32")
        self.narrow_index.add(b)
        return False

    def lane_expr(self):
        self.uses_lane = True
        return self.lane

    def wave_expr(self):
        self.uses_wave = True
        return self.wave

    def new_local(self, name, n, dtype) -> Buffer:
        b = Buffer(name, [n], dtype, "local")
        b._auto_name = False
        self.extra_allocs.append(b)
        return b

    def new_workspace(self, n, dtype) -> Buffer:
        self.ws_counter += 1
        b = Buffer(f"red_ws{self.ws_counter}", [n], dtype, "shared")
        b.layout = LinearLayout([n])
        b._auto_name = False
        self.flat[b] = b  # already flat: accesses and the allocation are the same buffer
        self.extra_allocs.append(b)
        return b


# ---------------------------------------------------------------------------
# per-element fragment resolution
# ---------------------------------------------------------------------------


def _affine(e, vars_: List[Var]):
    """``e`` as (coefficients over ``vars_``, constant) when it is an integer affine form of them."""
    v = as_int(e)
    if v is not None:
        return [0] * len(vars_), v
    if isinstance(e, Var):
        for i, x in enumerate(vars_):
            if x is e:
                c = [0] * len(vars_)
                c[i] = 1
                return c, 0
        return None
    if isinstance(e, BinOp) and e.op in ("+", "-", "*"):
        a, b = _affine(e.a, vars_), _affine(e.b, vars_)
        if a is None or b is None:
            return None
        if e.op == "+":
            return [x + y for x, y in zip(a[0], b[0])], a[1] + b[1]
        if e.op == "-":
            return [x - y for x, y in zip(a[0], b[0])], a[1] - b[1]
        if not any(a[0]):
            return [a[1] * y for y in b[0]], a[1] * b[1]
        if not any(b[0]):
            return [b[1] * x for x in a[0]], a[1] * b[1]
        return None
    return None


class _FragResolver:
    """Resolves ``frag[idx(loop vars)]`` to a constant register index for iteration r of a
    loop partitioned by ``loop_layout`` (checked for every thread of the block)."""

    def __init__(self, ctx: LowerCtx, loop_vars: List[Var], loop_mins: List[PrimExpr], loop_layout: Fragment):
        self.ctx = ctx
        self.vars = loop_vars
        self.mins = [as_int(m) or 0 for m in loop_mins]
        self.layout = loop_layout
        self.cache = {}
        # loop-var values per (thread, r)
        T = loop_layout.num_threads
        self.T = T

    def local_index(self, buf: Buffer, idx_exprs: List[PrimExpr], r: int) -> int:
        key = (id(buf), tuple(id(e) for e in idx_exprs), r)
        if key in self.cache:
            return self.cache[key]
        blay: Fragment = buf.layout
        aff = [_affine(e, self.vars) for e in idx_exprs]
        if all(a is not None for a in aff) and blay.num_threads == self.T:
            # native proof over every lane of the block (tilelang._tl_core.Fragment.resolve_affine)
            A = [c for a in aff for c in a[0]]
            b = [a[1] + sum(c * m for c, m in zip(a[0], self.mins)) for a in aff]
            li = self.layout.native.resolve_affine(blay.native, A, b, r)
            if li == -1:
                raise LoweringError(
                    f"layout conflict: a thread iterates an element of fragment {buf.name} it does not own "
                    f"(loop layout {self.layout}, buffer layout {blay})")
            if li == -2:
                raise LoweringError(f"fragment {buf.name}: register index of element differs across threads "
                                    f"(non-uniform access {idx_exprs})")
            self.cache[key] = li
            return li
        try:
            fns = [compile_py(e, self.vars) for e in idx_exprs]
        except Exception as ex:  # noqa: BLE001
            raise LoweringError(f"fragment {buf.name} indexed by {idx_exprs}: indices must depend only on the "
                                f"T.Parallel loop variables ({ex})") from None
        result = None
        tl_cache = getattr(blay, "_tlmap", None)
        if tl_cache is None:
            tl_cache = {}
            blay._tlmap = tl_cache
        for t in range(self.T):
            vals = self.layout.inverse(t, r)
            vals = [v + m for v, m in zip(vals, self.mins)]
            bidx = tuple(int(f(*vals)) for f in fns)
            m = tl_cache.get(t)
            if m is None:
                m = blay.thread_local_map(t)
                tl_cache[t] = m
            li = m.get(bidx)
            if li is None:
                raise LoweringError(
                    f"layout conflict: thread {t} iterates element {bidx} of fragment {buf.name} it does not own "
                    f"(loop layout {self.layout}, buffer layout {blay})")
            if result is None:
                result = li
            elif result != li:
                raise LoweringError(f"fragment {buf.name}: register index of element differs across threads "
                                    f"(non-uniform access {idx_exprs})")
        self.cache[key] = result
        return result


def _fold_guard(c):
    """True / False when a guard condition is decided regardless of the thread, else None."""
    from ..ir.expr import modular
    v = as_int(c)
    if v is not None:
        return bool(v)
    if isinstance(c, BinOp) and c.op in ("<", "<=", ">", ">=", "==", "!=") and as_int(c.b) is not None:
        a = c.a
        if isinstance(a, BinOp) and a.op == "%" and as_int(a.b) is not None:
            m = as_int(a.b)
            coeff, base = modular(a.a)
            if coeff % m == 0:  # a.a == base (mod m) for every thread
                lhs = base % m
                rhs = as_int(c.b)
                return {"<": lhs < rhs, "<=": lhs <= rhs, ">": lhs > rhs, ">=": lhs >= rhs, "==": lhs == rhs,
                        "!=": lhs != rhs}[c.op]
    return None


class _IterRewriter(Mutator):
    """Rewrite one iteration (register r) of a fragment-partitioned nest."""

    def __init__(self, ctx: LowerCtx, resolver: _FragResolver, r: int, vmap):
        self.ctx = ctx
        self.res = resolver
        self.r = r
        self.vmap = vmap
        self.sub = Substituter(vmap)

    def _load(self, n):
        if isinstance(n, BufferLoad):
            return self._access(n.buffer, n.indices)
        return None

    def _access(self, b: Buffer, idx):
        if b.scope == "fragment":
            li = self.res.local_index(b, idx, self.r)
            return BufferLoad(self.ctx.local_of(b), [IntImm(li)])
        idx2 = [substitute(i, self.vmap) for i in idx]
        idx2 = [transform(i, self._load_sub) for i in idx2]
        if b.scope in ("local", "var"):
            return BufferLoad(b, [b.offset_of(idx2)] if b.ndim != 1 else idx2)
        ld = BufferLoad(self.ctx.flat_of(b), [self.ctx.flat_index(b, idx2)])
        g = safe_guard(self.ctx, b, idx2)
        if g is not None:
            return select(g, ld, _safe_value(b))
        return ld

    def _load_sub(self, n):
        return None

    def visit_IfStmt(self, s):
        # a guard that is decided by the register index alone (e.g. ``j % 4 < 2`` where the 4
        # columns of a lane are its registers) folds away per iteration, so an access it protects
        # (``C[i, j + 2]``, owned by this thread only when the guard holds) is never lowered
        # for the registers where it does not hold
        c = _fold_guard(substitute(s.cond, self.vmap))
        if c is False:
            return self.stmt(s.else_body) if s.else_body is not None else S.SeqStmt([])
        if c is True:
            return self.stmt(s.then_body)
        return S.IfStmt(self.expr(s.cond), self.stmt(s.then_body), self.stmt(s.else_body))

    def expr(self, e):
        if not isinstance(e, PrimExpr):
            return e

        def fn(n):
            if isinstance(n, BufferLoad):
                return self._access(n.buffer, n.indices)
            if isinstance(n, Call):
                return _hoist_atomic_guard(n)
            return None

        # fragments must be resolved on the ORIGINAL (loop-var) indices, so transform first,
        # then substitute the loop vars in what is left.
        e2 = transform(e, fn)
        return substitute(e2, self.vmap)

    def store(self, s: S.StoreStmt):
        val = self.expr(s.value)
        b = s.buffer
        if b.scope == "fragment":
            li = self.res.local_index(b, s.indices, self.r)
            return S.StoreStmt(self.ctx.local_of(b), [IntImm(li)], val)
        idx = [self.expr(i) for i in s.indices]
        if b.scope in ("local", "var"):
            return S.StoreStmt(b, [b.offset_of(idx)] if b.ndim != 1 else idx, val)
        st = S.StoreStmt(self.ctx.flat_of(b), [self.ctx.flat_index(b, idx)], val)
        g = safe_guard(self.ctx, b, idx)
        return S.IfStmt(g, st) if g is not None else st

    def visit_LetStmt(self, s):
        return S.LetStmt(s.var, self.expr(s.value))

    def visit_EvaluateStmt(self, s):
        r = _rewrite_atomic(self, s)
        return r if r is not None else S.EvaluateStmt(self.expr(s.expr))

    def visit_ForStmt(self, s):
        return S.ForStmt(s.var, self.expr(s.min), self.expr(s.extent), s.kind, self.stmt(s.body), s.annotations)


# ---------------------------------------------------------------------------
# vectorisation of a group of per-element statements
# ---------------------------------------------------------------------------


def _const_diff(a: PrimExpr, b: PrimExpr, probe_vars: List[Var]) -> Optional[int]:
    """a - b if it is the same constant for sampled values of probe_vars (else None)."""
    d = binop("-", a, b)
    v = as_int(d)
    if v is not None:
        return v
    try:
        fv = free_vars(d)
        f = compile_py(d, fv)
    except Exception:  # noqa: BLE001
        return None
    import random
    rnd = random.Random(7)
    vals = None
    for _ in range(6):
        args = [rnd.randrange(0, 4096) for _ in fv]
        try:
            x = f(*args)
        except Exception:  # noqa: BLE001
            return None
        if vals is None:
            vals = x
        elif x != vals:
            return None
    return int(vals) if vals is not None else None


def _safe_value(b: Buffer) -> PrimExpr:
    """What an out-of-bounds guarded load reads: ``T.annotate_safe_value`` or 0."""
    v = getattr(b, "safe_value", None)
    return cast(v, b.dtype) if v is not None else const(0, b.dtype)


def safe_guard(ctx: LowerCtx, b: Buffer, idx) -> Optional[PrimExpr]:
    """Bounds condition for a global access that cannot be proven in range (ragged tiles,
    dynamic shapes); None when every index is provably inside the tensor."""
    if b.scope != "global" or ctx.pass_cfg.get("tl.disable_safe_memory_legalize") or getattr(b, "no_guard", False):
        return None
    idx = ctx.legal_index(b, idx)
    if ctx.wide_index(b):
        from ..ir.expr import widen_int64
        idx = [widen_int64(i) for i in idx]
    cond = None
    for i, s in zip(idx, b.shape):
        bd = bound(i, ctx.ranges)
        sv = as_int(s)
        if bd is not None and sv is not None and bd[0] >= 0 and bd[1] < sv:
            continue
        if bd is not None and bd[0] < 0:
            # can go below the tensor (a shifted window, ``A[i - 10]``): guard the low side too
            c = binop(">=", i, 0)
            cond = c if cond is None else logical_and(cond, c)
        if bd is not None and sv is not None and bd[1] < sv:
            continue
        c = binop("<", i, s)
        if as_int(c) == 1:
            continue
        cond = c if cond is None else logical_and(cond, c)
    return cond


def _guard_conds(e, target) -> Optional[List[PrimExpr]]:
    """Conditions under which ``target`` (a node of ``e``, by identity) is evaluated: the
    conditions of the selects / short-circuit operators on its path.  None if not found."""
    from ..ir.expr import Select, UnOp as _Un
    if e is target:
        return []
    if isinstance(e, Select):
        r = _guard_conds(e.cond, target)
        if r is not None:
            return r
        r = _guard_conds(e.t, target)
        if r is not None:
            return [e.cond] + r
        r = _guard_conds(e.f, target)
        return None if r is None else [logical_not(e.cond)] + r
    if isinstance(e, BinOp) and e.op in ("&&", "||"):
        r = _guard_conds(e.a, target)
        if r is not None:
            return r
        r = _guard_conds(e.b, target)
        return None if r is None else [e.a if e.op == "&&" else logical_not(e.a)] + r
    from ..ir.expr import children
    for c in children(e):
        r = _guard_conds(c, target)
        if r is not None:
            return r
    return None


def vectorize_group(ctx: LowerCtx, stmts: List[S.Stmt], known_div) -> Optional[List[S.Stmt]]:
    """``stmts[i]`` are the per-element copies (i = 0..W-1) of a single-store body.  If the
    stores (and the loads feeding them) are contiguous and aligned, emit vector accesses."""
    W = len(stmts)
    from ..ir.expr import structural_equal
    if W > 1 and all(isinstance(s, S.IfStmt) and s.else_body is None for s in stmts):
        c0 = stmts[0].cond
        if all(structural_equal(s.cond, c0) for s in stmts):
            inner = vectorize_group(ctx, [s.then_body for s in stmts], known_div)
            return [S.IfStmt(c0, S.SeqStmt(inner))] if inner is not None else None
        # per-element bounds guards (dynamic tails): the vector body runs when every element is
        # in range, the guarded scalar copies otherwise
        inner = vectorize_group(ctx, [s.then_body for s in stmts], known_div)
        if inner is None:
            return None
        pred = None
        for st in stmts:
            pred = st.cond if pred is None else logical_and(pred, st.cond)
        return [S.IfStmt(pred, S.SeqStmt(inner), S.SeqStmt(list(stmts)))]
    if W == 1 or not all(isinstance(s, S.StoreStmt) for s in stmts):
        return None
    b = stmts[0].buffer
    if any(s.buffer is not b for s in stmts):
        return None
    eb = b.dtype.bytes
    if W * eb > 16 or (W * eb) not in (2, 4, 8, 16):
        return None
    base = stmts[0].indices[0]
    probe = []
    for i, s in enumerate(stmts):
        d = _const_diff(s.indices[0], base, probe)
        if d != i:
            return None
    if b.scope != "local" and not divisible_by(base, W, known_div):
        return None
    # vectorise the loads feeding the stores: the i-th load (in post-order) of every group
    # member is the same access shifted by i elements when the body is contiguous
    vals = [s.value for s in stmts]
    pre = []
    po = [[n for n in post_order(v) if isinstance(n, BufferLoad)] for v in vals]
    if all(len(p) == len(po[0]) for p in po):
        if len(po[0]) == 1 and vals[0] is po[0][0] and po[0][0].buffer.dtype == b.dtype and \
                po[0][0].buffer.scope in ("global", "shared") and b.scope != "local":
            ld0 = po[0][0]
            if all(_const_diff(po[i][0].indices[0], ld0.indices[0], []) == i for i in range(W)) and \
                    divisible_by(ld0.indices[0], W, known_div):
                return [L.CopyBytesStmt(b, base, ld0.buffer, ld0.indices[0], W * eb)]
        repl = [dict() for _ in range(W)]
        for j, ld0 in enumerate(po[0]):
            if ld0.buffer.scope not in ("global", "shared"):
                continue
            leb = ld0.buffer.dtype.bytes
            if W * leb not in (2, 4, 8, 16):
                continue
            if not all(po[i][j].buffer is ld0.buffer and
                       _const_diff(po[i][j].indices[0], ld0.indices[0], []) == i for i in range(W)):
                continue
            if not divisible_by(ld0.indices[0], W, known_div):
                continue
            tmp = ctx.new_local(f"vtmp{len(ctx.extra_allocs)}", W, ld0.buffer.dtype)
            guards = [_guard_conds(vals[i], po[i][j]) for i in range(W)]
            if any(g is None for g in guards):
                continue
            vload = L.VecLoadStmt(tmp, 0, ld0.buffer, ld0.indices[0], W)
            # an LDS read needs no guard: gfx950 bounds-checks DS addresses against the workgroup's
            # allocation (out-of-range reads return 0, never fault), and a select then discards
            # the value -- guarding it turned a masked T.Parallel into per-element exec-mask
            # branches (SALU-bound; the Mamba chunk scan's causal CB mask, profiles/r4).  The CPU
            # target keeps the guard: a host array read out of range can fault.
            if any(guards) and (ld0.buffer.scope != "shared" or ctx.is_cpu):
                # the element loads sit under bounds guards (selects): the vector load may only
                # run when every lane's guard holds, otherwise fall back to guarded scalar loads
                pred = None
                for g in guards:
                    for c in g:
                        pred = c if pred is None else logical_and(pred, c)
                slow = []
                for i in range(W):
                    st = S.StoreStmt(tmp, [IntImm(i)], po[i][j])
                    gc = None
                    for c in guards[i]:
                        gc = c if gc is None else logical_and(gc, c)
                    slow.append(st if gc is None else S.IfStmt(gc, st))
                vload = S.IfStmt(pred, vload, S.SeqStmt(slow))
            pre.append(vload)
            for i in range(W):
                repl[i][id(po[i][j])] = BufferLoad(tmp, [IntImm(i)])
        if pre:
            vals = [transform(v, lambda n, r=repl[i]: r.get(id(n))) for i, v in enumerate(vals)]
    if b.scope == "local":
        # stores into a register array need no vector op
        return pre + [S.StoreStmt(b, [s.indices[0]], v) for s, v in zip(stmts, vals)] if pre else None
    return pre + [L.VecStoreStmt(b, base, vals)]


def _atomic_add_call(s) -> Optional[Call]:
    """The ``tl.atomic_add(dst[i], v)`` call of an atomic-add statement (no returned value)."""
    if isinstance(s, S.EvaluateStmt) and isinstance(s.expr, Call) and s.expr.op == "tl.atomic_add" and \
            len(s.expr.args) == 2 and isinstance(s.expr.args[0], BufferLoad) and not s.expr.attrs.get("return_prev"):
        return s.expr
    return None


def vectorize_atomic_group(ctx: LowerCtx, stmts: List[S.Stmt], known_div) -> Optional[List[S.Stmt]]:
    """AtomicAddVectorize (reference ``src/transform/atomicadd_vectorize.cc``), gfx950 form:
    ``stmts[i]`` are the per-element atomic adds of one thread (i = 0..W-1).  When they hit
    consecutive f16 / bf16 elements whose first element is pair-aligned, pairs become one
    ``tl.atomic_addx2`` (``global_atomic_pk_add_{f16,bf16}`` / ``ds_pk_add_*``).  f32 has no vector
    atomic on gfx950: those groups stay scalar (``global_atomic_add_f32`` each)."""
    W = len(stmts)
    if W < 2:
        return None
    from ..ir.expr import structural_equal
    if all(isinstance(s, S.IfStmt) and s.else_body is None for s in stmts):
        c0 = stmts[0].cond
        if not all(structural_equal(s.cond, c0) for s in stmts):
            return None
        inner = vectorize_atomic_group(ctx, [s.then_body for s in stmts], known_div)
        return [S.IfStmt(c0, S.SeqStmt(inner))] if inner is not None else None
    calls = [_atomic_add_call(s) for s in stmts]
    if any(c is None for c in calls):
        return None
    b = calls[0].args[0].buffer
    if b.dtype.name not in ("float16", "bfloat16") or b.scope not in ("global", "shared") or \
            any(c.args[0].buffer is not b or len(c.args[0].indices) != 1 for c in calls):
        return None
    base = calls[0].args[0].indices[0]
    for i, c in enumerate(calls):
        if _const_diff(c.args[0].indices[0], base, []) != i:
            return None
    if not divisible_by(base, 2, known_div):
        return None
    out = []
    for i in range(0, W - 1, 2):
        c0, c1 = calls[i], calls[i + 1]
        out.append(S.EvaluateStmt(Call("tl.atomic_addx2", [c0.args[0], c0.args[1], c1.args[1]], c0.dtype,
                                       dict(c0.attrs))))
    if W % 2:
        out.append(stmts[-1])
    return out


def _is_cast_of(v, ld):
    from ..ir.expr import Cast
    return isinstance(v, Cast) and v.value is ld


# ---------------------------------------------------------------------------
# the pass
# ---------------------------------------------------------------------------


class TileOpLowerer(Mutator):

    def __init__(self, ctx: LowerCtx):
        self.ctx = ctx
        self.known_div = {}
        if ctx.dynamic_alignment > 1:
            for v in ctx.dynamic_vars:
                self.known_div[v] = (ctx.dynamic_alignment, 0)

    # -- helpers -------------------------------------------------------------------
    def flat_access_expr(self, e):
        """Flatten non-fragment buffer loads inside a scalar expression (outside nests)."""
        ctx = self.ctx

        def fn(n):
            if isinstance(n, BufferLoad):
                b = n.buffer
                if b.scope == "fragment":
                    lay = b.layout
                    if isinstance(lay, Fragment) and lay.local_size == _prod(b.static_shape() or [0]) and \
                            lay.replicate_size == lay.num_threads:
                        return BufferLoad(ctx.local_of(b), [b.offset_of(n.indices)])
                    raise LoweringError(f"fragment {b.name} accessed outside T.Parallel; use a T.Parallel loop or "
                                        f"T.alloc_local for per-thread arrays")
                if b.scope in ("local", "var") and b.alias_of is None:
                    return BufferLoad(b, [b.offset_of(n.indices)] if b.ndim != 1 else n.indices)
                return BufferLoad(ctx.flat_of(b), [ctx.flat_index(b, n.indices)])
            return None

        return transform(e, fn)

    def expr(self, e):
        if isinstance(e, PrimExpr):
            return self.flat_access_expr(e)
        return e

    def store(self, s):
        b = s.buffer
        val = self.expr(s.value)
        idx = [self.expr(i) for i in s.indices]
        if b.scope == "fragment":
            lay = b.layout
            if isinstance(lay, Fragment) and lay.replicate_size == lay.num_threads:
                return S.StoreStmt(self.ctx.local_of(b), [b.offset_of(idx)], val)
            raise LoweringError(f"store to fragment {b.name} outside T.Parallel")
        if b.scope in ("local", "var"):
            return S.StoreStmt(b, [b.offset_of(idx)] if b.ndim != 1 else idx, val)
        return S.StoreStmt(self.ctx.flat_of(b), [self.ctx.flat_index(b, idx)], val)

    def visit_EvaluateStmt(self, s):
        e = s.expr
        if isinstance(e, Call) and e.op == "tl.print_buffer":
            return self._lower_print_buffer(e)
        if isinstance(e, Call) and e.op == "tl.print":
            msg, v = e.args[0], self.expr(e.args[1])
            return L.CallStmt("tl::print_val", [msg, v])
        if isinstance(e, Call) and e.op == "tl.sync_grid":
            self.ctx.uses_grid_sync = True
        return S.EvaluateStmt(self.expr(e))

    def _lower_print_buffer(self, e):
        """``T.print(buffer)`` (reference ``language/print.py:144-238``): a fragment prints every
        thread's registers (``thread t: name[i]`` in local order); a shared / global / local
        buffer is printed whole by one thread of the block."""
        ctx = self.ctx
        msg, name = e.args[0], e.args[1]
        b = e.attrs.get("buffer")
        if b is None:
            raise LoweringError("T.print of a buffer lost its buffer reference")
        if b.scope == "fragment":
            lb = ctx.local_of(b)
            n = int(lb.shape[0])
            return L.CallStmt("tl::print_buffer", [msg, name, L.BufferPtr(lb, 0), IntImm(n)])
        n = b.static_numel()
        if n is None:
            raise LoweringError(f"T.print({b.name}): needs a static shape")
        if b.scope in ("local", "var"):
            return L.CallStmt("tl::print_buffer", [msg, name, L.BufferPtr(b, 0), IntImm(n)])
        ptr = L.BufferPtr(ctx.flat_of(b), ctx.flat_index(b, [IntImm(0)] * b.ndim))
        st = L.CallStmt("tl::print_buffer", [msg, name, ptr, IntImm(n)])
        if ctx.is_cpu:
            return st
        return S.SeqStmt([L.CallStmt("tl::sync_threads", []),
                          S.IfStmt(binop("==", ctx.tid, IntImm(0)), st)])

    def visit_AllocStmt(self, s):
        b = s.buffer
        if b.scope == "fragment":
            return S.AllocStmt(self.ctx.local_of(b))
        if b.scope == "shared":
            return S.AllocStmt(self.ctx.flat_of(b))
        return s

    def visit_ForStmt(self, s: S.ForStmt):
        if s.kind == "parallel":
            return self.lower_nest(s)
        if s.kind == "vectorized" and not self.ctx.is_cpu:
            r = self.lower_vectorized(s)
            if r is not None:
                return r
        mn, ext = as_int(s.min), as_int(s.extent)
        if mn is not None and ext is not None and ext > 0:
            self.ctx.ranges[s.var] = (mn, mn + ext - 1)
        body = self.stmt(s.body)
        kind = s.kind if s.kind in ("serial", "unroll") else "serial"
        return S.ForStmt(s.var, self.expr(s.min), self.expr(s.extent), kind, body, s.annotations)

    def visit_IfStmt(self, s):
        rng = self._thread_range(s.cond)
        then = None
        if rng is not None:
            saved, saved_r = self.ctx.thread_range, self.ctx.ranges.get(self.ctx.tid)
            self.ctx.thread_range = rng
            self.ctx.ranges[self.ctx.tid] = (rng[0], rng[1] - 1)
            then = self.stmt(s.then_body)
            self.ctx.thread_range = saved
            self.ctx.ranges[self.ctx.tid] = saved_r
        else:
            then = self.stmt(s.then_body)
        return S.IfStmt(self.expr(s.cond), then, self.stmt(s.else_body) if s.else_body is not None else None)

    def _thread_range(self, cond):
        """``[lo, hi)`` when ``cond`` is a conjunction of comparisons of the (1-D) thread index
        with constants (``tx < 128``, ``tx >= 128 and tx < 256``) that narrows the block --
        tile ops under it are partitioned over those threads (the reference's thread-range
        aware layout inference, testing/python/language/test_tilelang_language_mask_op.py)."""
        from ..ir.expr import BinOp as _B
        k = self.ctx.kernel
        tvars = {self.ctx.tid}
        if len(k.threads) == 1:
            tvars |= set(k.thread_vars)
            if k.attrs.get("tid") is not None:
                tvars.add(k.attrs["tid"])
        lo, hi = 0, self.ctx.T
        stack = [cond]
        flip = {"<": ">", "<=": ">=", ">": "<", ">=": "<="}
        while stack:
            c = stack.pop()
            if not isinstance(c, _B):
                return None
            if c.op == "&&":
                stack += [c.a, c.b]
                continue
            if c.op not in flip:
                return None
            op, a, b = c.op, c.a, c.b
            if a not in tvars:
                op, a, b = flip[op], b, a
            if a not in tvars or as_int(b) is None:
                return None
            v = as_int(b)
            if op == "<":
                hi = min(hi, v)
            elif op == "<=":
                hi = min(hi, v + 1)
            elif op == ">":
                lo = max(lo, v + 1)
            else:
                lo = max(lo, v)
        if not (0 <= lo < hi <= self.ctx.T) or (lo, hi) == (0, self.ctx.T):
            return None
        return lo, hi

    def lower_vectorized(self, s: S.ForStmt):
        """``T.vectorized(n)`` over one store: chunks of W consecutive iterations become one
        vector access when every access is contiguous in the loop variable and W-aligned (the
        width follows the strides' common alignment, 16 bytes at most).  Anything else stays
        a serial loop (clang may still combine it)."""
        ctx = self.ctx
        ext = as_int(s.extent)
        if ext is None or ext < 2 or ctx.no_vectorize:
            return None
        body = list(s.body.stmts) if isinstance(s.body, S.SeqStmt) else [s.body]
        stores = [b for b in body if isinstance(b, S.StoreStmt)]
        if len(stores) != 1 or any(not isinstance(b, (S.StoreStmt, S.AttrStmt)) for b in body):
            return None
        eb = max([stores[0].buffer.dtype.bytes] + [n.buffer.dtype.bytes for n in post_order(stores[0].value)
                                                   if isinstance(n, BufferLoad)])
        W = 16 // eb
        while W >= 2:
            if ext % W == 0:
                o = Var("vo")
                saved = dict(ctx.ranges)
                ctx.ranges[o] = (0, ext // W - 1)
                group, pre = [], []
                for i in range(W):
                    it = binop("+", binop("+", s.min, binop("*", o, W)), i)
                    for b in body:
                        if isinstance(b, S.AttrStmt):
                            pre.append(self.stmt(S.AttrStmt(b.key, substitute(b.value, {s.var: it}), None)))
                        else:
                            group.append(self.stmt(Substituter({s.var: it}).stmt(b)))
                kd = dict(self.known_div)
                kd[o] = (1, 0)
                vec = vectorize_group(ctx, group, kd)
                ctx.ranges.clear()
                ctx.ranges.update(saved)
                if vec is not None:
                    return S.ForStmt(o, 0, ext // W, "serial", S.SeqStmt(pre + vec))
            W //= 2
        return None

    def visit_AttrStmt(self, s):
        if s.key != "assume":
            return S.AttrStmt(s.key, s.value, self.stmt(s.body) if s.body is not None else None)
        # T.assume(cond): divisibility facts (``N % 4 == 0``) feed the vectoriser, and the
        # condition reaches clang as __builtin_assume on the GPU
        from ..ir.expr import BinOp as _B
        stack = [s.value]
        while stack:
            c = stack.pop()
            if isinstance(c, _B) and c.op == "&&":
                stack += [c.a, c.b]
            elif isinstance(c, _B) and c.op == "==" and as_int(c.b) == 0 and isinstance(c.a, _B) and \
                    c.a.op == "%" and isinstance(c.a.a, Var) and as_int(c.a.b):
                self.known_div[c.a.a] = (as_int(c.a.b), 0)
        if self.ctx.is_cpu:
            return S.SeqStmt([])
        return L.CallStmt("__builtin_assume", [self.expr(s.value)])

    def visit_TileOpStmt(self, s):
        op = s.op
        fn = getattr(self, "lower_" + type(op).__name__, None)
        if fn is None:
            raise LoweringError(f"no lowering for tile op {type(op).__name__}")
        return fn(op)

    # -- parallel nests ----------------------------------------------------------------
    def lower_nest(self, outer: S.ForStmt, layout: Optional[Fragment] = None):
        nest = ParallelNest(_nest_loops(outer))
        if self.ctx.is_cpu:
            return self.lower_cpu_nest(nest)
        layout = layout or outer.annotations.get("_layout")
        if layout is not None:
            return self.lower_frag_nest(nest, layout)
        if nest.fragment_accesses():
            raise LoweringError("T.Parallel over fragments without an inferred layout")
        return self.lower_simt_nest(nest)

    def lower_cpu_nest(self, nest: ParallelNest) -> S.Stmt:
        """CPU target: one thread owns every fragment element (row-major local arrays), so a
        parallel nest is a plain loop nest."""
        ctx = self.ctx

        class _Cpu(_SimtRewriter):

            def _acc(self, n):
                if isinstance(n, BufferLoad) and n.buffer.scope == "fragment":
                    return BufferLoad(ctx.local_of(n.buffer), [n.buffer.offset_of(n.indices)])
                return _SimtRewriter._acc(self, n)

            def store(self, s):
                if s.buffer.scope == "fragment":
                    return S.StoreStmt(ctx.local_of(s.buffer), [s.buffer.offset_of([self.expr(i) for i in s.indices])],
                                       self.expr(s.value))
                return _SimtRewriter.store(self, s)

        saved = dict(ctx.ranges)
        for l in nest.loops:  # the loop vars' ranges let the bounds prover drop guards
            mn, ext = as_int(l.min), as_int(l.extent)
            if mn is not None and ext is not None and ext > 0:
                ctx.ranges[l.var] = (mn, mn + ext - 1)
        body = _Cpu(ctx, {}).stmt(nest.body)
        ctx.ranges.clear()
        ctx.ranges.update(saved)
        for l in reversed(nest.loops):
            body = S.ForStmt(l.var, l.min, l.extent, "serial", body)
        return body

    def lower_frag_nest(self, nest: ParallelNest, layout: Fragment) -> S.Stmt:
        ctx = self.ctx
        res = _FragResolver(ctx, nest.vars, nest.mins, layout)
        W = layout.inner_vector_width(len(nest.vars) - 1)
        out = []
        body_is_single_store = isinstance(nest.body, S.StoreStmt)
        body_is_atomic_add = _atomic_add_call(nest.body) is not None
        for r0 in range(0, layout.local_size, W):
            group = []
            for r in range(r0, r0 + W):
                idx = layout.inverse(ctx.tid, r)
                vmap = {v: binop("+", m, i) for v, m, i in zip(nest.vars, nest.mins, idx)}
                rw = _IterRewriter(ctx, res, r, vmap)
                group.append(rw.stmt(nest.body))
            if body_is_atomic_add and W > 1 and not ctx.no_vectorize:
                vec = vectorize_atomic_group(ctx, group, self.known_div)
                if vec is not None:
                    out.extend(vec)
                    continue
            if body_is_single_store and W > 1 and not ctx.no_vectorize:
                vec = vectorize_group(ctx, group, self.known_div)
                if vec is not None:
                    out.extend(vec)
                    continue
            if not body_is_single_store:
                # scope each iteration (let bindings are per-iteration)
                out.extend(_scoped(g) for g in group)
            else:
                out.extend(group)
        return S.SeqStmt(out)

    def lower_simt_nest(self, nest: ParallelNest) -> S.Stmt:
        """Partition a nest over plain (global/shared/local) buffers across the block's threads."""
        ctx = self.ctx
        exts = nest.extents
        if any(e is None for e in exts):
            return self.lower_dynamic_nest(nest)
        total = _prod(exts)
        T, tid = ctx.T, ctx.tid
        if ctx.thread_range is not None:
            # under ``if lo <= tx < hi``: the nest is partitioned over those hi - lo threads only
            lo, hi = ctx.thread_range
            T, tid = hi - lo, (binop("-", ctx.tid, lo) if lo else ctx.tid)
        inner_var = nest.vars[-1]
        # vector width: contiguous along the innermost loop var for every access
        vec = 1
        cw = nest.outer.annotations.get("coalesced_width")
        accs = nest.accesses()
        max_eb = max([b.dtype.bytes for b, _, _ in accs] or [4])
        cand = cw if cw else max(1, 16 // max_eb)
        ac = _atomic_add_call(nest.body)
        if ctx.no_vectorize or (ac is not None and not cw and str(ac.args[0].buffer.dtype) == "float32"):
            # f32 atomics have no vector form: one element per lane keeps each wave instruction on
            # 64 consecutive floats (256 bytes) instead of every fourth float of 1 KiB
            cand = 1
        while cand > 1:
            if exts[-1] % cand == 0 and total // cand >= 1 and self._vec_ok(nest, cand):
                vec = cand
                break
            cand //= 2
        slots = total // vec
        steps = -(-slots // T)
        out = []
        single_store = isinstance(nest.body, S.StoreStmt)
        for o in range(steps):
            slot = binop("+", binop("*", o, T), tid) if steps > 1 else tid
            guard = None
            if (o + 1) * T > slots:
                guard = binop("<", slot, slots)
            # inside the tail guard only threads tid < slots - o*T run: tighten tid's range so the
            # bounds prover can drop per-element guards that only the idle threads would fail
            saved = ctx.ranges.get(ctx.tid)
            lo = ctx.thread_range[0] if ctx.thread_range is not None else 0
            if guard is not None and saved is not None and lo + slots - o * T - 1 < saved[1]:
                ctx.ranges[ctx.tid] = (saved[0], lo + slots - o * T - 1)
            group = []
            for v in range(vec):
                lin = binop("+", binop("*", slot, vec), v) if vec > 1 else slot
                vals = _unflatten(lin, exts)
                vmap = {var: binop("+", m, x) for var, m, x in zip(nest.vars, nest.mins, vals)}
                rw = _SimtRewriter(ctx, vmap)
                group.append(rw.stmt(nest.body))
            if saved is not None:
                ctx.ranges[ctx.tid] = saved
            stmts = None
            if single_store and vec > 1:
                kd = dict(self.known_div)
                kd[ctx.tid] = (1, 0)
                stmts = vectorize_group(ctx, group, _slot_div(kd, ctx.tid, o, T, vec))
            elif vec > 1 and _atomic_add_call(nest.body) is not None:
                kd = dict(self.known_div)
                kd[ctx.tid] = (1, 0)
                stmts = vectorize_atomic_group(ctx, group, _slot_div(kd, ctx.tid, o, T, vec))
            if stmts is None:
                stmts = [_scoped(g) for g in group] if not single_store else group
            blk = S.SeqStmt(stmts)
            out.append(S.IfStmt(guard, blk) if guard is not None else blk)
        return S.SeqStmt(out)

    def _no_thread_range(self, op):
        """Paths that spread their work over all ctx.T threads refuse ``if lo <= tx < hi``
        partitioning instead of silently skipping the elements of the idle threads."""
        if self.ctx.thread_range is not None:
            raise LoweringError(f"{type(op).__name__} inside a thread-range condition "
                                f"(threads {self.ctx.thread_range[0]}..{self.ctx.thread_range[1] - 1} of "
                                f"{self.ctx.T}) is not supported: move it out of the condition")

    def lower_dynamic_nest(self, nest: ParallelNest) -> S.Stmt:
        ctx = self.ctx
        total = const(1)
        for l in nest.loops:
            total = total * l.extent
        it = Var("it")
        T, tid = ctx.T, ctx.tid
        if ctx.thread_range is not None:
            # under ``if lo <= tx < hi`` only those hi - lo threads run the nest (as lower_simt_nest)
            lo, hi = ctx.thread_range
            T, tid = hi - lo, (binop("-", ctx.tid, lo) if lo else ctx.tid)
        lin = binop("+", binop("*", it, T), tid)
        vals = _unflatten_dyn(lin, [l.extent for l in nest.loops])
        vmap = {var: binop("+", m, x) for var, m, x in zip(nest.vars, nest.mins, vals)}
        body = _SimtRewriter(ctx, vmap).stmt(nest.body)
        from ..ir.expr import ceildiv
        n_it = ceildiv(total, T)
        return S.ForStmt(it, 0, n_it, "serial", S.IfStmt(binop("<", lin, total), body))

    def _vec_ok(self, nest: ParallelNest, vec: int) -> bool:
        v = nest.vars[-1]
        for b, idx, _ in nest.accesses():
            if b.scope == "fragment":
                return False
            if not idx:
                continue
            # innermost buffer index must be v (+ something not involving v); other dims free of v
            for d, e in enumerate(idx):
                uses = any(n is v for n in post_order(e))
                if d < len(idx) - 1 and uses:
                    return False
            last = idx[-1]
            if any(n is v for n in post_order(last)):
                rest = substitute(last, {v: IntImm(0)})
                if _const_diff(last, rest, []) is None:
                    # coefficient of v must be exactly 1
                    d1 = _const_diff(substitute(last, {v: IntImm(1)}), rest, [])
                    if d1 != 1:
                        return False
                d1 = _const_diff(substitute(last, {v: IntImm(1)}), rest, [])
                if d1 != 1:
                    return False
                if b.scope == "global":
                    st = b.get_strides()
                    if as_int(st[-1]) != 1:
                        return False
                    for s_ in st[:-1]:
                        if not divisible_by(convert(s_), vec, self.known_div):
                            return False
                    if not divisible_by(rest, vec, self.known_div):
                        return False
                if b.scope == "shared" and b.layout is not None and isinstance(b.layout, SwizzleLayout):
                    if (vec * b.dtype.bytes) > 16 or (b.layout.epc % vec and vec % b.layout.epc):
                        return False
        return True

    # -- tile ops ---------------------------------------------------------------------
    def lower_FillOp(self, op: O.FillOp):
        b = op.dst.buffer
        val = self.expr(op.value)
        if b.scope == "fragment":
            lb = self.ctx.local_of(b)
            if not _full(op.dst):
                raise LoweringError("T.fill on a fragment must cover the whole fragment")
            v = cast(val, b.dtype)
            if ctx_is_cpu(self.ctx):
                i = Var("fi")
                return S.ForStmt(i, 0, lb.shape[0], "serial", S.StoreStmt(lb, [i], v))
            return S.SeqStmt([S.StoreStmt(lb, [IntImm(i)], v) for i in range(lb.shape[0])])
        if b.scope in ("local", "var"):
            n = as_int(b.numel())
            return S.SeqStmt([S.StoreStmt(b, [IntImm(i)], cast(val, b.dtype)) for i in range(n)])
        nest = _region_nest(op.dst, lambda idx: (op.dst.buffer, idx, cast(val, b.dtype)))
        return self.lower_nest(nest)

    def lower_CopyOp(self, op: O.CopyOp):
        src, dst = op.src, op.dst
        sf, df = src.buffer.scope == "fragment", dst.buffer.scope == "fragment"
        if sf or df:
            return self.lower_frag_copy(op)
        if src.buffer.scope == "local" and dst.buffer.scope == "local":
            pass
        nest = _copy_nest(src, dst, op.coalesced_width)
        return self.lower_nest(nest)

    def lower_frag_copy(self, op: O.CopyOp):
        src, dst = op.src, op.dst
        frag_side = dst if dst.buffer.scope == "fragment" else src
        fb = frag_side.buffer
        if not _full(frag_side):
            return self.lower_partial_frag_copy(op, frag_side is dst)
        nest = _copy_nest(src, dst, None)
        loops = _nest_loops(nest)
        fshape = fb.static_shape()
        # loop dims correspond to the squeezed extents; map fragment dims onto loop vars
        lay = fb.layout
        squeezed_lay = _squeeze_fragment(lay, fshape)
        loop_lay = squeezed_lay
        if [as_int(l.extent) for l in loops] != squeezed_lay.shape:
            raise LoweringError(f"T.copy shape mismatch for fragment {fb.name}")
        return self.lower_nest(nest, loop_lay)

    def lower_partial_frag_copy(self, op: O.CopyOp, into_frag: bool):
        """Copy between a sub-tile of a fragment and another buffer (e.g. the valid rows of a
        padded MFMA tile): iterate the whole fragment with its own partition and predicate the
        elements that fall inside the region."""
        fr, other = (op.dst, op.src) if into_frag else (op.src, op.dst)
        fb = fr.buffer
        fshape = fb.static_shape()
        fext, oext = fr.static_extents(), other.static_extents()
        fmins = [as_int(m) for m in fr.mins]
        if fext is None or oext is None or any(m is None for m in fmins):
            raise LoweringError(f"T.copy on a sub-tile of fragment {fb.name} needs static bounds")
        fd = [d for d, e in enumerate(fext) if e != 1]
        od = [d for d, e in enumerate(oext) if e != 1]
        if [fext[d] for d in fd] != [oext[d] for d in od]:
            raise LoweringError(f"T.copy extents mismatch: {fb.name}{fext} vs {other.buffer.name}{oext}")
        vars_ = [Var(f"pf{d}") for d in range(len(fshape))]
        conds = []
        for d, (m, e, s) in enumerate(zip(fmins, fext, fshape)):
            if m == 0 and e == s:
                continue
            if e == 1:
                conds.append(binop("==", vars_[d], m))
            else:
                conds.append(logical_and(binop(">=", vars_[d], m), binop("<", vars_[d], m + e)))
        oidx = list(other.mins)
        for k, d in enumerate(od):
            oidx[d] = binop("+", other.mins[d], binop("-", vars_[fd[k]], fmins[fd[k]]))
        fl = BufferLoad(fb, list(vars_))
        ol = BufferLoad(other.buffer, oidx)
        if into_frag:
            body = S.StoreStmt(fb, list(vars_), cast(ol, fb.dtype))
        else:
            body = S.StoreStmt(other.buffer, oidx, cast(fl, other.buffer.dtype))
        cond = None
        for c in conds:
            cond = c if cond is None else logical_and(cond, c)
        if cond is not None:
            body = S.IfStmt(cond, body)
        for v, s in reversed(list(zip(vars_, fshape))):
            body = S.ForStmt(v, 0, s, "parallel", body)
        return self.lower_nest(body, fb.layout)

    def lower_GemmOp(self, op: O.GemmOp):
        ctx = self.ctx
        plan = getattr(op, "plan", None)
        if plan is None:
            plan = gemm_lower.gemm_plan(op, ctx.T, ctx.target,
                                        op.A.buffer.layout if op.A.buffer.scope == "fragment" else None)
        A, B, C = op.A.buffer, op.B.buffer, op.C.buffer
        if C.scope != "fragment":
            raise LoweringError("T.gemm accumulator must be a fragment (T.alloc_fragment)")
        out = []
        cl = ctx.local_of(C)
        if op.clear_accum is not False and op.clear_accum is not None:
            zero = S.SeqStmt([S.StoreStmt(cl, [IntImm(i)], const(0.0, C.dtype)) for i in range(cl.shape[0])])
            ca = op.clear_accum
            if isinstance(ca, bool) or as_int(ca) is not None:
                if bool(as_int(ca) if not isinstance(ca, bool) else ca):
                    out.append(zero)
            else:
                out.append(S.IfStmt(self.expr(ca), zero))
        ctype = _dt.hip_type(A.dtype)
        if op.is_mx:
            return self._lower_mx_gemm(op, plan, cl, out)
        if op.is_sp:
            return self._lower_sp_gemm(op, plan, cl, out)
        if ctx.is_cpu:
            pa = self._operand_ptr(op.A)
            pb = self._operand_ptr(op.B)
            a_cols = (A.static_shape() or [0])[-1]
            b_cols = (B.static_shape() or [0])[-1]
            out.append(L.CallStmt("tl::cpu_gemm", [pa, pb, L.BufferPtr(cl, 0)],
                                  [_dt.cpu_type(A.dtype), plan["M"], plan["N"], plan["K"], int(op.trans_A),
                                   int(op.trans_B), a_cols, b_cols]))
            return S.SeqStmt(out)
        if B.scope != "shared":
            raise LoweringError("T.gemm: B operand must be in shared memory on gfx950")
        pb = self._operand_ptr(op.B)
        if plan.get("int8"):
            pa = self._operand_ptr(op.A)
            out.append(L.CallStmt("tl::gemm_ss_i8", [pa, pb, L.BufferPtr(cl, 0), ctx.wave_expr()], [
                plan["mfma"][0], plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"],
                A.static_shape()[-1], f"{gemm_lower.encode_swizzle(A.layout)}u",
                B.static_shape()[-1], f"{gemm_lower.encode_swizzle(B.layout)}u"]))
            return S.SeqStmt(out)
        if plan.get("f32"):
            pa = self._operand_ptr(op.A)
            out.append(L.CallStmt("tl::gemm_ss_f32", [pa, pb, L.BufferPtr(cl, 0), ctx.wave_expr()], [
                plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"], _b(op.trans_A), _b(op.trans_B),
                A.static_shape()[-1], B.static_shape()[-1]]))
            return S.SeqStmt(out)
        vm = [self.expr(op.valid_m)] if getattr(op, "valid_m", None) is not None else []
        if vm and (plan.get("int8") or plan.get("f32") or A.dtype.bits == 8 or A.scope != "shared"):
            raise LoweringError("T.gemm(valid_m=) is supported for f16/bf16 GEMMs with both operands in shared "
                                "memory")
        if plan.get("mfma") == (32, 32, 16) and A.scope == "fragment":
            if vm:
                raise LoweringError("T.gemm(valid_m=) needs both operands in shared memory")
            out.append(L.CallStmt("tl::gemm_rs_32", [L.BufferPtr(ctx.local_of(A), 0), pb, L.BufferPtr(cl, 0),
                                                     ctx.wave_expr()], [
                ctype, plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"], _b(op.trans_B),
                B.static_shape()[-1], f"{gemm_lower.encode_swizzle(B.layout)}u", plan.get("a_kperm", 0)]))
            return S.SeqStmt(out)
        if plan.get("mfma") == (32, 32, 16):
            pa = self._operand_ptr(op.A)
            out.append(L.CallStmt("tl::gemm_ss_32", [pa, pb, L.BufferPtr(cl, 0)] + (vm or [IntImm(0x3fffffff)]) +
                                  [ctx.wave_expr()], [
                ctype, plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"], _b(op.trans_A),
                _b(op.trans_B), A.static_shape()[-1], f"{gemm_lower.encode_swizzle(A.layout)}u",
                B.static_shape()[-1], f"{gemm_lower.encode_swizzle(B.layout)}u"]))
            return S.SeqStmt(out)
        if A.dtype.bits == 8:
            pa = self._operand_ptr(op.A)
            out.append(L.CallStmt("tl::gemm_ss_f8", [pa, pb, L.BufferPtr(cl, 0), ctx.wave_expr()], [
                _dt.hip_type(A.dtype), _dt.hip_type(B.dtype), plan["M"], plan["N"], plan["K"], plan["warp_m"],
                plan["warp_n"], A.static_shape()[-1], f"{gemm_lower.encode_swizzle(A.layout)}u",
                B.static_shape()[-1], f"{gemm_lower.encode_swizzle(B.layout)}u", _b(op.trans_B)
            ]))
            return S.SeqStmt(out)
        b_cols = B.static_shape()[-1]
        swz_b = gemm_lower.encode_swizzle(B.layout)
        frag = getattr(op, "frag", None)
        if frag is not None:
            # register-prefetched K-half schedule (transform/pipeline.py _prefetch_schedule)
            if A.scope != "shared":
                raise LoweringError("prefetched T.gemm needs both operands in shared memory")
            mode, var = frag[0], frag[1]
            shape = [ctype, plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"]]
            if mode == "decl":
                return L.ObjDeclStmt(f"tl::ss_frags<{', '.join(str(x) for x in shape)}>", var)
            ksteps = plan["K"] // 32
            m_rep = plan["M"] // plan["warp_m"] // 16
            n_rep = plan["N"] // plan["warp_n"] // 16
            nload = ksteps * (m_rep * (2 if op.trans_A else 1) + n_rep * (1 if op.trans_B else 2))
            if getattr(ctx.target, "gemm_interleave", None) is False:
                nload = 0
            calls = []
            if mode in ("load", "load_mma"):
                calls.append(L.CallStmt("tl::gemm_ss_load", [self._operand_ptr(op.A), pb, var, ctx.wave_expr()],
                                        shape + [_b(op.trans_A), _b(op.trans_B), A.static_shape()[-1],
                                                 f"{gemm_lower.encode_swizzle(A.layout)}u", b_cols, f"{swz_b}u"]))
            if mode in ("mma", "load_mma"):
                # interleaved with the load issued just before it (same phase, same basic block)
                mvar = frag[2] if mode == "load_mma" else var
                calls.append(L.CallStmt("tl::gemm_ss_mma", [mvar, L.BufferPtr(cl, 0)],
                                        shape + [nload if mode == "load_mma" else 0]))
            body = S.seq(*calls)
            if vm:
                # T.gemm(valid_m=): a wave whose rows are all padding skips its reads and MFMAs
                # (the tile's valid-row count is fixed over the K loop, so the two fragment sets
                # stay consistent); one uniform branch around the load+MMA pair keeps them in
                # one basic block for the interleave
                wm = binop("//", ctx.wave_expr(), IntImm(plan["warp_n"]))
                body = S.IfStmt(binop("<", binop("*", wm, IntImm(plan["M"] // plan["warp_m"])), vm[0]), body)
            out.append(body)
            return S.SeqStmt(out)
        if A.scope == "shared":
            pa = self._operand_ptr(op.A)
            a_cols = A.static_shape()[-1]
            swz_a = gemm_lower.encode_swizzle(A.layout)
            out.append(L.CallStmt("tl::gemm_ss", [pa, pb, L.BufferPtr(cl, 0)] + (vm or [IntImm(0x3fffffff)]) +
                                  [ctx.wave_expr()], [
                ctype, plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"], _b(op.trans_A),
                _b(op.trans_B), a_cols, f"{swz_a}u", b_cols, f"{swz_b}u"
            ]))
        elif A.scope == "fragment":
            al = ctx.local_of(A)
            # transpose_A: the fragment is the [M, K] layout with its dims swapped
            # (layout.mfma.transpose_fragment): the registers are consumed unchanged
            vmin = [self.expr(op.valid_m_min)] if getattr(op, "valid_m_min", None) is not None else []
            out.append(L.CallStmt("tl::gemm_rs", [L.BufferPtr(al, 0), pb, L.BufferPtr(cl, 0), ctx.wave_expr()] + vmin, [
                ctype, plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"], _b(op.trans_B), b_cols,
                f"{swz_b}u", plan.get("a_kperm", 0), int(getattr(ctx.target, "gemm_rs_pipe", None) or 0)
            ]))
        else:
            raise LoweringError(f"T.gemm: A operand scope {A.scope} unsupported")
        return S.SeqStmt(out)

    def _lower_mx_gemm(self, op: O.GemmOp, plan, cl, out):
        """``tl::gemm_ss_mx`` / ``tl::cpu_gemm_mx``: block-scaled (e8m0) fp8/fp4 GEMM."""
        A, B = op.A.buffer, op.B.buffer
        pa, pb = self._operand_ptr(op.A), self._operand_ptr(op.B)
        psa, psb = self._operand_ptr(op.scale_A), self._operand_ptr(op.scale_B)
        sa_shape, sb_shape = op.scale_A.buffer.static_shape(), op.scale_B.buffer.static_shape()
        if sa_shape is None or sb_shape is None:
            raise LoweringError("T.gemm_scaled: scale buffers need static shapes (row stride)")
        targs = [plan["a_code"], plan["b_code"], plan["M"], plan["N"], plan["K"]]
        ps = int(getattr(op, "scale_ps", False))
        if ps:
            # tile shapes checked at plan time (gemm_lower._mx_plan)
            if not self.ctx.is_cpu and ((plan["M"] // plan["warp_m"]) % 64 or (plan["N"] // plan["warp_n"]) % 64):
                raise LoweringError("T.gemm_scaled(scale_layout='preshuffled') needs warp tiles of 64 rows and "
                                    f"columns (got {plan['M'] // plan['warp_m']} x {plan['N'] // plan['warp_n']})")
        if self.ctx.is_cpu:
            targs += [A.static_shape()[-1], B.static_shape()[-1], sa_shape[-1], sb_shape[-1], ps]
            out.append(L.CallStmt("tl::cpu_gemm_mx", [pa, pb, psa, psb, L.BufferPtr(cl, 0)], targs))
            return S.SeqStmt(out)
        for buf in (A, B):
            # gemm_ss_mx computes each lane's swizzled address once from row bits 0..3 (the 16 rows
            # a lane group covers) and strides by 16 rows; a swizzle on a higher row bit breaks that
            swz = gemm_lower.encode_swizzle(buf.layout)
            hi = max(((swz >> (4 * cb)) & 15) for cb in range(8))
            if hi > 4:
                raise LoweringError(f"T.gemm_scaled: the LDS swizzle of {buf.name} XORs row bit {hi - 1} into the "
                                    "column; block-scaled GEMM operands may only swizzle on row bits 0..3 "
                                    "(drop the annotate_layout or use make_mfma_swizzle_layout)")
        targs += [plan["warp_m"], plan["warp_n"], A.static_shape()[-1], f"{gemm_lower.encode_swizzle(A.layout)}u",
                  B.static_shape()[-1], f"{gemm_lower.encode_swizzle(B.layout)}u", sa_shape[-1], sb_shape[-1], ps]
        out.append(L.CallStmt("tl::gemm_ss_mx", [pa, pb, psa, psb, L.BufferPtr(cl, 0), self.ctx.wave_expr()], targs))
        return S.SeqStmt(out)

    def _lower_sp_gemm(self, op: O.GemmOp, plan, cl, out):
        """``tl::gemm_sp_ss`` (v_smfmac_f32_16x16x64) / ``tl::cpu_gemm_sp``: 2:4 sparse A."""
        A, B, E = op.A.buffer, op.B.buffer, op.E.buffer
        pa, pb, pe = self._operand_ptr(op.A), self._operand_ptr(op.B), self._operand_ptr(op.E)
        e_shape = E.static_shape()
        if e_shape is None:
            raise LoweringError("T.gemm_sp: the metadata buffer needs a static shape (row stride)")
        ctype = (_dt.cpu_type if self.ctx.is_cpu else _dt.hip_type)(A.dtype)
        if self.ctx.is_cpu:
            out.append(L.CallStmt("tl::cpu_gemm_sp", [pa, pe, pb, L.BufferPtr(cl, 0)], [
                ctype, plan["M"], plan["N"], plan["K"], int(op.trans_A), int(op.trans_B), A.static_shape()[-1],
                e_shape[-1], B.static_shape()[-1]]))
            return S.SeqStmt(out)
        out.append(L.CallStmt("tl::gemm_sp_ss", [pa, pe, pb, L.BufferPtr(cl, 0), self.ctx.wave_expr()], [
            ctype, plan["M"], plan["N"], plan["K"], plan["warp_m"], plan["warp_n"], _b(op.trans_A), _b(op.trans_B),
            A.static_shape()[-1], f"{gemm_lower.encode_swizzle(A.layout)}u", e_shape[-1],
            B.static_shape()[-1], f"{gemm_lower.encode_swizzle(B.layout)}u"]))
        return S.SeqStmt(out)

    def _operand_ptr(self, r: BufferRegion):
        b = r.buffer
        mins = [self.expr(m) for m in r.mins]
        if b.scope == "fragment":
            return L.BufferPtr(self.ctx.local_of(b), 0)
        off = self.ctx.flat_index(b, mins)
        return L.BufferPtr(self.ctx.flat_of(b), off)

    def lower_ReduceOp(self, op: O.ReduceOp):
        ctx = self.ctx
        sb, db = op.src.buffer, op.dst.buffer
        if ctx.is_cpu:
            return self.lower_reduce_cpu(op)
        if sb.scope != "fragment" or db.scope != "fragment":
            return self.lower_reduce_simt(op)
        S_lay: Fragment = sb.layout
        D_lay: Fragment = db.layout
        kind = op.reduce_type
        dim = op.dim
        sl, dl = ctx.local_of(sb), ctx.local_of(db)
        dshape = db.static_shape()
        squeeze_dim = len(dshape) == len(S_lay.shape)  # dst keeps a unit dim
        # group source registers by destination register (must be thread-uniform).  When the
        # destination was laid out by another consumer first, reduce into the natural layout
        # (the reduced dim's digits dropped) and redistribute through LDS afterwards.
        groups = self._reduce_groups(S_lay, D_lay, dim, squeeze_dim)
        redistribute = None
        if groups is None:
            from .layout_inference import reduce_dst_layout
            redistribute = D_lay
            D_lay = reduce_dst_layout(S_lay, dim, dshape)
            if D_lay.num_threads < ctx.T:
                D_lay = D_lay.replicate(ctx.T // D_lay.num_threads)
            groups = self._reduce_groups(S_lay, D_lay, dim, squeeze_dim)
            if groups is None:
                raise LoweringError(f"reduce: cannot map {sb.name} onto a reduced layout")
        out = []
        accs = {}
        dt = sb.dtype
        for d, rs in sorted(groups.items()):
            xs = []
            for r in rs:
                x = BufferLoad(sl, [IntImm(r)])
                if kind in ("abssum", "absmax"):
                    x = call("abs", [x], dt)
                xs.append(x)
            accs[d] = _tree_combine(kind, xs)
        # cross-thread: thread digits of the reduced dim
        lane_mask, wave_digits = _reduce_thread_masks(S_lay, dim)
        opname = _REDUCE_OPS[kind][0]
        tmp_vars = {}
        for d, acc in accs.items():
            v = Var(f"red{d}", dt, nonneg=False)
            out.append(S.LetStmt(v, acc))
            tmp_vars[d] = v
        red_vals = {}
        if lane_mask:
            for d, v in tmp_vars.items():
                v2 = Var(f"redl{d}", dt, nonneg=False)
                out.append(S.LetStmt(v2, call("extern", ["tl::lane_allreduce<%s, %d>" % (opname, lane_mask), v], dt)))
                red_vals[d] = v2
        else:
            red_vals = dict(tmp_vars)
        if wave_digits:
            # cross-wave through an LDS workspace: ws[d][tid]
            nd = len(red_vals)
            ws = ctx.new_workspace(nd * ctx.T, dt)
            wsf = ctx.flat_of(ws)
            keys = sorted(red_vals)
            # barriers: only the one between the workspace stores and the partner loads is
            # structural; the ones before the stores (WAR against an earlier use of this
            # workspace) and after the loads are left to ThreadSync, which places them only
            # where an access since the last barrier conflicts (a softmax's max and sum
            # reductions in one tile had 3 barriers each, 2 of them redundant)
            if ctx.self_sync:
                out.append(L.CallStmt("tl::sync_threads", []))  # WAR vs an earlier use of the workspace
            for j, d in enumerate(keys):
                out.append(S.StoreStmt(wsf, [binop("+", j * ctx.T, ctx.tid)], red_vals[d]))
            out.append(L.CallStmt("tl::sync_threads", []))
            partners = _partner_offsets(ctx.tid, wave_digits)
            new_vals = {}
            for j, d in enumerate(keys):
                acc = None
                for p in partners:
                    x = BufferLoad(wsf, [binop("+", j * ctx.T, p)])
                    acc = x if acc is None else _combine(kind, acc, x)
                v3 = Var(f"redw{d}", dt, nonneg=False)
                out.append(S.LetStmt(v3, acc))
                new_vals[d] = v3
            red_vals = new_vals
            if ctx.self_sync:
                out.append(L.CallStmt("tl::sync_threads", []))
        if redistribute is not None:
            # natural-layout results -> LDS (logical row-major) -> the consumer's layout
            n = _prod(dshape)
            ws = ctx.new_workspace(n, dt)
            wsf = ctx.flat_of(ws)
            if ctx.self_sync:
                out.append(L.CallStmt("tl::sync_threads", []))
            for d, v in red_vals.items():  # (surrounding barriers: ThreadSync, as above)
                idx = D_lay.inverse(ctx.tid, d)
                out.append(S.StoreStmt(wsf, [_row_major(idx, dshape)], v))
            out.append(L.CallStmt("tl::sync_threads", []))
            red_vals = {}
            for r in range(redistribute.local_size):
                idx = redistribute.inverse(ctx.tid, r)
                v = Var(f"redx{r}", dt, nonneg=False)
                out.append(S.LetStmt(v, BufferLoad(wsf, [_row_major(idx, dshape)])))
                red_vals[r] = v
            if ctx.self_sync:
                out.append(L.CallStmt("tl::sync_threads", []))
        for d, v in red_vals.items():
            if op.clear:
                out.append(S.StoreStmt(dl, [IntImm(d)], cast(v, db.dtype)))
            else:
                out.append(S.StoreStmt(dl, [IntImm(d)], cast(_combine(kind, BufferLoad(dl, [IntImm(d)]), v),
                                                             db.dtype)))
        return _scoped(S.SeqStmt(out))

    def _reduce_groups(self, S_lay: Fragment, D_lay: Fragment, dim: int, squeeze_dim: bool):
        """src register -> dst register grouping, or None when some thread does not own the
        destination of an element it holds (the layouts are not reduce-compatible).  The proof
        runs over every thread of the block in the native core (csrc/core/fragment.cc
        ``reduce_owners``)."""
        from .._native import core
        own = core().reduce_owners(S_lay.native, D_lay.native, dim, bool(squeeze_dim), self.ctx.T)
        if len(own) == 0:
            return None
        groups: Dict[int, List[int]] = {}
        for r, li in enumerate(own):
            groups.setdefault(li, []).append(r)
        return groups

    def lower_reduce_cpu(self, op: O.ReduceOp):
        """CPU target: one thread owns every element (fragments are row-major local arrays), so a
        reduction is a loop nest -- not the GPU path's unrolled per-register combine tree, whose
        65k-term expressions host clang cannot digest for a 256x256 tile."""
        ctx = self.ctx
        src, dst = op.src, op.dst
        sext = src.static_extents()
        if sext is None:
            raise LoweringError("reduce needs static extents")
        dim = op.dim
        outer = [e for d, e in enumerate(sext) if d != dim]
        ovars = [Var(f"ro{i}") for i in range(len(outer))]
        k = Var("rk")
        sidx = list(ovars)
        sidx.insert(dim, k)
        sidx = [binop("+", m, i) for m, i in zip(src.mins, sidx)]
        didx = list(ovars)
        if len(dst.region) == len(src.region):
            didx.insert(dim, IntImm(0))
        didx = [binop("+", m, i) for m, i in zip(dst.mins, didx)]
        dt = src.buffer.dtype
        accb = ctx.new_local(f"racc{ctx.ws_counter}", 1, dt)
        ctx.ws_counter += 1
        x = BufferLoad(src.buffer, sidx)
        if op.reduce_type in ("abssum", "absmax"):
            x = call("abs", [x], dt)
        res = BufferLoad(accb, [IntImm(0)])
        if not op.clear:
            res = _combine(op.reduce_type, BufferLoad(dst.buffer, didx), res)
        body = S.SeqStmt([
            S.StoreStmt(accb, [IntImm(0)], _reduce_init(op.reduce_type, dt)),
            S.ForStmt(k, 0, sext[dim], "serial",
                      S.StoreStmt(accb, [IntImm(0)], _combine(op.reduce_type, BufferLoad(accb, [IntImm(0)]), x))),
            S.StoreStmt(dst.buffer, didx, cast(res, dst.buffer.dtype))])
        if not ovars:
            ovars, outer = [Var("ro0")], [1]
        for v, e in reversed(list(zip(ovars, outer))):
            body = S.ForStmt(v, 0, e, "parallel", body)
        return self.lower_cpu_nest(ParallelNest(_nest_loops(body)))

    def lower_reduce_simt(self, op: O.ReduceOp):
        """Reduction over shared/local buffers: each thread reduces whole rows serially."""
        self._no_thread_range(op)
        ctx = self.ctx
        src, dst = op.src, op.dst
        sext = src.static_extents()
        if sext is None:
            raise LoweringError("reduce needs static extents")
        dim = op.dim
        outer = [e for d, e in enumerate(sext) if d != dim]
        n_out = _prod(outer)
        red_n = sext[dim]
        dt = src.buffer.dtype
        steps = -(-n_out // ctx.T)
        out = []
        for o in range(steps):
            slot = binop("+", o * ctx.T, ctx.tid)
            oidx = _unflatten(slot, outer)
            k = Var("rk")
            sidx = list(oidx)
            sidx.insert(dim, k)
            sidx = [binop("+", m, i) for m, i in zip(src.mins, sidx)]
            didx = list(oidx)
            if len(dst.region) == len(src.region):
                didx.insert(dim, IntImm(0))
            didx = [binop("+", m, i) for m, i in zip(dst.mins, didx)]
            acc = Var("racc", dt, nonneg=False)
            accb = ctx.new_local(f"racc{ctx.ws_counter}_{o}", 1, dt)
            ctx.ws_counter += 1
            x = BufferLoad(src.buffer, sidx)
            if op.reduce_type in ("abssum", "absmax"):
                x = call("abs", [x], dt)
            body = [S.StoreStmt(accb, [IntImm(0)], _reduce_init(op.reduce_type, dt)),
                    S.ForStmt(k, 0, red_n, "serial",
                              S.StoreStmt(accb, [IntImm(0)], _combine(op.reduce_type, BufferLoad(accb, [IntImm(0)]),
                                                                      x)))]
            res = BufferLoad(accb, [IntImm(0)])
            if not op.clear:
                res = _combine(op.reduce_type, BufferLoad(dst.buffer, didx), res)
            body.append(S.StoreStmt(dst.buffer, didx, cast(res, dst.buffer.dtype)))
            blk = self.stmt(S.SeqStmt(body))
            out.append(S.IfStmt(binop("<", slot, n_out), blk) if (o + 1) * ctx.T > n_out else blk)
        return S.SeqStmt(out)

    def lower_CumSumOp(self, op: O.CumSumOp):
        """Inclusive scan along ``dim`` for shared/global buffers (one thread per row)."""
        self._no_thread_range(op)
        ctx = self.ctx
        src, dst = op.src, op.dst
        frag = src.buffer.scope == "fragment" or dst.buffer.scope == "fragment"
        if frag and ctx.is_cpu:
            return self.lower_cumsum_cpu(op)
        if frag:
            return self.lower_cumsum_fragment(op)
        sext = src.static_extents()
        dim = op.dim
        outer = [e for d, e in enumerate(sext) if d != dim]
        n_out = _prod(outer)
        n = sext[dim]
        dt = dst.buffer.dtype
        out = [L.CallStmt("tl::sync_threads", [])]
        steps = -(-n_out // ctx.T)
        for o in range(steps):
            slot = binop("+", o * ctx.T, ctx.tid)
            oidx = _unflatten(slot, outer)
            k = Var("ck")
            kk = binop("-", n - 1, k) if op.reverse else k
            sidx = list(oidx)
            sidx.insert(dim, kk)
            didx = list(sidx)
            sidx = [binop("+", m, i) for m, i in zip(src.mins, sidx)]
            didx = [binop("+", m, i) for m, i in zip(dst.mins, didx)]
            accb = ctx.new_local(f"cacc{ctx.ws_counter}", 1, dt)
            ctx.ws_counter += 1
            body = [S.StoreStmt(accb, [IntImm(0)], const(0, dt)),
                    S.ForStmt(k, 0, n, "serial", S.SeqStmt([
                        S.StoreStmt(accb, [IntImm(0)], BufferLoad(accb, [IntImm(0)]) +
                                    cast(BufferLoad(src.buffer, sidx), dt)),
                        S.StoreStmt(dst.buffer, didx, BufferLoad(accb, [IntImm(0)]))]))]
            blk = self.stmt(S.SeqStmt(body))
            out.append(S.IfStmt(binop("<", slot, n_out), blk) if (o + 1) * ctx.T > n_out else blk)
        out.append(L.CallStmt("tl::sync_threads", []))
        return S.SeqStmt(out)

    def lower_cumsum_cpu(self, op: O.CumSumOp):
        """CPU target: fragments are row-major local arrays of the one thread -- a serial scan
        per row, as a loop nest over the other dims."""
        src, dst = op.src, op.dst
        sext = src.static_extents()
        dim = op.dim
        outer = [e for d, e in enumerate(sext) if d != dim]
        ovars = [Var(f"co{i}") for i in range(len(outer))]
        n = sext[dim]
        k = Var("ck")
        kk = binop("-", n - 1, k) if op.reverse else k
        idx = list(ovars)
        idx.insert(dim, kk)
        sidx = [binop("+", m, i) for m, i in zip(src.mins, idx)]
        didx = [binop("+", m, i) for m, i in zip(dst.mins, idx)]
        dt = dst.buffer.dtype
        accb = self.ctx.new_local(f"cacc{self.ctx.ws_counter}", 1, dt)
        self.ctx.ws_counter += 1
        body = S.SeqStmt([
            S.StoreStmt(accb, [IntImm(0)], const(0, dt)),
            S.ForStmt(k, 0, n, "serial", S.SeqStmt([
                S.StoreStmt(accb, [IntImm(0)], BufferLoad(accb, [IntImm(0)]) + cast(BufferLoad(src.buffer, sidx), dt)),
                S.StoreStmt(dst.buffer, didx, BufferLoad(accb, [IntImm(0)]))]))])
        if not ovars:
            ovars, outer = [Var("co0")], [1]
        for v, e in reversed(list(zip(ovars, outer))):
            body = S.ForStmt(v, 0, e, "parallel", body)
        return self.lower_cpu_nest(ParallelNest(_nest_loops(body)))

    def lower_cumsum_fragment(self, op: O.CumSumOp):
        """``T.cumsum`` of a register fragment (reference ``src/op/reduce.cc:496-560``): the
        fragment goes to an LDS workspace through its layout, one thread per row scans it there,
        and the result comes back through the destination's layout.  A scan crosses the lanes
        that own a row; staging once through LDS costs two barriers and no shuffles."""
        ctx = self.ctx
        src, dst = op.src, op.dst
        for r in (src, dst):
            if r.buffer.scope == "fragment" and not _full(r):
                raise LoweringError("T.cumsum on a fragment must cover the whole fragment")
        sext = src.static_extents()
        if sext is None:
            raise LoweringError("T.cumsum needs static extents")
        dt = dst.buffer.dtype
        n_all = _prod(sext)
        ws = ctx.new_workspace(n_all, dt)

        def to_ws(r: BufferRegion):
            b = r.buffer
            if b.scope == "fragment":
                lay, lb = b.layout, ctx.local_of(b)
                return [S.StoreStmt(ws, [_row_major(lay.inverse(ctx.tid, i), sext)], cast(BufferLoad(lb, [IntImm(i)]),
                                                                                            dt))
                        for i in range(lay.local_size)]
            vars_ = [Var(f"cw{i}") for i in range(len(sext))]
            body = S.StoreStmt(ws, [_row_major(vars_, sext)],
                               cast(BufferLoad(b, [binop("+", m, v) for m, v in zip(r.mins, vars_)]), dt))
            for v, e in reversed(list(zip(vars_, sext))):
                body = S.ForStmt(v, 0, e, "parallel", body)
            return [self.lower_nest(body)]

        def from_ws(r: BufferRegion):
            b = r.buffer
            if b.scope == "fragment":
                lay, lb = b.layout, ctx.local_of(b)
                return [S.StoreStmt(lb, [IntImm(i)], cast(BufferLoad(ws, [_row_major(lay.inverse(ctx.tid, i), sext)]),
                                                          b.dtype))
                        for i in range(lay.local_size)]
            vars_ = [Var(f"cr{i}") for i in range(len(sext))]
            body = S.StoreStmt(b, [binop("+", m, v) for m, v in zip(r.mins, vars_)],
                               cast(BufferLoad(ws, [_row_major(vars_, sext)]), b.dtype))
            for v, e in reversed(list(zip(vars_, sext))):
                body = S.ForStmt(v, 0, e, "parallel", body)
            return [self.lower_nest(body)]

        out = [L.CallStmt("tl::sync_threads", [])] if ctx.self_sync else []
        out += to_ws(src)
        out.append(L.CallStmt("tl::sync_threads", []))
        dim = op.dim
        outer = [e for d, e in enumerate(sext) if d != dim]
        n_out = _prod(outer)
        n = sext[dim]
        steps = -(-n_out // ctx.T)
        for o in range(steps):
            slot = binop("+", o * ctx.T, ctx.tid)
            oidx = _unflatten(slot, outer)
            k = Var("ck")
            kk = binop("-", n - 1, k) if op.reverse else k
            idx = list(oidx)
            idx.insert(dim, kk)
            flat = _row_major(idx, sext)
            accb = ctx.new_local(f"cacc{ctx.ws_counter}", 1, dt)
            ctx.ws_counter += 1
            blk = S.SeqStmt([S.StoreStmt(accb, [IntImm(0)], const(0, dt)),
                             S.ForStmt(k, 0, n, "serial", S.SeqStmt([
                                 S.StoreStmt(accb, [IntImm(0)], BufferLoad(accb, [IntImm(0)]) + BufferLoad(ws, [flat])),
                                 S.StoreStmt(ws, [flat], BufferLoad(accb, [IntImm(0)]))]))])
            out.append(S.IfStmt(binop("<", slot, n_out), blk) if (o + 1) * ctx.T > n_out else blk)
        out.append(L.CallStmt("tl::sync_threads", []))
        out.extend(from_ws(dst))
        if ctx.self_sync:
            out.append(L.CallStmt("tl::sync_threads", []))
        return S.SeqStmt(out)

    def lower_AtomicOp(self, op: O.AtomicOp):
        dst = op.dst
        if op.return_prev:
            raise LoweringError("T.atomic_*(return_prev=True) returns one element's previous value: use the "
                                "element form (T.atomic_add(dst[i, j], v, return_prev=True)), not a tile")
        mo = {"memory_order": op.memory_order} if op.memory_order else {}
        if isinstance(op.src, BufferRegion):
            src = op.src
            staged = self.lower_atomic_staged(op, mo)
            if staged is not None:
                return staged
            nest = _copy_nest(src, dst, None, atomic=op.op, atomic_attrs=mo)
            lay = None
            if src.buffer.scope == "fragment":
                lay = _squeeze_fragment(src.buffer.layout, src.buffer.static_shape())
            return self.lower_nest(nest, lay)
        val = op.src
        nest = _region_nest(dst, lambda idx: None, atomic=(op.op, val), atomic_attrs=mo)
        return self.lower_nest(nest)

    # LDS budget of the row-contiguous staging of a fragment's f32 atomic adds
    ATOMIC_STAGE_BYTES = 96 * 1024

    def lower_atomic_staged(self, op: O.AtomicOp, mo):
        """``T.atomic_add(global_f32[...], fragment)``: the fragment goes through an LDS tile first so
        each wave instruction adds 64 consecutive floats of one row (256 contiguous bytes).  In the
        MFMA accumulator layout a wave instruction adds four 64-byte row pieces instead, and gfx950
        has no vector f32 atomic; global float atomics run at one chip-wide byte rate only when each
        instruction covers 256 contiguous bytes (cdna_hip_programming.md Guideline 12).  The LDS
        row pitch is padded by 4 floats so the accumulator layout's writes (lanes 16 apart are 4 rows
        apart) fall on disjoint bank halves.  None: the plain per-element lowering applies (other
        ops or dtypes, a thread-range partition, a tile over the budget, or the retry after an LDS
        plan that did not fit: target.no_atomic_stage)."""
        ctx, src, dst = self.ctx, op.src, op.dst
        if ctx.is_cpu or getattr(ctx.target, "no_atomic_stage", False) or op.op != "add" or \
                ctx.thread_range is not None or ctx.pass_cfg.get("tl.atomic_stage", True) is False:
            return None
        if src.buffer.scope != "fragment" or dst.buffer.scope != "global" or str(dst.buffer.dtype) != "float32":
            return None
        lay = getattr(src.buffer, "layout", None)
        sext = src.static_extents()
        if lay is None or sext is None or not _full(src) or len(sext) < 2 or sext[-1] < 64:
            return None
        sd, dd = _squeeze_pairs(src, dst)
        if len(sd) != len(sext):
            return None
        pitch = sext[-1] + 4 if sext[-1] % 8 == 0 else sext[-1]
        rows = _prod(sext[:-1])
        if rows * pitch * 4 > self.ATOMIC_STAGE_BYTES:
            return None
        ws = ctx.new_workspace(rows * pitch, "float32")

        def ws_at(idx):
            return binop("+", binop("*", _row_major(list(idx[:-1]), sext[:-1]), pitch), idx[-1])

        lb = ctx.local_of(src.buffer)
        out = [L.CallStmt("tl::sync_threads", [])] if ctx.self_sync else []
        out += [S.StoreStmt(ws, [ws_at(lay.inverse(ctx.tid, i))], cast(BufferLoad(lb, [IntImm(i)]), "float32"))
                for i in range(lay.local_size)]
        out.append(L.CallStmt("tl::sync_threads", []))
        vars_ = [Var(f"sa{i}") for i in range(len(sext))]
        didx = list(dst.mins)
        for v, d in zip(vars_, dd):
            didx[d] = binop("+", didx[d], v)
        body = S.EvaluateStmt(call("tl.atomic_add", [BufferLoad(dst.buffer, didx), BufferLoad(ws, [ws_at(vars_)])],
                                   dst.buffer.dtype, **mo))
        for v, e in reversed(list(zip(vars_, sext))):
            body = S.ForStmt(v, 0, e, "parallel", body, {"coalesced_width": 1})
        out.append(self.lower_nest(body))
        if ctx.self_sync:
            out.append(L.CallStmt("tl::sync_threads", []))
        return S.SeqStmt(out)

    def lower_FinalizeReducerOp(self, op):
        b = op.buf.buffer
        kind = getattr(b, "reducer_op", "sum")
        lay = b.layout
        # combine replicas: all-reduce over replication digits of the layout
        lane_mask, wave_digits = _replica_masks(lay)
        ctx = self.ctx
        lb = ctx.local_of(b)
        out = []
        opname = _REDUCE_OPS[kind][0]
        if lane_mask:
            for i in range(lb.shape[0]):
                out.append(S.StoreStmt(lb, [IntImm(i)], call("extern", ["tl::lane_allreduce<%s, %d>" % (opname,
                                                                                                       lane_mask),
                                                                         BufferLoad(lb, [IntImm(i)])], b.dtype)))
        if wave_digits and not ctx.is_cpu:
            # replicas in other waves: every thread publishes its (lane-combined) partials to an
            # LDS workspace ws[i][tid] and folds in its partner waves' copies
            n = lb.shape[0]
            ws = ctx.new_workspace(n * ctx.T, b.dtype)
            out.append(L.CallStmt("tl::sync_threads", []))
            for i in range(n):
                out.append(S.StoreStmt(ws, [binop("+", i * ctx.T, ctx.tid)], BufferLoad(lb, [IntImm(i)])))
            out.append(L.CallStmt("tl::sync_threads", []))
            partners = _partner_offsets(ctx.tid, wave_digits)
            for i in range(n):
                acc = None
                for p in partners:
                    x = BufferLoad(ws, [binop("+", i * ctx.T, p)])
                    acc = x if acc is None else _combine(kind, acc, x)
                out.append(S.StoreStmt(lb, [IntImm(i)], cast(acc, b.dtype)))
            if ctx.self_sync:
                out.append(L.CallStmt("tl::sync_threads", []))
        return S.SeqStmt(out)

    def lower_AsyncCopyOp(self, op: AsyncCopyOp):
        ctx = self.ctx
        p = op.plan
        if p.get("gather"):
            return self.lower_async_gather(op)
        if p.get("small"):
            return self.lower_async_small(op)
        src, dst = op.src, op.dst
        NB = dst.buffer
        lay = NB.layout
        epc = 16 // p["eb"]
        nw = p["nwaves"]
        wave = ctx.wave_expr()
        if p.get("dup"):
            wave = binop("%", wave, nw)  # waves past the tile re-fetch a covered piece
        lane = ctx.lane_expr()
        stage = self.expr(dst.mins[0])
        base_off = ctx.flat_index(NB, [stage, 0, 0])
        out = []
        smins = [self.expr(m) for m in src.mins]
        for i in range(p["instrs"]):
            chunk_base = binop("*", binop("+", i * nw, wave), 64)
            P = binop("+", chunk_base, lane)
            row = binop("//", P, p["cpr"])
            pch = binop("%", P, p["cpr"])
            if isinstance(lay, SwizzleLayout) and lay.bits:
                lch = binop("^", pch, lay._xor_term(row))
            else:
                lch = pch
            col = binop("*", lch, epc)
            idx = list(smins)
            if p["rdim"] is not None:
                idx[p["rdim"]] = binop("+", idx[p["rdim"]], row)
            idx[p["cdim"]] = binop("+", idx[p["cdim"]], col)
            gidx = ctx.flat_index(src.buffer, idx)
            lds_off = binop("+", base_off, binop("*", chunk_base, epc))
            if p.get("oob_bytes"):
                # ragged outer dim: buffer LDS-DMA, lanes past the tensor end write zeros
                rsrc = call("extern", ["tl::make_rsrc", L.BufferPtr(ctx.flat_of(src.buffer), 0),
                                       IntImm(p["oob_bytes"], _dt.uint32)], _dt.handle)
                voff = cast(binop("*", gidx, p["eb"]), _dt.uint32)
                out.append(L.CallStmt("tl::buffer_lds16", [rsrc, voff, L.BufferPtr(ctx.flat_of(NB), lds_off)]))
                continue
            out.append(L.CallStmt("tl::glds16", [L.BufferPtr(ctx.flat_of(src.buffer), gidx),
                                                 L.BufferPtr(ctx.flat_of(NB), lds_off)]))
        return S.SeqStmt(out)

    def lower_QuadGemmLoopOp(self, op):
        """``tl::gemm_quad_nt_x``: the whole 256x256x64 NT main loop (transform/pipeline.py
        _quad_schedule, tl/gemm_quad.h); the accumulators keep their GEMMs' register layouts."""
        ctx = self.ctx

        def ptr(r):
            return L.BufferPtr(ctx.flat_of(r.buffer), ctx.flat_index(r.buffer, [self.expr(m) for m in r.mins]))

        def i32(e):
            return cast(self.expr(convert(e)), _dt.int32)

        a, b = op.a.buffer, op.b.buffer
        gather = op.idx is not None or op.row_mode
        no_rows = call("extern", ["tl::quad::no_rows"], _dt.handle)
        if op.idx is not None:  # row gather: tensor base + the tile's row list
            mins = [IntImm(0)] + [self.expr(m) for m in op.a.mins[1:]]
            a_ptr = L.BufferPtr(ctx.flat_of(a), ctx.flat_index(a, mins))
            rows, row0, a_rows = ptr(op.idx), IntImm(0), i32(a.shape[0])
        elif op.row_mode:  # dense rows row0.. range-checked against the tensor
            mins = [IntImm(0)] + [self.expr(m) for m in op.a.mins[1:]]
            a_ptr = L.BufferPtr(ctx.flat_of(a), ctx.flat_index(a, mins))
            rows, row0, a_rows = no_rows, i32(op.a.mins[0]), i32(a.shape[0])
        else:
            a_ptr, rows, row0, a_rows = ptr(op.a), no_rows, IntImm(0), IntImm(0)
        cl = L.BufferPtr(ctx.local_of(op.C.buffer), 0)
        b_rm = getattr(op, "b_row_mode", False)
        k_len = getattr(op, "k_len", None)
        if b_rm:  # B rows n0.. range-checked against the tensor: tensor base + the tile's first row
            bmins = [IntImm(0)] + [self.expr(m) for m in op.b.mins[1:]]
            b_ptr, b_row0, b_rows = L.BufferPtr(ctx.flat_of(b), ctx.flat_index(b, bmins)), i32(op.b.mins[0]), \
                i32(b.shape[0])
        else:
            b_ptr, b_row0, b_rows = ptr(op.b), IntImm(0), IntImm(0)
        args = [a_ptr, i32(a.get_strides()[op.a_rdim]), rows, row0, a_rows, b_ptr, i32(b.get_strides()[op.b_rdim]),
                i32(op.n), L.BufferPtr(ctx.flat_of(op.lds_a), 0), L.BufferPtr(ctx.flat_of(op.lds_b), 0),
                L.BufferPtr(ctx.flat_of(op.lds_x if op.lds_x is not None else op.lds_a), 0), cl,
                L.BufferPtr(ctx.local_of(op.Cx.buffer), 0) if op.Cx is not None else cl,
                i32(op.m_limit) if op.m_limit is not None else IntImm(0x3fffffff), ctx.wave_expr()]
        targs = [_dt.hip_type(a.dtype), _b(gather), 32 if op.Cx is not None else 0]
        if b_rm or k_len is not None:  # ragged N / K (defaults otherwise: the aligned form's source)
            args += [b_row0, b_rows, IntImm(k_len if k_len is not None else 0)]
            targs += [_b(b_rm), _b(k_len is not None)]
        return S.SeqStmt([L.CallStmt("tl::gemm_quad_nt_x", args, targs)])

    def lower_async_small(self, op: AsyncCopyOp):
        """Small-tile DMA (pipeline._small_dma_plan): one 4-byte buffer LDS-DMA per wave; lane chunk
        ``P = wave * 64 + lane`` of the row-major tile, lanes past the tile (or the tensor) get an
        out-of-range offset and write a zero into the slot's padding."""
        ctx = self.ctx
        p = op.plan
        src, dst = op.src, op.dst
        NB = dst.buffer
        eb, cpr = p["eb"], p["cpr"]
        epc = max(1, 4 // eb)
        wave, lane = ctx.wave_expr(), ctx.lane_expr()
        stage = self.expr(dst.mins[0])
        base_off = ctx.flat_index(NB, [stage] + [IntImm(0)] * (NB.ndim - 1))
        P = binop("+", binop("*", wave, 64), lane)
        row = binop("//", P, cpr)
        col = binop("*", binop("%", P, cpr), epc)
        idx = [self.expr(m) for m in src.mins]
        if p["rdim"] is not None:
            idx[p["rdim"]] = binop("+", idx[p["rdim"]], row)
        idx[p["cdim"]] = binop("+", idx[p["cdim"]], col)
        gidx = ctx.flat_index(src.buffer, idx)
        rsrc = call("extern", ["tl::make_rsrc", L.BufferPtr(ctx.flat_of(src.buffer), 0),
                               IntImm(p["oob_bytes"], _dt.uint32)], _dt.handle)
        ok = binop("<", P, p["nchunks"])
        voff = select(ok, cast(binop("*", gidx, eb), _dt.uint32), IntImm(0xFFFFFFF0, _dt.uint32))
        lds_off = binop("+", base_off, binop("*", binop("*", wave, 64), epc if eb <= 4 else 1))
        return S.SeqStmt([L.CallStmt("tl::buffer_lds4", [rsrc, voff, L.BufferPtr(ctx.flat_of(NB), lds_off)])])

    def lower_async_gather(self, op: AsyncCopyOp):
        """Row gather as buffer LDS-DMA: each lane fetches the 16-byte chunk that lands at its
        lane-linear LDS slot, from the row named by the index tensor.  The resource is based at
        row 0 of the gathered dim (``num_records`` = whole dim), and invalid indices get an
        offset past ``num_records`` so the hardware writes zeros."""
        ctx = self.ctx
        p = op.plan
        src, dst = op.src, op.dst
        NB = dst.buffer
        lay = NB.layout
        epc = 16 // p["eb"]
        nw, cpr, rdim = p["nwaves"], p["cpr"], p["rdim"]
        wave, lane = ctx.wave_expr(), ctx.lane_expr()
        if p.get("dup"):
            wave = binop("%", wave, nw)  # waves past the tile re-fetch a covered chunk
        stage = self.expr(dst.mins[0])
        base_off = ctx.flat_index(NB, [stage, 0, 0])
        smins = [self.expr(m) for m in src.mins]
        smins[rdim] = IntImm(0)
        sb = src.buffer
        base = ctx.flat_index(sb, smins)
        stride_r = self.expr(convert(sb.get_strides()[rdim]))
        nrows = self.expr(convert(sb.shape[rdim]))
        rsrc = call("extern", ["tl::make_rsrc", L.BufferPtr(ctx.flat_of(sb), base),
                               cast(binop("*", binop("*", nrows, stride_r), p["eb"]), _dt.uint32)], _dt.handle)
        out = []
        regs = ctx.staging.get(("gidx", op.key)) if op.key is not None else None
        if op.key is not None and regs is None:
            raise LoweringError("gather DMA issued before its index prefetch")
        for i in range(p["instrs"]):
            chunk_base, row, pch = _gather_geom(i, nw, cpr, wave, lane)
            if isinstance(lay, SwizzleLayout) and lay.bits:
                lch = binop("^", pch, lay._xor_term(row))
            else:
                lch = pch
            if regs is not None:
                iv = BufferLoad(regs, [IntImm(i)])
            else:
                iv = self.expr(_gather_index(op.idx, row))
            # invalid rows (negative or past the tensor) clamp to row ``nrows`` as unsigned: their
            # offset is at or past num_records, so the hardware writes zeros -- one v_min_u32
            # instead of two compares, a select and the exec-mask juggling around the offset
            u32 = _dt.uint32
            iu = binop("min", cast(iv, u32), cast(nrows, u32))
            off = binop("*", binop("+", binop("*", iu, cast(stride_r, u32)), cast(binop("*", lch, epc), u32)),
                        IntImm(p["eb"], u32))
            voff = off
            lds_off = binop("+", base_off, binop("*", chunk_base, epc))
            out.append(L.CallStmt("tl::buffer_lds16", [rsrc, voff, L.BufferPtr(ctx.flat_of(NB), lds_off)]))
        return S.SeqStmt(out)

    def lower_GatherIndexOp(self, op: GatherIndexOp):
        ctx = self.ctx
        p = op.plan
        regs = ctx.staging.get(("gidx", op.key))
        if regs is None:
            regs = ctx.new_local(f"gidx{op.key}", p["instrs"], _dt.int32)
            ctx.staging[("gidx", op.key)] = regs
        wave, lane = ctx.wave_expr(), ctx.lane_expr()
        out = []
        for i in range(p["instrs"]):
            _, row, _ = _gather_geom(i, p["nwaves"], p["cpr"], binop("%", wave, p["nwaves"]) if p.get("dup") else wave,
                                     lane)
            # (kept in VGPRs: a scalar row base per instruction measured slower, 416 vs 531 TF
            # on sparse MLA -- the SALU address chains serialise the DMA issue)
            v = cast(self.expr(_gather_index(op.idx, row)), _dt.int32)
            out.append(S.StoreStmt(regs, [IntImm(i)], v))
        return S.SeqStmt(out)

    def lower_GatherRowsOp(self, op: O.GatherRowsOp):
        """Synchronous row gather (outside pipelined loops / CPU): a SIMT copy nest."""
        src, dst, rdim = op.src, op.dst, op.row_dim
        dd = [d for d, e in enumerate(dst.extents) if as_int(e) != 1]
        if len(dd) != 2:
            raise LoweringError("T.gather_rows destination must be a 2-D tile")
        cols = [d for d, e in enumerate(src.extents) if d != rdim and as_int(e) != 1]
        if len(cols) != 1:
            raise LoweringError("T.gather_rows source needs exactly one column dim besides row_dim")
        cdim = cols[0]
        r, c = Var("gr"), Var("gc")
        iv = _gather_index(op.idx, r)
        ok = logical_and(binop(">=", iv, 0), binop("<", iv, src.buffer.shape[rdim]))
        sidx = list(src.mins)
        sidx[rdim] = select(ok, iv, 0)
        sidx[cdim] = binop("+", sidx[cdim], c)
        didx = list(dst.mins)
        didx[dd[0]] = binop("+", didx[dd[0]], r)
        didx[dd[1]] = binop("+", didx[dd[1]], c)
        val = select(ok, cast(BufferLoad(src.buffer, sidx), dst.buffer.dtype), const(0, dst.buffer.dtype))
        body = S.StoreStmt(dst.buffer, didx, val)
        nest = S.ForStmt(r, 0, dst.extents[dd[0]], "parallel", S.ForStmt(c, 0, dst.extents[dd[1]], "parallel", body))
        return self.lower_nest(nest)

    def lower_StagedCopyOp(self, op: StagedCopyOp):
        """Register-staged copy: phase 'load' fills a staging array, 'store' writes it to LDS."""
        ctx = self.ctx
        steps = _simt_copy_steps(ctx, op.src, op.dst, self.known_div)
        nelem = sum(st["vec"] for st in steps)
        stage = ctx.staging.get(op.key)
        if stage is None:
            stage = ctx.new_local(f"stage{op.key}", max(1, nelem), op.src.buffer.dtype)
            ctx.staging[op.key] = stage
        out = []
        pos = 0
        for st in steps:
            vec = st["vec"]
            if op.phase == "load":
                sidx = [self.expr(i) for i in st["src_idx"]]
                sflat = ctx.flat_index(op.src.buffer, sidx)
                if st["guard"] is not None:
                    # out-of-range lanes load zeros (keeps the staging array defined)
                    zero = S.SeqStmt([S.StoreStmt(stage, [IntImm(pos + j)], const(0, stage.dtype))
                                      for j in range(vec)])
                    body = L.VecLoadStmt(stage, pos, ctx.flat_of(op.src.buffer), sflat, vec) if vec > 1 else \
                        S.StoreStmt(stage, [IntImm(pos)], BufferLoad(ctx.flat_of(op.src.buffer), [sflat]))
                    out.append(S.IfStmt(self.expr(st["guard"]), body, zero))
                else:
                    out.append(L.VecLoadStmt(stage, pos, ctx.flat_of(op.src.buffer), sflat, vec) if vec > 1 else
                               S.StoreStmt(stage, [IntImm(pos)], BufferLoad(ctx.flat_of(op.src.buffer), [sflat])))
            else:
                didx = [self.expr(i) for i in st["dst_idx"]]
                dflat = ctx.flat_index(op.dst.buffer, didx)
                vals = [cast(BufferLoad(stage, [IntImm(pos + j)]), op.dst.buffer.dtype) for j in range(vec)]
                s_ = L.VecStoreStmt(ctx.flat_of(op.dst.buffer), dflat, vals) if vec > 1 else \
                    S.StoreStmt(ctx.flat_of(op.dst.buffer), [dflat], vals[0])
                if st["dst_guard"] is not None:
                    s_ = S.IfStmt(self.expr(st["dst_guard"]), s_)
                out.append(s_)
            pos += vec
        return S.SeqStmt(out)

    def lower_CommBroadcastOp(self, op):
        from ..parallel.comm_lower import lower_comm
        return lower_comm(self, op)

    lower_CommPutOp = lower_CommBroadcastOp
    lower_CommAllGatherOp = lower_CommBroadcastOp
    lower_CommAllReduceOp = lower_CommBroadcastOp
    lower_CommBarrierOp = lower_CommBroadcastOp
    lower_CommFenceOp = lower_CommBroadcastOp

    def lower_Im2ColOp(self, op):
        """``T.c2d_im2col(img[N,H,W,C], col[bm, bk], nhw_step, c_step, K, S, D, P)``: gather one
        implicit-GEMM A tile (rows = output pixels, cols = (kh, kw, c)) with zero padding
        (reference src/op/copy.cc:1878 Conv2DIm2ColOpNode::Lower)."""
        img, col = op.img.buffer, op.col
        shp = img.static_shape()
        if shp is None or len(shp) != 4:
            raise LoweringError("T.c2d_im2col needs a static NHWC image tensor")
        _, H, W, C = shp
        KH = KW = int(op.kernel)
        Sd, Dd, Pd = int(op.stride), int(op.dilation), int(op.pad)
        OH = (H + 2 * Pd - Dd * (KH - 1) - 1) // Sd + 1
        OW = (W + 2 * Pd - Dd * (KW - 1) - 1) // Sd + 1
        ext = col.static_extents()
        if ext is None or len([e for e in ext if e != 1]) != 2:
            raise LoweringError("T.c2d_im2col destination must be a 2-D tile")
        bm, bk = [e for e in ext if e != 1]
        i, j = Var("ic_i"), Var("ic_j")
        m = binop("+", binop("*", op.nhw_step, bm), i)
        k = binop("+", binop("*", op.c_step, bk), j)
        n = binop("//", m, OH * OW)
        oh = binop("//", binop("%", m, OH * OW), OW)
        ow = binop("%", m, OW)
        h = binop("-", binop("+", binop("*", oh, Sd), binop("*", binop("//", k, KW * C), Dd)), Pd)
        w = binop("-", binop("+", binop("*", ow, Sd), binop("*", binop("%", binop("//", k, C), KW), Dd)), Pd)
        inb = logical_and(logical_and(binop(">=", h, 0), binop("<", h, H)),
                          logical_and(binop(">=", w, 0), binop("<", w, W)))
        # clamp the gather address so the load itself stays inside the image
        hc = binop("min", binop("max", h, 0), H - 1)
        wc = binop("min", binop("max", w, 0), W - 1)
        val = select(inb, BufferLoad(img, [n, hc, wc, binop("%", k, C)]), const(0, img.dtype))
        cidx = list(col.mins)
        nz = [d for d, e in enumerate(ext) if e != 1]
        cidx[nz[0]] = binop("+", cidx[nz[0]], i)
        cidx[nz[1]] = binop("+", cidx[nz[1]], j)
        body = S.StoreStmt(col.buffer, cidx, cast(val, col.buffer.dtype))
        nest = S.ForStmt(i, 0, bm, "parallel", S.ForStmt(j, 0, bk, "parallel", body))
        return self.lower_nest(nest)


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------


def ctx_is_cpu(ctx):
    return ctx.is_cpu


def _b(x):
    return "true" if x else "false"


def _scoped(s):
    s = S.SeqStmt([s]) if not isinstance(s, S.SeqStmt) else s
    s.scoped = True
    return s


def _nest_loops(outer: S.ForStmt) -> List[S.ForStmt]:
    loops = [outer]
    cur = outer
    while isinstance(cur.body, S.ForStmt) and cur.body.kind == "parallel":
        cur = cur.body
        loops.append(cur)
    return loops


def _unflatten(lin, exts):
    vals = []
    rem = lin
    for i, e in enumerate(reversed(exts)):
        if i == len(exts) - 1:
            vals.append(rem)
        else:
            vals.append(binop("%", rem, e))
            rem = binop("//", rem, e)
    return list(reversed(vals))


def _unflatten_dyn(lin, exts):
    return _unflatten(lin, exts)


def _slot_div(kd, tid, o, T, vec):
    return kd


def _full(r: BufferRegion) -> bool:
    ext = r.static_extents()
    shp = r.buffer.static_shape()
    return ext is not None and shp is not None and ext == shp and all(as_int(m) == 0 for m in r.mins)


def _squeeze_pairs(src: BufferRegion, dst: BufferRegion):
    se, de = src.extents, dst.extents
    sd = [d for d, e in enumerate(se) if as_int(e) != 1]
    dd = [d for d, e in enumerate(de) if as_int(e) != 1]
    sv = [as_int(se[d]) for d in sd]
    dv = [as_int(de[d]) for d in dd]
    if len(sd) != len(dd):
        raise LoweringError(f"T.copy: incompatible regions {src} -> {dst}")
    for a, b in zip(sv, dv):
        if a is not None and b is not None and a != b:
            raise LoweringError(f"T.copy: extent mismatch {src} -> {dst}")
    return sd, dd


def _gather_geom(i, nw, cpr, wave, lane):
    """(chunk base, tile row, physical chunk in the row) of LDS-DMA instruction ``i`` of a gather."""
    chunk_base = binop("*", binop("+", i * nw, wave), 64)
    if cpr % 64 == 0:
        row = binop("//", chunk_base, cpr)  # one row per wave instruction: uniform index
        pch = binop("+", binop("%", chunk_base, cpr), lane)
    else:
        row = binop("+", binop("//", chunk_base, cpr), binop("//", lane, cpr))
        pch = binop("%", lane, cpr)
    return chunk_base, row, pch


def _gather_index(idx: BufferRegion, row) -> PrimExpr:
    """``indices[row]`` for a 1-D index region (its single non-unit dim, else the last dim)."""
    nonunit = [d for d, e in enumerate(idx.extents) if as_int(e) != 1]
    d = nonunit[0] if nonunit else len(idx.extents) - 1
    ii = list(idx.mins)
    ii[d] = binop("+", ii[d], row)
    return BufferLoad(idx.buffer, ii)


def _copy_nest(src: BufferRegion, dst: BufferRegion, coalesced_width, atomic=None, atomic_attrs=None) -> S.ForStmt:
    sd, dd = _squeeze_pairs(src, dst)
    exts = [dst.extents[d] for d in dd] if dd else []
    vars_ = [Var(f"c{i}") for i in range(len(exts))]
    sidx = [m for m in src.mins]
    didx = [m for m in dst.mins]
    for v, s, d in zip(vars_, sd, dd):
        sidx[s] = binop("+", sidx[s], v)
        didx[d] = binop("+", didx[d], v)
    val = BufferLoad(src.buffer, sidx)
    if atomic is not None:
        body = S.EvaluateStmt(call(f"tl.atomic_{atomic}", [BufferLoad(dst.buffer, didx), val], dst.buffer.dtype,
                                   **(atomic_attrs or {})))
    else:
        body = S.StoreStmt(dst.buffer, didx, cast(val, dst.buffer.dtype))
    if not exts:
        vars_ = [Var("c0")]
        exts = [1]
    ann = {"coalesced_width": coalesced_width} if coalesced_width else {}
    for v, e in reversed(list(zip(vars_, exts))):
        body = S.ForStmt(v, 0, e, "parallel", body, ann)
    return body


def _region_nest(r: BufferRegion, mk, atomic=None, atomic_attrs=None) -> S.ForStmt:
    exts = list(r.extents)
    vars_ = [Var(f"f{i}") for i in range(len(exts))]
    idx = [binop("+", m, v) for m, v in zip(r.mins, vars_)]
    if atomic is not None:
        kind, val = atomic
        body = S.EvaluateStmt(call(f"tl.atomic_{kind}", [BufferLoad(r.buffer, idx), convert(val)], r.buffer.dtype,
                                   **(atomic_attrs or {})))
    else:
        b, _, val = mk(idx)
        body = S.StoreStmt(b, idx, val)
    for v, e in reversed(list(zip(vars_, exts))):
        body = S.ForStmt(v, 0, e, "parallel", body)
    return body


def _squeeze_fragment(lay: Fragment, shape) -> Fragment:
    """Drop unit dims of a fragment layout (so it matches a squeezed copy nest)."""
    keep = [d for d, s in enumerate(shape) if s != 1]
    if len(keep) == len(shape):
        return lay
    from ..layout.fragment import Digit
    remap = {old: new for new, old in enumerate(keep)}
    td = [Digit(remap[d.dim], d.stride, d.size) if d.dim >= 0 else d for d in lay.thread_digits]
    ld = [Digit(remap[d.dim], d.stride, d.size) for d in lay.local_digits]
    return Fragment([shape[d] for d in keep], td, ld, lay.name)


def _hoist_atomic_guard(n: Call):
    """An atomic used as a value (``T.atomic_load``, ``return_prev``) takes its first argument by
    address: a bounds-guarded element ``cond ? A[i] : 0`` becomes ``cond ? atomic(&A[i]) : 0``."""
    from ..ir.expr import Select
    if not (isinstance(n.op, str) and n.op.startswith("tl.atomic_") and n.args):
        return None
    a0 = n.args[0]
    if isinstance(a0, Select) and isinstance(a0.t, BufferLoad):
        inner = Call(n.op, [a0.t] + list(n.args[1:]), n.dtype, dict(n.attrs))
        return select(a0.cond, inner, const(0, n.dtype))
    return None


def _rewrite_atomic(rw, s: S.EvaluateStmt):
    """``tl.atomic_*(buf[idx], v)``: the destination is an address, never a guarded load --
    an out-of-bounds destination skips the whole atomic instead."""
    e = s.expr
    if not (isinstance(e, Call) and isinstance(e.op, str) and e.op.startswith("tl.atomic_") and e.args
            and isinstance(e.args[0], BufferLoad)):
        return None
    ld = e.args[0]
    b = ld.buffer
    if b.scope in ("fragment", "local", "var"):
        return None
    idx = [rw.expr(i) for i in ld.indices]
    dst = BufferLoad(rw.ctx.flat_of(b), [rw.ctx.flat_index(b, idx)])
    new = S.EvaluateStmt(Call(e.op, [dst] + [rw.expr(a) for a in e.args[1:]], e.dtype, dict(e.attrs)))
    g = safe_guard(rw.ctx, b, idx)
    return S.IfStmt(g, new) if g is not None else new


class _SimtRewriter(Mutator):

    def __init__(self, ctx, vmap):
        self.ctx = ctx
        self.vmap = vmap

    def visit_EvaluateStmt(self, s):
        r = _rewrite_atomic(self, s)
        return r if r is not None else S.EvaluateStmt(self.expr(s.expr))

    def _acc(self, n):
        if isinstance(n, BufferLoad):
            b = n.buffer
            idx = [substitute(i, self.vmap) for i in n.indices]
            if b.scope in ("local", "var"):
                return BufferLoad(b, [b.offset_of(idx)] if b.ndim != 1 else idx)
            if b.scope == "fragment":
                raise LoweringError(f"fragment {b.name} in a non-fragment T.Parallel nest")
            ld = BufferLoad(self.ctx.flat_of(b), [self.ctx.flat_index(b, idx)])
            g = safe_guard(self.ctx, b, idx)
            return select(g, ld, _safe_value(b)) if g is not None else ld
        if isinstance(n, Call):
            return _hoist_atomic_guard(n)
        return None

    def expr(self, e):
        if not isinstance(e, PrimExpr):
            return e
        return substitute(transform(e, self._acc), self.vmap)

    def store(self, s):
        b = s.buffer
        val = self.expr(s.value)
        idx = [self.expr(i) for i in s.indices]
        if b.scope in ("local", "var"):
            return S.StoreStmt(b, [b.offset_of(idx)] if b.ndim != 1 else idx, val)
        st = S.StoreStmt(self.ctx.flat_of(b), [self.ctx.flat_index(b, idx)], val)
        g = safe_guard(self.ctx, b, idx)
        return S.IfStmt(g, st) if g is not None else st


def _sample_threads(T):
    if T <= 256:
        return range(T)
    return list(range(0, T, 1))


def _thread_digit_weights(lay: Fragment):
    weights = []
    w = 1
    for d in reversed(lay.thread_digits):
        weights.append((d, w))
        w *= d.size
    return list(reversed(weights))


def _reduce_thread_masks(lay: Fragment, dim: int):
    lane_mask = 0
    wave_digits = []
    for d, w in _thread_digit_weights(lay):
        if d.dim != dim:
            continue
        if w * d.size <= 64:
            for b in range(int(math.log2(d.size))):
                lane_mask |= w << b
        elif w >= 64:
            wave_digits.append((d, w))
        elif 64 % w == 0 and d.size % (64 // w) == 0:
            # the digit straddles the wave boundary: its low part is reduced with lane
            # shuffles, its high part across waves through LDS
            lo = 64 // w
            for b in range(int(math.log2(lo))):
                lane_mask |= w << b
            wave_digits.append((Digit(d.dim, d.stride * lo, d.size // lo), 64))
        else:
            raise LoweringError("reduction digit straddles the wave boundary")
    return lane_mask, wave_digits


def _row_major(idx, shape) -> PrimExpr:
    acc = None
    for i, s in zip(idx, shape):
        acc = convert(i) if acc is None else binop("+", binop("*", acc, s), i)
    return acc if acc is not None else IntImm(0)


def _replica_masks(lay: Fragment):
    lane_mask = 0
    wave_digits = []
    for d, w in _thread_digit_weights(lay):
        if d.dim >= 0:
            continue
        if w * d.size <= 64:
            for b in range(int(math.log2(d.size))):
                lane_mask |= w << b
        else:
            wave_digits.append((d, w))
    return lane_mask, wave_digits


def _partner_offsets(tid, wave_digits):
    """Thread ids of all partners (including self) that differ only in the given digits."""
    exprs = [tid]
    for d, w in wave_digits:
        new = []
        for e in exprs:
            cur = binop("%", binop("//", e, w), d.size)
            for v in range(d.size):
                new.append(binop("+", e, binop("*", binop("-", v, cur), w)))
        exprs = new
    return exprs


def _simt_copy_steps(ctx: LowerCtx, src: BufferRegion, dst: BufferRegion, known_div) -> List[dict]:
    """Thread mapping of a plain copy: list of per-step {src_idx, dst_idx, vec, guard}."""
    if ctx.thread_range is not None:
        raise LoweringError("a register-staged copy inside a thread-range condition is not supported")
    sd, dd = _squeeze_pairs(src, dst)
    exts = [as_int(dst.extents[d]) for d in dd]
    if any(e is None for e in exts):
        raise LoweringError("register-staged copy needs static extents")
    total = _prod(exts) if exts else 1
    eb = max(src.buffer.dtype.bytes, dst.buffer.dtype.bytes)
    vec = 1 if ctx.no_vectorize else max(1, 16 // eb)
    while vec > 1:
        if exts and exts[-1] % vec == 0 and _copy_vec_ok(src, dst, sd, dd, vec, known_div):
            break
        vec //= 2
    slots = total // vec
    steps = -(-slots // ctx.T)
    out = []
    for o in range(steps):
        slot = binop("+", o * ctx.T, ctx.tid) if steps > 1 else ctx.tid
        lin = binop("*", slot, vec)
        vals = _unflatten(lin, exts) if exts else []
        sidx = list(src.mins)
        didx = list(dst.mins)
        for v, s, d in zip(vals, sd, dd):
            sidx[s] = binop("+", sidx[s], v)
            didx[d] = binop("+", didx[d], v)
        guard = binop("<", slot, slots) if (o + 1) * ctx.T > slots else None
        # source bounds (zero-fill) for ragged tiles
        sg = _bounds_guard(src, sidx, sd, vals, vec)
        g = guard if sg is None else (sg if guard is None else logical_and(guard, sg))
        dg = guard
        out.append(dict(src_idx=sidx, dst_idx=didx, vec=vec, guard=g, dst_guard=dg))
    return out


def _bounds_guard(r: BufferRegion, idx, dims, vals, vec):
    b = r.buffer
    if b.scope != "global":
        return None
    conds = None
    for d, i in enumerate(idx):
        s = b.shape[d]
        ext = r.extents[d]
        # skip dims provably in range
        c = binop("<", binop("+", i, vec - 1) if d == len(idx) - 1 else i, s)
        if as_int(c) == 1:
            continue
        conds = c if conds is None else logical_and(conds, c)
    return conds


def _copy_vec_ok(src, dst, sd, dd, vec, known_div) -> bool:
    for r, dims in ((src, sd), (dst, dd)):
        b = r.buffer
        if not dims:
            return False
        last = dims[-1]
        if last != len(r.region) - 1:
            return False
        if b.scope == "global":
            st = b.get_strides()
            if as_int(st[-1]) != 1:
                return False
            for s_ in st[:-1]:
                if not divisible_by(convert(s_), vec):
                    return False
        if not divisible_by(r.region[last][0], vec, known_div):
            return False
        if b.scope == "shared" and isinstance(b.layout, SwizzleLayout):
            if vec > b.layout.epc:
                return False
    return True


def _mesh_usage(kernel: S.KernelStmt):
    """(comm ops, uses T.comm.current_core) of a kernel, before lowering."""
    comm = [s.op for s in S.walk(kernel) if isinstance(s, S.TileOpStmt) and isinstance(s.op, O.CommOp)]
    found = []

    class _F(Mutator):

        def expr(self, e):
            if isinstance(e, PrimExpr) and not found:
                for n in post_order(e):
                    if isinstance(n, Call) and n.op == "tl.mesh_rank":
                        found.append(n)
                        break
            return e

    _F().stmt(kernel.body)
    return comm, bool(found)


def lower_tile_ops(kernel: S.KernelStmt, target, pass_cfg=None):
    ctx = LowerCtx(kernel, target, pass_cfg)
    comm_ops, uses_rank = _mesh_usage(kernel)
    ctx.mesh = None
    if comm_ops or uses_rank:
        from ..parallel import comm_lower
        ctx.mesh_slot_bytes = max([comm_lower.op_slot_bytes(o) for o in comm_ops] or [256])
        shapes = {tuple(o.mesh) for o in comm_ops if o.mesh is not None}
        if len(shapes) > 1:
            raise LoweringError(f"T.comm ops of one kernel were traced for different mesh shapes: {sorted(shapes)}")
        comm_lower.mesh_state(ctx, shapes.pop() if shapes else None)
    lw = TileOpLowerer(ctx)
    body = lw.stmt(kernel.body)
    allocs = [S.AllocStmt(b) for b in ctx.extra_allocs]
    if ctx.mesh is not None:
        allocs = allocs + ctx.mesh.prologue()
    k = S.KernelStmt(kernel.grid, kernel.threads, kernel.block_vars, kernel.thread_vars,
                     S.SeqStmt(allocs + [body]), kernel.is_cpu, kernel.prelude)
    k.attrs = dict(kernel.attrs)
    k.attrs["narrow_index"] = {b.name for b in ctx.narrow_index}
    k.attrs["cooperative"] = ctx.uses_grid_sync
    if ctx.uses_grid_sync and not kernel.is_cpu:
        # per-launch barrier state + the device error word (tl/common.h sync_grid, runtime/errors.py)
        from ..ir.expr import Var as _Var
        k.attrs["extra_params"] = list(k.attrs.get("extra_params", [])) + [
            dict(kind="extra", name="tl_gsync_ws", var=_Var("tl_gsync_ws", "int64"), ctype="long long", nbytes=8,
                 runtime="gsync"),
            dict(kind="extra", name="tl_dev_err", var=_Var("tl_dev_err", "int64"), ctype="long long", nbytes=8,
                 runtime="err")]
    if ctx.mesh is not None:
        k.attrs["extra_params"] = list(k.attrs.get("extra_params", [])) + ctx.mesh.extra_params()
        k.attrs["mesh"] = ctx.mesh.meta()
        k.attrs["mesh_rank_var"] = ctx.mesh.rank
    k.attrs["tid"] = ctx.tid
    k.attrs["lane"] = ctx.lane if ctx.uses_lane else None
    k.attrs["wave"] = ctx.wave if ctx.uses_wave else None
    k.attrs["flat"] = ctx.flat
    return k, ctx
