"""Layout inference: assign a Fragment to every ``local.fragment`` buffer and a
(swizzled) Layout to every shared operand buffer.

Reference: ``src/transform/layout_inference.cc`` (strict -> common -> free
levels, BFS propagation, ``LayoutConflictException``) and each op's
``InferLayout``.  Here:

* **strict**  — ``T.gemm`` accumulators get the CDNA4 MFMA C layout, register A
  operands an MFMA A layout (k-permuted when it comes from an accumulator), shared
  operands a bank-model-chosen swizzle; user ``T.annotate_layout`` wins.
* **common**  — propagate through reductions (row projections with replication),
  fragment->fragment copies/casts, and ``T.Parallel`` nests (an anchor fragment
  indexed by exactly the loop variables fixes the loop's thread partition;
  other fragments in the nest are projected/permuted from it).
* **free**    — fragments still unconstrained get a vectorised linear layout.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import Var, as_int, loads_of
from ..layout.fragment import Digit, Fragment, make_linear_fragment, make_replicated_fragment
from ..layout.layout import LinearLayout
from ..layout import mfma as MF


class LayoutConflictError(Exception):
    pass


def _frag_view_base(b: Buffer):
    """The fragment a ``T.reshape`` / ``T.view`` buffer aliases (None for other buffers)."""
    a = getattr(b, "alias_of", None)
    if b.scope == "fragment" and a is not None and a[0].scope == "fragment":
        return a[0]
    return None


def _is_frag(b: Buffer) -> bool:
    return b.scope == "fragment"


def _full_region(r: BufferRegion) -> bool:
    ext = r.static_extents()
    shp = r.buffer.static_shape()
    if ext is None or shp is None:
        return False
    # allow leading unit dims on the buffer side
    return all(as_int(m) == 0 for m in r.mins) and ext == shp


class ParallelNest:
    """A maximal nest of T.Parallel loops."""

    def __init__(self, loops: List[S.ForStmt]):
        self.loops = loops
        self.vars = [l.var for l in loops]
        self.extents = [as_int(l.extent) for l in loops]
        self.mins = [l.min for l in loops]
        self.body = loops[-1].body
        self.layout: Optional[Fragment] = None
        self.outer = loops[0]

    @property
    def static(self) -> bool:
        return all(e is not None for e in self.extents)

    def accesses(self):
        """(buffer, indices, is_store) for every access in the body."""
        out = []
        for s in S.walk(self.body):
            if isinstance(s, S.StoreStmt):
                out.append((s.buffer, s.indices, True))
                for e in [s.value] + list(s.indices):
                    for ld in loads_of(e):
                        out.append((ld.buffer, ld.indices, False))
            elif isinstance(s, (S.LetStmt, )):
                for ld in loads_of(s.value):
                    out.append((ld.buffer, ld.indices, False))
            elif isinstance(s, S.IfStmt):
                for ld in loads_of(s.cond):
                    out.append((ld.buffer, ld.indices, False))
            elif isinstance(s, S.EvaluateStmt):
                for ld in loads_of(s.expr):
                    out.append((ld.buffer, ld.indices, False))
        return out

    def fragment_accesses(self):
        return [(b, idx, st) for b, idx, st in self.accesses() if _is_frag(b)]


def collect_nests(body: S.Stmt) -> List[ParallelNest]:
    nests = []

    def visit(s, inside):
        if isinstance(s, S.ForStmt) and s.kind == "parallel" and not inside:
            loops = [s]
            cur = s
            while isinstance(cur.body, S.ForStmt) and cur.body.kind == "parallel":
                cur = cur.body
                loops.append(cur)
            nests.append(ParallelNest(loops))
            # nested non-perfect parallel loops inside the body are part of this nest's body
            return
        for c in S.stmt_children(s):
            visit(c, inside)

    visit(body, False)
    return nests


def _index_map(indices, loop_vars) -> Optional[List[Optional[int]]]:
    """If every index is exactly a loop var (or a constant 0 on a unit dim), return for
    each buffer dim the loop-dim it maps to (None for constant dims)."""
    out = []
    for e in indices:
        if isinstance(e, Var):
            try:
                out.append([v is e for v in loop_vars].index(True))
            except ValueError:
                return None
        elif as_int(e) is not None:
            out.append(None)
        else:
            return None
    return out


def _is_flat_index(indices, loop_vars, loop_shape, buf_shape) -> bool:
    """True when a buffer of the loop domain's size is indexed by the row-major flattening of the
    loop vars (``B[i * bn + j]`` in ``T.Parallel(bm, bn)``, the reference's composable index):
    its layout is then the nest's, reshaped (Fragment.reshape)."""
    import random
    from ..ir.expr import EvalError, evaluate
    n_loop, n_buf = 1, 1
    for e in loop_shape:
        n_loop *= int(e)
    for e in buf_shape or [0]:
        n_buf *= int(e)
    if n_loop != n_buf or len(indices) != 1 or len(buf_shape) != 1:
        return False
    rnd = random.Random(11)
    for _ in range(8):
        env = {v: rnd.randrange(int(e)) for v, e in zip(loop_vars, loop_shape)}
        flat = 0
        for v, e in zip(loop_vars, loop_shape):
            flat = flat * int(e) + env[v]
        try:
            if int(evaluate(indices[0], env)) != flat:
                return False
        except (EvalError, TypeError, KeyError):
            return False
    return True


def project_layout(loop_layout: Fragment, dim_map: List[Optional[int]], buf_shape: List[int]) -> Fragment:
    """Layout of a buffer accessed as ``buf[loop_vars[dim_map[0]], ...]`` inside a nest
    partitioned by ``loop_layout`` (loop dims not used by the buffer become replication)."""
    used = {ld: bd for bd, ld in enumerate(dim_map) if ld is not None}
    td = []
    for d in loop_layout.thread_digits:
        if d.dim >= 0 and d.dim in used:
            td.append(Digit(used[d.dim], d.stride, d.size))
        else:
            td.append(Digit(-1, 1, d.size))
    ld_ = [Digit(used[d.dim], d.stride, d.size) for d in loop_layout.local_digits if d.dim in used]
    # merge adjacent replication digits
    merged = []
    for d in td:
        if merged and d.dim < 0 and merged[-1].dim < 0:
            merged[-1] = Digit(-1, 1, merged[-1].size * d.size)
        else:
            merged.append(d)
    return Fragment(buf_shape, merged, ld_, loop_layout.name + "_proj")


def lift_layout(buf_layout: Fragment, dim_map: List[Optional[int]], loop_shape: List[int]) -> Optional[Fragment]:
    """Loop partition induced by an anchor buffer accessed with ``dim_map``.

    Only valid when the buffer covers every loop dim (a permutation)."""
    if sorted(d for d in dim_map if d is not None) != list(range(len(loop_shape))):
        return None
    inv = {bd: ld for bd, ld in enumerate(dim_map) if ld is not None}
    td = [Digit(inv[d.dim], d.stride, d.size) if d.dim >= 0 else d for d in buf_layout.thread_digits]
    ld_ = [Digit(inv[d.dim], d.stride, d.size) for d in buf_layout.local_digits]
    try:
        return Fragment(loop_shape, td, ld_, buf_layout.name + "_loop")
    except ValueError:
        return None


def extend_layout(buf_layout: Fragment, dim_map: List[Optional[int]], loop_shape: List[int],
                  vec: int = 4) -> Optional[Fragment]:
    """Loop partition for a nest whose only laid-out fragment covers a *subset* of the loop
    dims (e.g. ``x[i, j] * row_scale[i]``): keep the buffer's placement of its dims, spread
    the missing loop dims over the buffer's replication threads (lane-fastest) and registers
    (innermost ``vec`` elements contiguous), so every thread owns what it iterates."""
    used = {ld: bd for bd, ld in enumerate(dim_map) if ld is not None}
    if len(used) != len([d for d in dim_map if d is not None]):
        return None
    missing = [ld for ld in range(len(loop_shape)) if ld not in used and loop_shape[ld] > 1]
    td = []
    for d in buf_layout.thread_digits:
        if d.dim < 0:
            td.append(["rep", d.size])
        else:
            td.append(Digit(dim_map[d.dim], d.stride, d.size))
    ld_ = [Digit(dim_map[d.dim], d.stride, d.size) for d in buf_layout.local_digits]
    import math as _m
    tail_local = []
    for md in reversed(missing):
        E = loop_shape[md]
        stride = 1
        v = _m.gcd(E, max(1, vec)) if md == len(loop_shape) - 1 else 1
        if v > 1:
            tail_local.insert(0, Digit(md, 1, v))
            stride = v
        rem = E // v
        # fill replication thread digits, least significant first
        for k in range(len(td) - 1, -1, -1):
            if rem == 1:
                break
            ent = td[k]
            if isinstance(ent, list):
                t = _m.gcd(ent[1], rem)
                if t > 1:
                    new = []
                    if ent[1] // t > 1:
                        new.append(["rep", ent[1] // t])
                    new.append(Digit(md, stride, t))
                    td[k:k + 1] = new
                    stride *= t
                    rem //= t
        if rem > 1:
            ld_.insert(0, Digit(md, stride, rem))
    thread = [Digit(-1, 1, e[1]) if isinstance(e, list) else e for e in td]
    try:
        return Fragment(loop_shape, thread, ld_ + tail_local, buf_layout.name + "_ext")
    except ValueError:
        return None


def reduce_dst_layout(src: Fragment, dim: int, dst_shape: List[int]) -> Fragment:
    """Layout of reduce(src, dim): the reduced dim's digits become replication (threads)
    or disappear (registers)."""
    keep = [d for d in range(len(src.shape)) if d != dim]
    remap = {old: new for new, old in enumerate(keep)}
    td = [Digit(remap[d.dim], d.stride, d.size) if (d.dim >= 0 and d.dim != dim) else Digit(-1, 1, d.size)
          for d in src.thread_digits]
    merged = []
    for d in td:
        if merged and d.dim < 0 and merged[-1].dim < 0:
            merged[-1] = Digit(-1, 1, merged[-1].size * d.size)
        else:
            merged.append(d)
    ld_ = [Digit(remap[d.dim], d.stride, d.size) for d in src.local_digits if d.dim != dim]
    shape = [src.shape[d] for d in keep]
    if len(dst_shape) != len(shape):
        # dst keeps a unit dim in place of the reduced one
        if len(dst_shape) == len(src.shape) and dst_shape[dim] == 1:
            td2 = [Digit(d.dim + (1 if d.dim >= dim else 0), d.stride, d.size) if d.dim >= 0 else d
                   for d in merged]
            ld2 = [Digit(d.dim + (1 if d.dim >= dim else 0), d.stride, d.size) for d in ld_]
            return Fragment(dst_shape, td2, ld2, src.name + "_red")
        raise LayoutConflictError(f"reduce output shape {dst_shape} incompatible with {src.shape} along dim {dim}")
    return Fragment(shape, merged, ld_, src.name + "_red")


class LayoutInference:

    def __init__(self, func: S.PrimFunc, num_threads: int, target=None):
        self.func = func
        self.T = num_threads
        self.target = target
        self.frag: Dict[Buffer, Fragment] = {}
        self.strict: set = set()
        self.gemm_info: Dict[int, dict] = {}
        self.nest_layouts: Dict[int, Fragment] = {}
        self.smem_reads: Dict[Buffer, dict] = {}

    # ------------------------------------------------------------------------------
    def set_frag(self, buf: Buffer, lay: Fragment, why: str, strict: bool = False):
        if _frag_view_base(buf) is not None:
            return False  # a reshaped view of a fragment: its layout follows the base's
        old = self.frag.get(buf)
        if old is not None:
            if old.is_equal(lay):
                return False
            if buf in self.strict and not strict:
                raise LayoutConflictError(f"layout conflict on fragment {buf.name}: {old} vs {lay} ({why})")
            if strict and buf in self.strict:
                raise LayoutConflictError(f"two strict layouts for fragment {buf.name} ({why}): {old} vs {lay}")
        if lay.num_threads != self.T:
            if lay.num_threads < self.T and self.T % lay.num_threads == 0:
                lay = lay.replicate(self.T // lay.num_threads)
            else:
                raise LayoutConflictError(f"{buf.name}: layout over {lay.num_threads} threads, block has {self.T}")
        self.frag[buf] = lay
        if strict:
            self.strict.add(buf)
        return True

    def run(self):
        body = self.func.body
        kernel = [s for s in S.walk(body) if isinstance(s, S.KernelStmt)]
        if not kernel:
            return {}
        kernel = kernel[0]
        # layouts are per-compilation results: forget those of an earlier lowering of the same
        # PrimFunc (e.g. for another target); only user annotations persist
        for s in S.walk(kernel):
            if isinstance(s, S.AllocStmt) and not getattr(s.buffer, "layout_annotated", False):
                if s.buffer.scope in ("fragment", "shared"):
                    s.buffer.layout = None
        frags = [s.buffer for s in S.walk(kernel) if isinstance(s, S.AllocStmt) and _is_frag(s.buffer)]
        for b in frags:
            if getattr(b, "layout_annotated", False) and isinstance(b.layout, Fragment):
                self.set_frag(b, b.layout, "annotate_layout", strict=True)
        ops = [s.op for s in S.walk(kernel) if isinstance(s, S.TileOpStmt)]
        nests = collect_nests(kernel)
        self.nests = nests

        # strict: gemm
        for op in ops:
            if isinstance(op, O.GemmOp):
                self.infer_gemm(op, level="strict")
        # common: propagate to fixpoint
        for _ in range(32):
            changed = False
            for op in ops:
                changed |= self.infer_op(op)
            for n in nests:
                changed |= self.infer_nest(n, free=False)
            for op in ops:
                if isinstance(op, O.GemmOp):
                    changed |= self.infer_gemm(op, level="common")
            if not changed:
                break
        # free: unconstrained fragments in nests/copies get default layouts.  Larger iteration
        # domains choose first (the reference's per-component root search): a 2-D tile nest
        # fixes the partition its 1-D row statistics then inherit, not the other way round.
        def _domain(n):
            sz = 1
            for e in n.extents:
                sz *= e if e is not None else 1
            return -sz
        free_order = sorted(nests, key=_domain)
        for _ in range(64):
            changed = False
            for n in free_order:
                changed |= self.infer_nest(n, free=True)
                if changed:
                    break
            if not changed:
                for b in frags:
                    if b not in self.frag:
                        self.set_frag(b, self.default_fragment(b), "free")
                        changed = True
                        break
            if changed:
                for _ in range(32):
                    c2 = False
                    for op in ops:
                        c2 |= self.infer_op(op)
                    for n in nests:
                        c2 |= self.infer_nest(n, free=False)
                    if not c2:
                        break
            else:
                break
        # final gemm plans (register-A k-permutation is known now) -> shared operand swizzles
        self.smem_reads = {}
        for op in ops:
            if isinstance(op, O.GemmOp):
                self.infer_gemm(op, level="final")
        self.assign_shared_layouts()
        for b, lay in self.frag.items():
            b.layout = lay
        # views of fragments (T.reshape / T.view): the base's layout over the view's shape
        for op in ops:
            for r in op.regions():
                base = _frag_view_base(r.buffer)
                if base is not None and isinstance(base.layout, Fragment):
                    r.buffer.layout = base.layout.reshape(r.buffer.static_shape())
        for n in nests:
            if n.layout is not None:
                n.outer.annotations["_layout"] = n.layout
        return self.frag

    # ------------------------------------------------------------------------------
    def default_fragment(self, b: Buffer) -> Fragment:
        shape = b.static_shape()
        if shape is None:
            raise LayoutConflictError(f"fragment {b.name} needs a static shape")
        vec = max(1, 16 // b.dtype.bytes)
        try:
            return make_linear_fragment(shape, self.T, vec, name=f"linear_{b.name}")
        except ValueError:
            return make_replicated_fragment(shape, self.T)

    def infer_gemm(self, op: O.GemmOp, level: str) -> bool:
        from .gemm_lower import gemm_plan
        changed = False
        A = op.A.buffer
        plan = gemm_plan(op, self.T, self.target, self.frag.get(A) if _is_frag(A) else None)
        self.gemm_info[id(op)] = plan
        op.plan = plan
        C = op.C.buffer
        if _is_frag(C) and level == "strict":
            changed |= self.set_frag(C, plan["c_layout"], "gemm C", strict=True)
        if _is_frag(A) and plan.get("mfma") is None:
            if A not in self.frag and level == "common":
                changed |= self.set_frag(A, self.default_fragment(A), "cpu gemm A")
        elif _is_frag(A):
            lay_cur = self.frag.get(A)
            mn = tuple(plan["mfma"][:2]) if plan["mfma"][:2] == (32, 32) else (16, 16)
            k0 = MF.mfma_a_fragment(plan["M"], plan["K"], plan["warp_m"], plan["warp_n"], 0, mn, op.trans_A)
            k1 = MF.mfma_a_fragment(plan["M"], plan["K"], plan["warp_m"], plan["warp_n"], 1, mn, op.trans_A)
            if lay_cur is not None:
                if lay_cur.is_equal(k1) or _equal_rep(lay_cur, k1, self.T):
                    plan["a_kperm"] = 1
                elif lay_cur.is_equal(k0) or _equal_rep(lay_cur, k0, self.T):
                    plan["a_kperm"] = 0
                else:
                    raise LayoutConflictError(
                        f"T.gemm: register A operand {A.name} has layout {lay_cur}, which is not an MFMA A "
                        f"layout for warp partition {plan['warp_m']}x{plan['warp_n']}; use "
                        f"policy=T.GemmWarpPolicy.FullRow on the GEMM producing it")
            elif level == "common":
                # prefer the layout that matches an accumulator source (checked later), else natural
                changed |= self.set_frag(A, k0, "gemm A", strict=True)
                plan["a_kperm"] = 0
        for reg, role in ((op.A, "a"), (op.B, "b")):
            b = reg.buffer
            if b.scope == "shared" and plan.get(f"{role}_kind"):
                self.smem_reads.setdefault(b, {})[(id(op), role)] = plan[f"{role}_kind"]
        return changed

    def assign_shared_layouts(self):
        """One swizzle per shared operand tile, chosen against ALL its MFMA read patterns."""
        for b, kinds in self.smem_reads.items():
            if getattr(b, "layout_annotated", False):
                continue
            shp = b.static_shape()
            if len(shp) != 2:
                b.layout = LinearLayout(shp)
                continue
            eb = b.dtype.bytes
            if eb not in (1, 2):
                b.layout = LinearLayout(shp)
                continue
            b.layout = MF.operand_swizzle_multi(tuple(kinds.values()), shp, eb)

    def infer_op(self, op) -> bool:
        changed = False
        if isinstance(op, O.ReduceOp):
            s, d = op.src.buffer, op.dst.buffer
            if _is_frag(s) and _is_frag(d) and s in self.frag and d not in self.frag:
                if not _full_region(op.src):
                    raise LayoutConflictError("T.reduce on a fragment must cover the whole fragment")
                lay = reduce_dst_layout(self.frag[s], op.dim, d.static_shape())
                changed |= self.set_frag(d, lay, "reduce")
        elif isinstance(op, O.CopyOp):
            s, d = op.src.buffer, op.dst.buffer
            if _is_frag(s) and _is_frag(d) and _full_region(op.src) and _full_region(op.dst):
                if s in self.frag and d not in self.frag:
                    changed |= self.set_frag(d, self.frag[s], "copy")
                elif d in self.frag and s not in self.frag:
                    changed |= self.set_frag(s, self.frag[d], "copy")
        elif isinstance(op, O.CumSumOp):
            pass
        elif isinstance(op, O.CommAllReduceOp) and op.dim is None:
            s, d = op.src.buffer, op.dst.buffer
            if _is_frag(s) and _is_frag(d):
                if s in self.frag and d not in self.frag:
                    changed |= self.set_frag(d, self.frag[s], "comm all_reduce_tile")
                elif d in self.frag and s not in self.frag:
                    changed |= self.set_frag(s, self.frag[d], "comm all_reduce_tile")
        elif isinstance(op, O.CommAllReduceOp) and op.tmp is not None:
            # partial = reduce(src, dim) gets the reduce layout; out follows the partial
            s, t, d = op.src.buffer, op.tmp.buffer, op.dst.buffer
            if _is_frag(s) and _is_frag(t) and s in self.frag and t not in self.frag:
                if not _full_region(op.src):
                    raise LayoutConflictError("T.comm.all_reduce on a fragment must cover the whole fragment")
                changed |= self.set_frag(t, reduce_dst_layout(self.frag[s], op.dim, t.static_shape()), "comm reduce")
            if _is_frag(t) and _is_frag(d) and t in self.frag and d not in self.frag:
                changed |= self.set_frag(d, self.frag[t], "comm all_reduce out")
        elif isinstance(op, O.CommAllGatherOp):
            # recv[k] is laid out like send: each thread holds slice k of the elements it sends
            s, r = op.send.buffer, op.recv.buffer
            if _is_frag(s) and _is_frag(r) and s in self.frag and r not in self.frag and _full_region(op.send):
                sl = self.frag[s]
                G = r.static_shape()[0]
                td = [Digit(d.dim + 1, d.stride, d.size) if d.dim >= 0 else d for d in sl.thread_digits]
                ld = [Digit(0, 1, G)] + [Digit(d.dim + 1, d.stride, d.size) for d in sl.local_digits]
                changed |= self.set_frag(r, Fragment([G] + list(sl.shape), td, ld, sl.name + "_gather"), "all_gather")
        elif isinstance(op, (O.CommBroadcastOp, O.CommPutOp)):
            s, d = op.src.buffer, op.dst.buffer
            if _is_frag(s) and _is_frag(d) and _full_region(op.src) and _full_region(op.dst) and \
                    s.static_shape() == d.static_shape():
                if s in self.frag and d not in self.frag:
                    changed |= self.set_frag(d, self.frag[s], "comm")
                elif d in self.frag and s not in self.frag:
                    changed |= self.set_frag(s, self.frag[d], "comm")
        return changed

    def infer_nest(self, n: ParallelNest, free: bool) -> bool:
        if not n.static:
            if n.fragment_accesses():
                raise LayoutConflictError("T.Parallel over fragments needs static extents")
            return False
        shape = n.extents
        changed = False
        if n.layout is None:
            # find an anchor
            for b, idx, _ in n.fragment_accesses():
                if b in self.frag:
                    dm = _index_map(idx, n.vars)
                    if dm is None:
                        if _is_flat_index(idx, n.vars, shape, b.static_shape()) and all(as_int(m) == 0 for m in n.mins):
                            try:
                                n.layout = self.frag[b].reshape(shape)
                                changed = True
                                break
                            except ValueError:
                                pass
                        continue
                    lifted = lift_layout(self.frag[b], dm, shape)
                    if lifted is not None and all(as_int(m) == 0 for m in n.mins):
                        n.layout = lifted
                        changed = True
                        break
            if n.layout is None and free and n.fragment_accesses():
                # a laid-out fragment covering part of the loop dims: extend its partition
                eb = max(b.dtype.bytes for b, _, _ in n.fragment_accesses())
                for b, idx, _ in n.fragment_accesses():
                    if b in self.frag and all(as_int(m) == 0 for m in n.mins):
                        dm = _index_map(idx, n.vars)
                        if dm is None:
                            continue
                        ext = extend_layout(self.frag[b], dm, shape, max(1, 16 // eb))
                        if ext is not None and ext.num_threads == self.T:
                            n.layout = ext
                            changed = True
                            break
            if n.layout is None and free and n.fragment_accesses():
                # choose a default partition for the nest
                unknown = [b for b, _, _ in n.fragment_accesses() if b not in self.frag]
                if unknown:
                    eb = max(b.dtype.bytes for b, _, _ in n.fragment_accesses())
                    vec = max(1, 16 // eb)
                    try:
                        n.layout = make_linear_fragment(shape, self.T, vec, name="loop")
                    except ValueError:
                        n.layout = make_linear_fragment(shape, self.T, 1, name="loop")
                    changed = True
        if n.layout is not None:
            for b, idx, _ in n.fragment_accesses():
                if b in self.frag:
                    continue
                dm = _index_map(idx, n.vars)
                bshape = b.static_shape()
                if dm is None:
                    if _is_flat_index(idx, n.vars, shape, bshape) and all(as_int(m) == 0 for m in n.mins):
                        try:
                            changed |= self.set_frag(b, n.layout.reshape(bshape), "parallel (flattened index)")
                        except ValueError:
                            pass
                    continue
                try:
                    lay = project_layout(n.layout, dm, bshape)
                except ValueError:
                    continue  # the nest covers only part of b (constant index); b is laid out elsewhere
                changed |= self.set_frag(b, lay, "parallel")
        return changed


def _same_layout(a, b) -> bool:
    try:
        return a.signature() == b.signature()
    except Exception:  # noqa: BLE001
        return a is b


def _equal_rep(a: Fragment, b: Fragment, T: int) -> bool:
    if b.num_threads < T and T % b.num_threads == 0:
        b = b.replicate(T // b.num_threads)
    if a.num_threads < T and T % a.num_threads == 0:
        a = a.replicate(T // a.num_threads)
    return a.is_equal(b)


def infer_layouts(func: S.PrimFunc, num_threads: int, target=None) -> LayoutInference:
    li = LayoutInference(func, num_threads, target)
    li.run()
    li.shared_buffers = [s.buffer for s in S.walk(func.body)
                         if isinstance(s, S.AllocStmt) and s.buffer.scope == "shared"]
    return li
