"""Insert block barriers for LDS (shared memory) hazards.

Reference: ``src/transform/thread_storage_sync.cc`` + ``storage_access.cc``
(``ThreadSync("shared")``).  Runs on the lowered per-thread IR: a linear scan
tracks buffers written/read since the last barrier and inserts
``__syncthreads()`` before a RAW/WAR/WAW conflict; loops are scanned twice for
loop-carried hazards; barriers are never placed inside divergent ``if`` bodies
(they are hoisted in front of the ``if``).  Accesses that the software pipeline
manages itself (multi-versioned stage buffers inside a pipelined loop) are
skipped: that loop already carries one raw ``s_barrier`` per iteration and a
``__syncthreads()`` there would drain the in-flight LDS-DMA (``vmcnt(0)``).
"""
from __future__ import annotations

from typing import List, Set, Tuple

from ..ir import stmt as S
from ..ir import lowered as L
from ..ir.buffer import Buffer
from ..ir.expr import BufferLoad, PrimExpr, post_order

_BARRIERS = {"tl::sync_threads", "tl::barrier_raw"}


def _shared(b) -> bool:
    return isinstance(b, Buffer) and b.scope == "shared"


def _atomic_targets(e) -> list:
    """The LDS element loads that are the *target* of an atomic call in ``e`` (``tl.atomic_*``
    first argument): an atomic read-modify-write, not a plain read."""
    from ..ir.expr import Call
    out = []
    for n in post_order(e):
        if isinstance(n, Call) and n.op.startswith("tl.atomic") and n.args:
            a0 = n.args[0]
            if isinstance(a0, BufferLoad) and _shared(a0.buffer):
                out.append(a0)
    return out


def _expr_reads(e, out: Set, atoms: Set = None):
    """Shared buffers ``e`` reads; with ``atoms`` given, buffers it updates atomically go there
    instead of ``out`` (atomics of one buffer commute, so they need no barrier between them)."""
    if not isinstance(e, PrimExpr):
        return
    skip = set()
    if atoms is not None:
        for a0 in _atomic_targets(e):
            skip.add(id(a0))
            atoms.add(a0.buffer)
    for n in post_order(e):
        if isinstance(n, BufferLoad) and _shared(n.buffer) and id(n) not in skip:
            out.add(n.buffer)
        if isinstance(n, L.BufferPtr) and _shared(n.buffer):
            out.add(n.buffer)


class _State:

    def __init__(self, reads=None, writes=None, atoms=None):
        self.reads: Set = set(reads or ())
        self.writes: Set = set(writes or ())
        self.atoms: Set = set(atoms or ())  # buffers updated by atomics since the last barrier

    def copy(self):
        return _State(self.reads, self.writes, self.atoms)

    def merge(self, o):
        return _State(self.reads | o.reads, self.writes | o.writes, self.atoms | o.atoms)

    def add(self, r, w, a):
        return _State(self.reads | r, self.writes | w, self.atoms | a)


def _stmt_access(s, managed) -> Tuple[Set, Set, Set, bool]:
    """(reads, writes, atomics, is_barrier) of a leaf statement.  ``atomics``: shared buffers
    updated by ``tl.atomic_*`` (with or without a returned old value) -- they conflict with plain
    reads and writes of the buffer but not with each other."""
    r, w, a = set(), set(), set()
    if isinstance(s, L.CallStmt):
        if s.name in _BARRIERS:
            return r, w, a, True
        if s.name in ("tl::glds16", "tl::glds4", "tl::buffer_lds16", "tl::glds16_nt"):
            # async LDS-DMA is only produced by the software pipeline, which orders it with
            # counted vmcnt waits + raw barriers itself (a __syncthreads here would drain it)
            return r, w, a, False
        for x in s.args:
            _expr_reads(x, r, a)
        if s.name.startswith("tl::mesh") or s.name.startswith("tl::comm"):
            for x in s.args:
                if isinstance(x, L.BufferPtr) and _shared(x.buffer):
                    w.add(x.buffer)
        return r - managed, w - managed, a - managed, False
    if isinstance(s, S.StoreStmt):
        for i in s.indices:
            _expr_reads(i, r, a)
        _expr_reads(s.value, r, a)
        if _shared(s.buffer):
            w.add(s.buffer)
    elif isinstance(s, L.VecStoreStmt):
        _expr_reads(s.index, r, a)
        for v in s.values:
            _expr_reads(v, r, a)
        if _shared(s.buffer):
            w.add(s.buffer)
    elif isinstance(s, L.VecLoadStmt):
        # the address may itself read LDS (a row id staged in shared memory: Contrib[pos[r], c])
        _expr_reads(s.src_index, r, a)
        if _shared(s.src):
            r.add(s.src)
        if _shared(s.dst):
            w.add(s.dst)
    elif isinstance(s, L.CopyBytesStmt):
        _expr_reads(s.src_index, r, a)
        _expr_reads(s.dst_index, r, a)
        if _shared(s.src):
            r.add(s.src)
        if _shared(s.dst):
            w.add(s.dst)
    elif isinstance(s, S.LetStmt):
        _expr_reads(s.value, r, a)
    elif isinstance(s, S.EvaluateStmt):
        from ..ir.expr import Call
        if isinstance(s.expr, Call) and s.expr.op in ("tl.sync_threads", "tl.sync_grid"):
            return r, w, a, True
        _expr_reads(s.expr, r, a)
    elif isinstance(s, S.AssertStmt):
        _expr_reads(s.cond, r, a)
    return r - managed, w - managed, a - managed, False


def _sync():
    return L.CallStmt("tl::sync_threads", [])


class ThreadSync:

    def __init__(self):
        self.managed: Set = set()
        self.tvars = ()
        self.tdims = None
        self.nthreads = 0
        self.loop_ranges = {}  # enclosing constant-bounded loops (for the divergent-branch proof)
        self.uniform = set()

    def needs(self, st: _State, r, w, a=frozenset()) -> bool:
        # RAW and WAR hazards; WAW between different threads writing the same location is
        # a program race in the tile model and is not ordered by the compiler (as in the reference).
        # An atomic update conflicts with plain accesses of its buffer, never with another atomic
        # (they commute: a histogram's per-element atomics need no barrier between iterations).
        return bool((r & st.writes) or (w & st.reads) or ((r | w) & st.atoms) or (a & (st.reads | st.writes)))

    def scan(self, s, st: _State):
        """Returns (new_stmt, state_after, inserted_at_front)."""
        if isinstance(s, S.SeqStmt):
            out = []
            for c in s.stmts:
                nc, st = self.scan_one(c, st, out)
            ns = S.SeqStmt(out)
            if getattr(s, "scoped", False):
                ns.scoped = True
            return ns, st
        out = []
        ns, st = self.scan_one(s, st, out)
        return (out[0] if len(out) == 1 else S.SeqStmt(out)), st

    def first_access(self, s) -> Tuple[Set, Set, Set]:
        """Accesses of ``s`` before its first unconditional barrier (conservative)."""
        r_all, w_all, a_all = set(), set(), set()
        for x in _leaves(s):
            r, w, a, bar = _stmt_access(x, self.managed)
            if bar:
                break
            r_all |= r
            w_all |= w
            a_all |= a
        return r_all, w_all, a_all

    def scan_one(self, c, st: _State, out: List):
        if isinstance(c, S.SeqStmt):
            nc, st = self.scan(c, st)
            out.append(nc)
            return nc, st
        if isinstance(c, (S.ForStmt, S.WhileStmt)):
            body = c.body
            managed_here = set()
            if isinstance(c, S.ForStmt) and c.annotations.get("pipelined"):
                for x in _leaves(body):
                    if isinstance(x, L.CallStmt) and x.name.startswith("tl::glds"):
                        managed_here.add(x.args[1].buffer)
                    if isinstance(x, L.CallStmt) and x.name in ("tl::gemm_ss", "tl::gemm_rs"):
                        pass
                # stage buffers: any shared buffer with a `stages_of`
                for x in _leaves(body):
                    for b in _buffers_of(x):
                        if getattr(getattr(b, "orig", None), "stages_of", None) is not None:
                            managed_here.add(b)
            saved = set(self.managed)
            self.managed |= managed_here
            saved_ranges = self.loop_ranges
            if isinstance(c, S.ForStmt):
                from ..ir.expr import as_int
                lo, ext = as_int(c.min), as_int(c.extent)
                if lo is not None and ext is not None:
                    self.loop_ranges = {**self.loop_ranges, c.var: range(lo, lo + ext)}
            # hazard with what precedes the loop: barrier in front
            r0, w0, a0 = self.first_access(body)
            if self.needs(st, r0, w0, a0):
                out.append(_sync())
                st = _State()
            nb, st_end = self.scan(body, st.copy())
            # loop-carried: entry of iteration i+1 after end of iteration i
            r1, w1, a1 = self.first_access(nb)
            if self.needs(st_end, r1, w1, a1):
                nb = S.SeqStmt([_sync(), nb])
                nb, st_end = self.scan(nb, _State())
            self.managed = saved
            self.loop_ranges = saved_ranges
            if isinstance(c, S.ForStmt):
                nc = S.ForStmt(c.var, c.min, c.extent, c.kind, nb, c.annotations)
            else:
                nc = S.WhileStmt(c.cond, nb)
            out.append(nc)
            return nc, st.merge(st_end)
        if isinstance(c, S.IfStmt):
            # barriers must not be inside divergent branches: pre-sync if any branch conflicts
            r0, w0, a0 = set(), set(), set()
            for x in _leaves(c):
                r, w, a, _ = _stmt_access(x, self.managed)
                r0 |= r
                w0 |= w
                a0 |= a
            if self.needs(st, r0, w0, a0):
                out.append(_sync())
                st = _State()
            if _thread_dependent(c.cond, self.tvars, self.uniform):
                # divergent branch: a barrier inside would deadlock the workgroup.  Accesses in
                # it are ordered against the surroundings by the barrier in front (above) and
                # by the next conflicting access after it.  Inside, a hazard needs no barrier
                # only when a thread reads back exactly the elements it wrote itself (same
                # index expression); anything else crosses threads (possibly waves) and is
                # refused rather than emitted as a silent race.
                _check_divergent_hazards(c, self.managed, self.nthreads, self.tvars, self.loop_ranges, self.tdims)
                out.append(c)
                return c, st.add(r0, w0, a0)
            # block-uniform condition: scan the branches for internal hazards
            tb, st_t = self.scan(c.then_body, st.copy())
            eb, st_e = (self.scan(c.else_body, st.copy()) if c.else_body is not None else (None, st.copy()))
            nc = S.IfStmt(c.cond, tb, eb)
            out.append(nc)
            return nc, st_t.merge(st_e)
        if isinstance(c, S.KernelStmt):
            self.tvars = tuple(c.thread_vars or ())
            self.tdims = [int(n) for n in (c.threads or [1])]
            self.nthreads = 1
            for n in (c.threads or [1]):
                self.nthreads *= int(n)
            self.uniform = _uniform_registers(c, self.tvars)
            nb, st2 = self.scan(c.body, _State())
            k = S.KernelStmt(c.grid, c.threads, c.block_vars, c.thread_vars, nb, c.is_cpu, c.prelude)
            k.attrs = dict(c.attrs)
            out.append(k)
            return k, st2
        r, w, a, bar = _stmt_access(c, self.managed)
        if bar:
            out.append(c)
            return c, _State()
        if self.needs(st, r, w, a):
            out.append(_sync())
            st = _State()
        out.append(c)
        return c, st.add(r, w, a)


def _indexed_access(s, managed):
    """[(buffer, 'r'|'w', [index exprs] | None, width)] of the LDS accesses of one leaf; None =
    an access whose extent is unknown (a pointer handed to a device call)."""
    out = []

    def reads_of(e):
        if not isinstance(e, PrimExpr):
            return
        tgt = _atomic_targets(e)
        skip = {id(a0) for a0 in tgt}
        for a0 in tgt:  # an atomic target is an update (ordered like a write), not a plain read
            out.append((a0.buffer, "w", list(a0.indices), 1))
        for n in post_order(e):
            if isinstance(n, BufferLoad) and _shared(n.buffer) and id(n) not in skip:
                out.append((n.buffer, "r", list(n.indices), 1))
            elif isinstance(n, L.BufferPtr) and _shared(n.buffer):
                out.append((n.buffer, "r", None, 0))

    if isinstance(s, L.CallStmt):
        if s.name in ("tl::glds16", "tl::glds4", "tl::buffer_lds16", "tl::glds16_nt"):
            return []
        writes = s.name.startswith("tl::mesh") or s.name.startswith("tl::comm")  # as _stmt_access
        for a in s.args:
            if isinstance(a, L.BufferPtr) and _shared(a.buffer):
                out.append((a.buffer, "r", None, 0))
                if writes:
                    out.append((a.buffer, "w", None, 0))
            else:
                reads_of(a)
    elif isinstance(s, S.StoreStmt):
        for i in s.indices:
            reads_of(i)
        reads_of(s.value)
        if _shared(s.buffer):
            out.append((s.buffer, "w", list(s.indices), 1))
    elif isinstance(s, L.VecStoreStmt):
        reads_of(s.index)
        for v in s.values:
            reads_of(v)
        if _shared(s.buffer):
            out.append((s.buffer, "w", [s.index], len(s.values)))
    elif isinstance(s, L.VecLoadStmt):
        reads_of(s.src_index)
        if _shared(s.src):
            out.append((s.src, "r", [s.src_index], s.n))
    elif isinstance(s, L.CopyBytesStmt):
        reads_of(s.src_index)
        reads_of(s.dst_index)
        if _shared(s.src):
            out.append((s.src, "r", [s.src_index], max(1, s.nbytes // s.src.dtype.bytes)))
        if _shared(s.dst):
            out.append((s.dst, "w", [s.dst_index], max(1, s.nbytes // s.dst.dtype.bytes)))
    elif isinstance(s, S.EvaluateStmt):
        reads_of(s.expr)
    elif isinstance(s, (S.LetStmt, S.AssertStmt)):
        reads_of(s.value if isinstance(s, S.LetStmt) else s.cond)
    return [a for a in out if a[0] not in managed]


_MAX_ENUM = 1 << 16  # threads x loop-iteration points enumerated by the ownership proof


def _loop_ranges(body):
    """var -> range of the constant-bounded loops inside ``body``."""
    from ..ir.expr import as_int
    out = {}
    for x in S.walk(body) if body is not None else ():
        if isinstance(x, S.ForStmt):
            lo, ext = as_int(x.min), as_int(x.extent)
            if lo is not None and ext is not None:
                out[x.var] = range(lo, lo + ext)
    return out


def _thread_env(t, tvars):
    """Values of the thread-index variables for flat thread id ``t`` (None if the expression
    would need a variable this model does not know)."""
    env = {}
    for v in tvars:
        env[v] = t
    return env


def _elements_by_thread(accs, cond, nthreads, tvars, ranges, tdims=None):
    """{(kind, element): {threads}} over every guard-satisfying thread and loop point, or None
    when an index cannot be evaluated (unknown variable, register load, pointer access).
    Thread ``t`` is the flat id; with several thread dimensions (``tdims`` = (X, Y, ...)) each
    thread variable takes its own component ``(t // (X..)) % dim`` — without the dimensions a
    multi-dimensional block is not provable here."""
    import itertools
    from ..ir.expr import EvalError, Var, evaluate, free_vars
    tvars = tuple(tvars)
    multi = len(tvars) > 1
    if multi and (tdims is None or len(tdims) != len(tvars)):
        return None
    strides = []
    acc = 1
    for d in (tdims or [nthreads])[:max(1, len(tvars))]:
        strides.append(acc)
        acc *= int(d)
    x_dim = int(tdims[0]) if multi else nthreads
    names = {"tid": lambda t: t, "tid_": lambda t: t, "tx": lambda t: t % x_dim, "lane": lambda t: t % 64,
             "lane_": lambda t: t % 64, "wave": lambda t: t // 64, "wave_": lambda t: t // 64}

    def tval(v, t):
        if v in tvars:
            d = tvars.index(v)
            return (t // strides[d]) % int(tdims[d]) if multi else t
        return names[v.name](t)

    out = {}
    for kind, idx, width in accs:
        if idx is None or any(not isinstance(i, PrimExpr) for i in idx):
            return None
        fv = set()
        for i in idx:
            fv |= set(free_vars(i))
        if any(isinstance(n, BufferLoad) for i in idx for n in post_order(i)):
            return None
        loops = [v for v in fv if v in ranges]
        thread_like = [v for v in fv if v in tvars or v.name in names]
        if len(loops) + len(thread_like) != len(fv):
            return None  # a variable of unknown range (outer loop, block index): not provable here
        pts = 1
        for v in loops:
            pts *= len(ranges[v])
        if pts * nthreads > _MAX_ENUM:
            return None
        for t in range(nthreads):
            env = {v: tval(v, t) for v in thread_like}
            try:
                cenv = {v: tval(v, t) for v in free_vars(cond)
                        if v in tvars or v.name in names} if cond is not None else {}
                if cond is not None and not evaluate(cond, cenv):
                    continue
            except EvalError:
                pass  # a condition on other values: every thread may take the branch
            for combo in itertools.product(*[ranges[v] for v in loops]):
                e2 = dict(env)
                e2.update(zip(loops, combo))
                try:
                    el = tuple(evaluate(i, e2) for i in idx)
                except EvalError:
                    return None
                for w in range(width):
                    key = (kind, el[:-1] + (el[-1] + w, ))
                    out.setdefault(key, set()).add(t)
    return out


def _owned_per_instance(b, accs, cond, nthreads, tvars, inner, outer, tdims=None):
    """True if, for every instance of the enclosing loops (barriers separate instances: the
    scan puts one in front of a loop-carried hazard), no element of ``b`` is written by one
    thread and read by another inside the branch; raises on a proven cross-thread pair;
    False if not provable (unknown index variables / too many points)."""
    import itertools
    from ..ir.expr import free_vars
    used = set()
    for _, idx, _ in accs:
        for i in (idx or ()):
            used |= set(free_vars(i))
    outer_vars = [v for v in used if v in outer and v not in inner]
    n_inst = 1
    for v in outer_vars:
        n_inst *= len(outer[v])
    if n_inst > 64:
        return False
    for combo in itertools.product(*[outer[v] for v in outer_vars]):
        fixed = dict(zip(outer_vars, combo))
        from ..ir.expr import substitute
        accs_i = [(k, [substitute(i, fixed) for i in idx] if idx is not None else None, w) for k, idx, w in accs]
        owners = _elements_by_thread(accs_i, cond, nthreads, tvars, inner, tdims)
        if owners is None:
            return False
        for (kind, el), ts in owners.items():
            if kind != "w":
                continue
            readers = owners.get(("r", el), set())
            if readers and len(ts | readers) > 1:
                raise RuntimeError(
                    f"LDS hazard inside a thread-dependent branch (if {cond}): element {list(el)} of "
                    f"'{b.name}' is written by thread(s) {sorted(ts)[:4]} and read by thread(s) "
                    f"{sorted(readers)[:4]}; a barrier cannot be placed inside the branch. Move the "
                    f"shared-memory exchange out of the branch.")
    return True


def _check_divergent_hazards(c: "S.IfStmt", managed, nthreads=0, tvars=(), outer_ranges=None, tdims=None):
    """Raise on an LDS hazard between accesses INSIDE a thread-dependent branch that crosses
    threads: a barrier cannot be placed there (it would deadlock), and leaving it out would be a
    race.  A write and a read (either order) of one element by two different threads is such a
    hazard; a thread re-reading elements it wrote itself is ordered by program order.  Proof by
    enumeration of the threads that take the branch and of the branch's constant-bounded loops;
    anything not provable that way must at least use the same index expression for the write
    and the read."""
    for body in (c.then_body, c.else_body):
        if body is None:
            continue
        from ..ir.expr import substitute
        by_buf, lets = {}, {}
        for x in _leaves(body):
            if isinstance(x, S.LetStmt):
                lets[x.var] = substitute(x.value, lets) if lets else x.value
            for b, kind, idx, width in _indexed_access(x, managed):
                if idx is not None and lets:
                    idx = [substitute(i, lets) for i in idx]
                by_buf.setdefault(b, []).append((kind, idx, width))
        inner = _loop_ranges(body)
        for b, accs in by_buf.items():
            kinds = {k for k, _, _ in accs}
            if kinds != {"r", "w"}:
                continue
            if nthreads and _owned_per_instance(b, accs, c.cond, nthreads, tvars, inner, outer_ranges or {},
                                                tdims):
                continue
            keys_w = {repr(i) for k, i, _ in accs if k == "w"}
            keys_r = {repr(i) for k, i, _ in accs if k == "r"}
            if any(i is None for _, i, _ in accs) or keys_w != keys_r or len(keys_w) != 1:
                raise RuntimeError(
                    f"LDS hazard inside a thread-dependent branch (if {c.cond}): buffer '{b.name}' is "
                    f"written and read at elements that cannot be shown to belong to one thread; a "
                    f"barrier cannot be placed inside the branch. Move the shared-memory exchange out "
                    f"of the branch.")


def _leaves(s):
    """Leaf statements in program order; control expressions (if / while conditions, loop
    bounds) appear as ``EvaluateStmt`` pseudo-leaves so their LDS reads are seen too."""
    if s is None:
        return
    if isinstance(s, S.SeqStmt):
        for c in s.stmts:
            yield from _leaves(c)
    elif isinstance(s, S.ForStmt):
        yield S.EvaluateStmt(s.min)
        yield S.EvaluateStmt(s.extent)
        yield from _leaves(s.body)
    elif isinstance(s, S.WhileStmt):
        yield S.EvaluateStmt(s.cond)
        yield from _leaves(s.body)
    elif isinstance(s, S.IfStmt):
        yield S.EvaluateStmt(s.cond)
        yield from _leaves(s.then_body)
        yield from _leaves(s.else_body)
    elif isinstance(s, S.AttrStmt):
        yield from _leaves(s.body)
    else:
        yield s


# thread-index variables: the user's T.Kernel thread vars plus the lowering's own
# (lower_tile_op.LowerCtx: tid / lane / wave, printed with a trailing underscore)
_THREAD_NAMES = {"tid", "lane", "wave", "tid_", "tx", "ty", "tz", "lane_", "wave_"}


def _thread_dependent(e, tvars, uniform=()) -> bool:
    """May ``e`` differ between the threads of a block?  Thread ids do; a register variable does
    unless every store to it is block-uniform (``uniform``); a memory load does iff its address does."""
    from ..ir.expr import Var
    if not isinstance(e, PrimExpr):
        return False
    for n in post_order(e):
        if isinstance(n, Var) and (n in tvars or n.name in _THREAD_NAMES):
            return True
        if isinstance(n, BufferLoad):
            sc = getattr(n.buffer, "scope", "")
            if sc not in ("global", "shared") and n.buffer not in uniform:
                return True  # a register value may differ per thread
    return False


def _register_stores(s, guards, out):
    """(store, enclosing if-conditions / loop bounds) of every register store under ``s``."""
    if s is None:
        return
    if isinstance(s, S.StoreStmt):
        if getattr(s.buffer, "scope", "") not in ("global", "shared"):
            out.setdefault(s.buffer, []).append((s, guards))
    elif isinstance(s, S.SeqStmt):
        for c in s.stmts:
            _register_stores(c, guards, out)
    elif isinstance(s, S.IfStmt):
        g = guards + (s.cond,)
        _register_stores(s.then_body, g, out)
        _register_stores(s.else_body, g, out)
    elif isinstance(s, S.ForStmt):
        _register_stores(s.body, guards + (s.min, s.extent), out)
    elif isinstance(s, S.WhileStmt):
        _register_stores(s.body, guards + (s.cond,), out)
    elif isinstance(s, (S.KernelStmt, S.AttrStmt)) or hasattr(s, "body"):
        _register_stores(getattr(s, "body", None), guards, out)


def _uniform_registers(k: S.KernelStmt, tvars) -> set:
    """Register buffers (``T.alloc_var`` / locals) whose every store is block-uniform (fixpoint).
    A store counts as uniform only if its value, its indices AND every condition / loop bound
    it sits under are: ``if tid == 0: flag = 1`` leaves ``flag`` thread-dependent."""
    stores = {}
    _register_stores(k.body, (), stores)
    uniform = set(stores)
    changed = True
    while changed:
        changed = False
        for b in list(uniform):
            for st, guards in stores[b]:
                if _thread_dependent(st.value, tvars, uniform) or \
                        any(_thread_dependent(i, tvars, uniform) for i in st.indices) or \
                        any(_thread_dependent(g, tvars, uniform) for g in guards):
                    uniform.discard(b)
                    changed = True
                    break
    return uniform


def _has_barrier(s) -> bool:
    for x in _leaves(s):
        if isinstance(x, L.CallStmt) and x.name in _BARRIERS:
            return True
        if isinstance(x, S.EvaluateStmt):
            from ..ir.expr import Call
            if isinstance(x.expr, Call) and x.expr.op in ("tl.sync_threads", "tl.sync_grid"):
                return True
    return False


def check_divergent_barriers(s, tvars=(), where="kernel", uniform=()):
    """A block barrier inside a thread-dependent branch or loop deadlocks the workgroup on the
    GPU: refuse to emit such code (the reference's ThreadSync has the same rule)."""
    if s is None:
        return
    if isinstance(s, S.SeqStmt):
        for c in s.stmts:
            check_divergent_barriers(c, tvars, where, uniform)
    elif isinstance(s, S.KernelStmt):
        tv = tuple(s.thread_vars or ())
        check_divergent_barriers(s.body, tv, where, _uniform_registers(s, tv))
    elif isinstance(s, S.IfStmt):
        if _thread_dependent(s.cond, tvars, uniform) and (_has_barrier(s.then_body) or _has_barrier(s.else_body)):
            raise RuntimeError(f"{where}: a block barrier is required inside a thread-dependent branch "
                               f"(if {s.cond}); move the shared-memory communication out of the branch")
        check_divergent_barriers(s.then_body, tvars, where, uniform)
        check_divergent_barriers(s.else_body, tvars, where, uniform)
    elif isinstance(s, S.ForStmt):
        if (_thread_dependent(s.min, tvars, uniform) or _thread_dependent(s.extent, tvars, uniform)) and \
                _has_barrier(s.body):
            raise RuntimeError(f"{where}: a block barrier is required inside a loop with a thread-dependent "
                               f"trip count ({s.var})")
        check_divergent_barriers(s.body, tvars, where, uniform)
    elif isinstance(s, S.WhileStmt):
        if _thread_dependent(s.cond, tvars, uniform) and _has_barrier(s.body):
            raise RuntimeError(f"{where}: a block barrier is required inside a loop with a thread-dependent "
                               f"condition ({s.cond})")
        check_divergent_barriers(s.body, tvars, where, uniform)
    elif isinstance(s, S.AttrStmt):
        check_divergent_barriers(s.body, tvars, where, uniform)


def _buffers_of(x):
    out = []
    if isinstance(x, L.CallStmt):
        for a in x.args:
            if isinstance(a, L.BufferPtr):
                out.append(a.buffer)
    if isinstance(x, S.StoreStmt):
        out.append(x.buffer)
        for n in post_order(x.value):
            if isinstance(n, BufferLoad):
                out.append(n.buffer)
    if isinstance(x, (L.VecStoreStmt, )):
        out.append(x.buffer)
    if isinstance(x, (L.VecLoadStmt, L.CopyBytesStmt)):
        out += [x.src, x.dst]
    return out


def insert_thread_sync(kernel: S.KernelStmt) -> S.KernelStmt:
    ts = ThreadSync()
    out = []
    k, _ = ts.scan_one(kernel, _State(), out)
    if not getattr(k, "is_cpu", False):
        check_divergent_barriers(k)
    return k
