"""``T.Pipelined(order=, stage=, group=)``: user-specified software-pipeline schedules.

Reference semantics (``src/ir.cc:82-113`` records them; ``src/transform/inject_pipeline.cc``
executes them; used by ``examples/flash_attention/example_mha_fwd_bshd_wgmma_pipelined.py:144``):
the loop body's top-level statements are partitioned into groups (``group``, default one statement
per group); group g runs ``stage[g]`` iterations behind stage 0, and within one iteration of the new
loop the groups run in ascending ``order[g]``.  Groups with ``order == stage == -1`` are producers
(global->shared copies) that the gfx950 pipeline turns into LDS-DMA issued ahead.

So for the FlashAttention schedule ``order=[-1,0,3,1,-1,2], stage=[-1,0,0,1,-1,1]`` iteration t runs
``QK^T(t)``, then ``rescale(t-1)``, ``PV(t-1)`` and ``softmax(t)``: the matrix-core work of one tile
sits next to the VALU/transcendental work of the other with no data dependence between them, which
is what lets the scheduler interleave MFMA with ``v_exp_f32`` inside a wave.

Lowering (before layout inference, so every copy of a statement gets its layouts):

  prologue   t = 0 .. S-1        groups with stage <= t, for iteration t - stage (guarded < n)
  main       t = S .. n-1        every group, for iteration t - stage        <- T.Pipelined ring
  epilogue   t = max(n,S) .. n+S-1  groups with stage >= 1, for iteration t - stage (guarded)

A producer runs in the stage of its first consumer, immediately before it.  The main loop keeps
``num_stages`` and goes through the ordinary pipeline pass (``pipeline.py``).  A fragment written
by a group and read by a group of a later stage must not be overwritten in between (the new loop
does not multi-version registers); such schedules are rejected.
"""
from __future__ import annotations

from typing import List

from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.expr import IntImm, as_int, binop
from .utils import Mutator, flatten_seq, subst_stmt


def _reads_writes(st):
    """(buffers read, buffers written) by a pre-lowering statement."""
    from ..ir.expr import post_order, BufferLoad
    reads, writes = set(), set()
    for x in S.walk(st):
        exprs = []
        if isinstance(x, S.TileOpStmt):
            for r in x.op.reads():
                reads.add(r.buffer)
            for r in x.op.writes():
                writes.add(r.buffer)
        elif isinstance(x, S.StoreStmt):
            writes.add(x.buffer)
            exprs = [x.value] + list(x.indices)
        elif isinstance(x, S.LetStmt):
            exprs = [x.value]
        elif isinstance(x, S.EvaluateStmt):
            exprs = [x.expr]
        elif isinstance(x, (S.IfStmt, S.WhileStmt)):
            exprs = [x.cond]
        elif isinstance(x, S.ForStmt):
            exprs = [x.min, x.extent]
        for e in exprs:
            if hasattr(e, "dtype"):
                for nd in post_order(e):
                    if isinstance(nd, BufferLoad):
                        reads.add(nd.buffer)
    return reads, writes


def _is_producer(st):
    return isinstance(st, S.TileOpStmt) and isinstance(st.op, O.CopyOp) and \
        st.op.src.buffer.scope == "global" and st.op.dst.buffer.scope == "shared"


class _StageSchedule(Mutator):

    def visit_ForStmt(self, s: S.ForStmt):
        body = self.stmt(s.body)
        ann = s.annotations
        if s.kind != "pipelined" or ("order" not in ann and "stage" not in ann):
            return S.ForStmt(s.var, s.min, s.extent, s.kind, body, ann)
        stmts = flatten_seq(body)
        group = ann.get("group") or [[i] for i in range(len(stmts))]
        order, stage = list(ann.get("order") or []), list(ann.get("stage") or [])
        if not order:
            order = list(range(len(group)))
        if not stage:
            stage = [0] * len(group)
        flat = sorted(i for g in group for i in g)
        if flat != list(range(len(stmts))):
            raise ValueError(f"T.Pipelined group={group} must partition the {len(stmts)} statements of the loop body")
        if len(order) != len(group) or len(stage) != len(group):
            raise ValueError(f"T.Pipelined order={order} / stage={stage} need one entry per group ({len(group)})")
        order_alt = list(ann.get("order_alt") or [])
        if order_alt:
            if len(order_alt) != len(group):
                raise ValueError(f"T.Pipelined order_alt={order_alt} needs one entry per group ({len(group)})")
            if any((order_alt[g] == -1) != (order[g] == -1) for g in range(len(group))):
                raise ValueError("T.Pipelined: order_alt must keep the producers (order -1) of order")
        groups = [[stmts[i] for i in g] for g in group]
        compute = [gi for gi in range(len(groups)) if not (order[gi] == -1 and stage[gi] == -1)]
        producers = [gi for gi in range(len(groups)) if order[gi] == -1 and stage[gi] == -1]
        for gi in producers:
            if not all(_is_producer(x) for x in groups[gi]):
                raise ValueError("T.Pipelined: order = stage = -1 is for global->shared copies only")
        if any(stage[gi] < 0 for gi in compute):
            raise ValueError("T.Pipelined: stages of compute groups must be >= 0")
        seq = sorted(compute, key=lambda gi: order[gi])
        # producers go right before their first consumer, in its stage
        rw = {gi: _reads_writes(S.seq(*groups[gi])) for gi in range(len(groups))}
        placed = {}
        for pi in producers:
            dsts = {x.op.dst.buffer for x in groups[pi]}
            first = next((gi for gi in seq if rw[gi][0] & dsts or _uses_buffers(groups[gi], dsts)), None)
            placed.setdefault(first, []).append(pi)
        plan: List[tuple] = []  # (stage, [stmts])
        for pi in placed.get(None, []):
            plan.append((0, groups[pi]))
        for gi in seq:
            for pi in placed.get(gi, []):
                plan.append((stage[gi], groups[pi]))
            plan.append((stage[gi], groups[gi]))
        self._check_hazards(seq, stage, order, groups)
        alt_plan = None
        if order_alt:
            seq_alt = sorted(compute, key=lambda gi: order_alt[gi])
            self._check_hazards(seq_alt, stage, order_alt, groups)
            alt_plan = [(stage[gi], groups[gi]) for gi in seq_alt]
        S_max = max(st for st, _ in plan)
        k, n, mn = s.var, s.extent, s.min
        main_ann = {kk: v for kk, v in ann.items() if kk not in ("order", "stage", "group", "sync", "order_alt",
                                                                  "alt_cond")}
        if S_max == 0:
            return S.ForStmt(k, mn, n, "pipelined", S.seq(*[x for _, g in plan for x in g]), main_ann)
        nv = as_int(n)

        prologue = []
        for t in range(S_max):
            parts = []
            for st_, g in plan:
                if st_ > t:
                    continue
                j = t - st_
                body_j = S.seq(*[subst_stmt(x, {k: binop("+", mn, IntImm(j))}) for x in g])
                if nv is not None:
                    if j < nv:
                        parts.append(body_j)
                else:
                    parts.append(S.IfStmt(binop("<", IntImm(j), n), body_j))
            prologue += parts
        # the main loop reuses the loop variable as the new-loop iteration counter t
        main_body = []
        if alt_plan is None:
            for st_, g in plan:
                main_body += [subst_stmt(x, {k: binop("-", k, st_)}) for x in g]
        else:
            # producers first (their copies become LDS-DMA issued ahead by the pipeline pass, so
            # their place in the body only sets the issue point), then the compute in either order
            prod_set = {id(x) for pi in producers for x in groups[pi]}
            for st_, g in plan:
                if all(id(x) in prod_set for x in g):
                    main_body += [subst_stmt(x, {k: binop("-", k, st_)}) for x in g]
            comp = [subst_stmt(x, {k: binop("-", k, st_)}) for st_, g in plan for x in g if id(x) not in prod_set]
            comp_alt = [subst_stmt(x, {k: binop("-", k, st_)}) for st_, g in alt_plan for x in g]
            # tl.unswitch: the condition is loop-invariant and wave-uniform; after pipelining and
            # barrier placement the loop is unswitched (transform/unswitch.py) so each wave group
            # runs a loop of its own order (one loop with the branch inside spilled: both orders'
            # live ranges meet at the join)
            from ..ir.expr import call as _call
            cond = _call("tl.unswitch", [ann["alt_cond"]], "bool")
            main_body.append(S.IfStmt(cond, S.seq(*comp_alt), S.seq(*comp)))
        main = S.ForStmt(k, binop("+", mn, S_max), binop("-", n, S_max), "pipelined", S.seq(*main_body), main_ann)
        if nv is not None and nv <= S_max:
            main = None
        from ..ir.expr import Var
        from ..ir.expr import max_expr as _max
        e = Var(k.name + "_epi", k.dtype)
        epi_body = []
        for st_, g in plan:
            if st_ < 1:
                continue
            jj = binop("-", e, st_)
            body_j = S.seq(*[subst_stmt(x, {k: binop("+", mn, jj)}) for x in g])
            epi_body.append(S.IfStmt(binop("&&", binop(">=", jj, 0), binop("<", jj, n)), body_j))
        start = _max(n, IntImm(S_max))
        epilogue = S.ForStmt(e, start, binop("-", binop("+", n, S_max), start), "serial", S.seq(*epi_body), {})
        return S.seq(*(prologue + ([main] if main is not None else []) + [epilogue]))

    @staticmethod
    def _check_hazards(seq, stage, order, groups):
        info = {gi: _reads_writes(S.seq(*groups[gi])) for gi in seq}
        for w in seq:
            for r in seq:
                if stage[r] <= stage[w]:
                    continue
                shared = {b for b in info[w][1] & info[r][0] if b.scope in ("fragment", "local", "var")}
                if not shared:
                    continue
                if stage[r] - stage[w] > 1 or order[w] < order[r]:
                    names = ", ".join(sorted(b.name for b in shared))
                    raise NotImplementedError(
                        f"T.Pipelined: {names} is written in stage {stage[w]} and read in stage {stage[r]} after "
                        f"being overwritten by the next iteration; order the reader before the writer")


def _uses_buffers(stmts, bufs):
    return any(_reads_writes(st)[0] & bufs for st in stmts)


def apply_stage_schedules(kernel):
    return _StageSchedule().stmt(kernel)
