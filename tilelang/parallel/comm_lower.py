"""Lowering of ``T.comm`` tile ops to device-initiated xGMI transfers (gfx950) or to the
same protocol on the CPU plumbing target.

Reference: ``src/op/comm.cc`` — ``BroadcastOpNode::Lower`` (:121-218), ``PutOpNode::Lower``
(:259-385), ``AllgatherOpNode::Lower`` (:479-598), ``AllreduceOpNode::Lower`` (:783-919).  The
reference routes everything over a 2-D mesh as chains of row/column ``broadcast_`` calls and
stops at TIR.  On MI355X every GPU pair has a dedicated xGMI link, so each op becomes a set of
direct point-to-point tile transfers executed by the kernel itself:

  * broadcast(src_core, dir): src -> every member of its row/column/mesh (itself included);
  * put(src, dst):            src -> dst (one hop, no intermediate core);
  * all_gather(dir):          every core -> every member of its group, slice = member index;
  * all_reduce(dir):          local reduce along ``dim`` -> all-gather of the partials into the
                              workspace -> every core combines the partials in core-id order
                              (bitwise identical results on every rank);
  * barrier(group), fence().

A transfer is three phases (``include/tl/mesh.h``): the receiver posts *ready*, the sender
waits for it, stores the tile (vectorised, every thread its own fragment registers) into the
receiver's workspace slot and publishes a tagged flag; the receiver waits for the flag and
reads the slot into its destination.  The logical routing schedule of the reference (for
inspection and parity tests) is ``tilelang.parallel.comm_plan``.
"""
from __future__ import annotations

from typing import List, Optional

from ..ir import dtypes as _dt
from ..ir import lowered as L
from ..ir import stmt as S
from ..ir import tileop as O
from ..ir.buffer import Buffer, BufferRegion
from ..ir.expr import BufferLoad, IntImm, Var, as_int, binop, call, cast, const

DIR = {"h": 0, "v": 1, "all": 2}


class CommLoweringError(Exception):
    pass


def _ext(name, args, dtype=_dt.int32):
    return call("extern", [name] + list(args), dtype)


def _align(n, a=256):
    return (int(n) + a - 1) // a * a


def op_slot_bytes(op) -> int:
    """Workspace bytes one source needs for this op (per block)."""
    if isinstance(op, (O.CommBroadcastOp, O.CommPutOp)):
        return op.size * op.src.buffer.dtype.bytes
    if isinstance(op, O.CommAllGatherOp):
        return op.size * op.send.buffer.dtype.bytes
    if isinstance(op, O.CommAllReduceOp):
        part = op.src if op.dim is None else op.tmp
        ext = (part or op.dst).static_extents()
        n = 1
        for e in ext:
            n *= e
        G = _op_group_size(op)
        if _two_shot(op, n, G):
            return (n // G) * (part or op.dst).buffer.dtype.bytes
        return n * (part or op.dst).buffer.dtype.bytes
    return 0


# all_reduce partials of at least this many bytes go reduce-scatter + all-gather ("two-shot"):
# every rank moves 2 (G-1)/G of a tile instead of (G-1) tiles and the workspace shrinks G-fold
TWO_SHOT_MIN_BYTES = 4096


def _op_group_size(op) -> int:
    nrow, ncol = op.mesh if op.mesh is not None else (1, 1)
    return {"h": ncol, "v": nrow, "all": nrow * ncol}[op.direction]


def _two_shot(op, n: int, G: int) -> bool:
    part = op.src if op.dim is None else op.tmp
    nbytes = n * (part or op.dst).buffer.dtype.bytes
    return G > 2 and n % G == 0 and nbytes >= TWO_SHOT_MIN_BYTES


class MeshState:
    """Per-kernel mesh lowering state: runtime parameters, op numbering, slot size."""

    def __init__(self, kernel: S.KernelStmt, nrow: int, ncol: int, slot_bytes: int):
        self.nrow, self.ncol = nrow, ncol
        self.rank = Var("tl_mesh_rank", _dt.int32)
        self.rank.nonneg = True
        self.ws = Var("tl_mesh_ws", _dt.int64)
        self.epoch = Var("tl_mesh_epoch", _dt.uint32)
        self.err = Var("tl_mesh_err", _dt.int64)
        self.mctx = Var("tl_mctx", _dt.handle)
        self.blk = Var("tl_mblk", _dt.int32)
        self.blk.nonneg = True
        self.nops = 0
        self.slot_bytes = _align(max(slot_bytes, 256))
        self.counters: List[Buffer] = []
        self.kernel = kernel
        nb = 1
        for g in kernel.grid:
            v = as_int(g)
            if v is None:
                raise CommLoweringError("kernels using T.comm need a static grid (the mesh workspace is sized "
                                        "per block)")
            nb *= v
        self.nblocks = nb

    @property
    def nranks(self):
        return self.nrow * self.ncol

    def ws_bytes(self) -> int:
        flags = _align(self.nblocks * max(self.nops, 1) * self.nranks * 4)
        return 2 * flags + self.nblocks * self.nops * self.nranks * self.slot_bytes if self.nops else 0

    def extra_params(self):
        return [dict(kind="extra", name="tl_mesh_rank", var=self.rank, ctype="int", nbytes=4),
                dict(kind="extra", name="tl_mesh_ws", var=self.ws, ctype="long long", nbytes=8),
                dict(kind="extra", name="tl_mesh_epoch", var=self.epoch, ctype="unsigned", nbytes=4),
                dict(kind="extra", name="tl_mesh_err", var=self.err, ctype="long long", nbytes=8)]

    def prologue(self) -> List[S.Stmt]:
        k = self.kernel
        out = [S.AllocStmt(c) for c in self.counters]
        out += [S.StoreStmt(c, [IntImm(0)], const(0, _dt.uint32)) for c in self.counters]
        blk = None
        for v, g in reversed(list(zip(k.block_vars, k.grid))):
            blk = v if blk is None else binop("+", v, binop("*", blk, g))
        out.append(S.LetStmt(self.blk, blk if blk is not None else IntImm(0)))
        out.append(L.AutoLetStmt(self.mctx, _ext("tl::mesh::make_ctx", [
            self.rank, self.nrow, self.ncol, self.ws, self.epoch, self.err, self.nblocks, max(self.nops, 1),
            IntImm(self.slot_bytes, _dt.int64)], _dt.handle)))
        return out

    def meta(self) -> dict:
        return dict(shape=(self.nrow, self.ncol), nops=self.nops, slot_bytes=self.slot_bytes,
                    nblocks=self.nblocks, ws_bytes=self.ws_bytes())


def mesh_state(ctx, shape=None) -> MeshState:
    st = getattr(ctx, "mesh", None)
    if st is None:
        if shape is None:
            from .mesh import get_device_mesh_config
            shape = get_device_mesh_config()
        st = MeshState(ctx.kernel, shape[0], shape[1], getattr(ctx, "mesh_slot_bytes", 256))
        ctx.mesh = st
    elif shape is not None and tuple(shape) != (st.nrow, st.ncol):
        raise CommLoweringError(f"T.comm ops traced for different mesh shapes in one kernel: {shape} vs "
                                f"{(st.nrow, st.ncol)}")
    return st


# ---------------------------------------------------------------------------------------
# data movement nests
# ---------------------------------------------------------------------------------------


def _slot_view(name, dtype, n) -> Buffer:
    b = Buffer(name, [n], dtype, "global")
    b.no_guard = True
    b._auto_name = False
    return b


def _flat(vars_, exts):
    q = None
    for v, e in zip(vars_, exts):
        q = v if q is None else binop("+", binop("*", q, e), v)
    return q if q is not None else IntImm(0)


def _check_region(r: BufferRegion, what: str, on_cpu: bool):
    b = r.buffer
    ext = r.static_extents()
    if ext is None:
        raise CommLoweringError(f"T.comm {what}: {b.name} needs static extents")
    if b.scope in ("local", "var") and not on_cpu:
        raise CommLoweringError(f"T.comm {what}: {b.name} is a per-thread local buffer; use a fragment or shared "
                                f"buffer")
    if b.scope == "fragment":
        shp = b.static_shape()
        if ext != shp or any(as_int(m) != 0 for m in r.mins):
            raise CommLoweringError(f"T.comm {what}: fragment {b.name} must be used whole")
    return ext


def _nest(lw, region: BufferRegion, make_body):
    """Parallel nest over ``region``; ``make_body(idx, flat, vars)`` returns the statement."""
    ext = region.static_extents()
    vars_ = [Var(f"cm{i}") for i in range(len(ext))]
    idx = [binop("+", m, v) for m, v in zip(region.mins, vars_)]
    body = make_body(idx, _flat(vars_, ext), vars_)
    for v, e in reversed(list(zip(vars_, ext))):
        body = S.ForStmt(v, 0, e, "parallel", body)
    b = region.buffer
    layout = b.layout if b.scope == "fragment" and not lw.ctx.is_cpu else None
    return lw.lower_nest(body, layout)


def _write_nest(lw, src: BufferRegion, slot: Buffer, size: int):
    n = 1
    for e in src.static_extents():
        n *= e

    def mk(idx, q, _):
        st = S.StoreStmt(slot, [q], cast(BufferLoad(src.buffer, idx), slot.dtype))
        return S.IfStmt(binop("<", q, size), st) if size < n else st

    return _nest(lw, src, mk)


def _read_nest(lw, dst: BufferRegion, slot: Buffer, size: int, lead_stride: Optional[int] = None):
    """dst <- slot.  With ``lead_stride`` the first dst dim selects the source slot (all_gather)."""
    ext = dst.static_extents()

    def mk(idx, q, vars_):
        if lead_stride is None:
            n = 1
            for e in ext:
                n *= e
            st = S.StoreStmt(dst.buffer, idx, cast(BufferLoad(slot, [q]), dst.buffer.dtype))
            return S.IfStmt(binop("<", q, size), st) if size < n else st
        inner = _flat(vars_[1:], ext[1:])
        n_inner = 1
        for e in ext[1:]:
            n_inner *= e
        si = binop("+", binop("*", vars_[0], lead_stride), inner)
        st = S.StoreStmt(dst.buffer, idx, cast(BufferLoad(slot, [si]), dst.buffer.dtype))
        return S.IfStmt(binop("<", inner, size), st) if size < n_inner else st

    return _nest(lw, dst, mk)


# ---------------------------------------------------------------------------------------
# ops
# ---------------------------------------------------------------------------------------


def _begin(st: MeshState, name: str):
    oi = st.nops
    st.nops += 1
    cnt = Buffer(f"tl_mcnt{oi}", [1], _dt.uint32, "local")
    cnt._auto_name = False
    st.counters.append(cnt)
    tag = Var(f"tl_mtag{oi}", _dt.uint32)
    pre = [L.CommentStmt(f"T.comm.{name} (mesh op {oi})"),
           S.StoreStmt(cnt, [IntImm(0)], binop("+", BufferLoad(cnt, [IntImm(0)]), const(1, _dt.uint32))),
           S.LetStmt(tag, _ext("tl::mesh::tag", [st.mctx, BufferLoad(cnt, [IntImm(0)])], _dt.uint32))]
    return oi, tag, pre


def _scoped(stmts):
    s = S.SeqStmt(list(stmts))
    s.scoped = True
    return s


def _send_loop(lw, st, oi, tag, src: BufferRegion, size: int, anchor, dirn: int, count: int, slot_dt):
    """for k < count: d = k-th member (rotated from anchor); handshake; store tile into slot@d."""
    k = Var("cmk")
    d = Var("cmdst", _dt.int32)
    view = _slot_view("cm_out", slot_dt, st.slot_bytes // slot_dt.bytes)
    flat = lw.ctx.flat_of(view)
    body = [S.LetStmt(d, _ext("tl::mesh::group_member_rot", [st.mctx, dirn, anchor, k])),
            L.CallStmt("tl::mesh::wait_ready", [st.mctx, st.blk, oi, d, tag]),
            L.PtrDeclStmt(flat, _ext("tl::mesh::slot", [st.mctx, d, st.blk, oi, st.rank], _dt.handle)),
            _write_nest(lw, src, view, size),
            L.CallStmt("tl::mesh::publish", [st.mctx, st.blk, oi, d, tag])]
    return S.ForStmt(k, 0, count, "serial", _scoped(body))


def _post_ready_loop(st, oi, tag, dirn, count):
    k = Var("cmk")
    return S.ForStmt(k, 0, count, "serial", L.CallStmt(
        "tl::mesh::post_ready", [st.mctx, st.blk, oi, _ext("tl::mesh::group_member", [st.mctx, dirn, st.rank, k]),
                                 tag]))


def _wait_data_loop(st, oi, tag, dirn, count):
    k = Var("cmk")
    return S.ForStmt(k, 0, count, "serial", L.CallStmt(
        "tl::mesh::wait_data", [st.mctx, st.blk, oi, _ext("tl::mesh::group_member", [st.mctx, dirn, st.rank, k]),
                                tag]))


def _group_size(st, dirn):
    return {0: st.ncol, 1: st.nrow, 2: st.nranks}[dirn]


def _member_stride(st, dirn):
    """Distance (in source slots) between consecutive members of a group."""
    return {0: 1, 1: st.ncol, 2: 1}[dirn]


def lower_broadcast(lw, op: O.CommBroadcastOp):
    st = mesh_state(lw.ctx, op.mesh)
    cpu = lw.ctx.is_cpu
    _check_region(op.src, "broadcast", cpu)
    _check_region(op.dst, "broadcast", cpu)
    c, dirn = int(op.src_core), DIR[op.direction]
    oi, tag, out = _begin(st, "broadcast")
    in_grp = _ext("tl::mesh::in_group", [st.mctx, dirn, c, st.rank], _dt.boolean)
    out.append(S.IfStmt(in_grp, L.CallStmt("tl::mesh::post_ready", [st.mctx, st.blk, oi, c, tag])))
    out.append(S.IfStmt(binop("==", st.rank, c),
                        _send_loop(lw, st, oi, tag, op.src, op.size, c, dirn, _group_size(st, dirn),
                                   op.src.buffer.dtype)))
    view = _slot_view("cm_in", op.src.buffer.dtype, st.slot_bytes // op.src.buffer.dtype.bytes)
    recv = [L.CallStmt("tl::mesh::wait_data", [st.mctx, st.blk, oi, c, tag]),
            L.PtrDeclStmt(lw.ctx.flat_of(view), _ext("tl::mesh::slot", [st.mctx, st.rank, st.blk, oi, c], _dt.handle)),
            _read_nest(lw, op.dst, view, op.size)]
    out.append(S.IfStmt(in_grp, _scoped(recv)))
    return _scoped(out)


def lower_put(lw, op: O.CommPutOp):
    st = mesh_state(lw.ctx, op.mesh)
    cpu = lw.ctx.is_cpu
    _check_region(op.src, "put", cpu)
    _check_region(op.dst, "put", cpu)
    c, d = int(op.src_core), int(op.dst_core)
    oi, tag, out = _begin(st, "put")
    is_dst = binop("==", st.rank, d)
    out.append(S.IfStmt(is_dst, L.CallStmt("tl::mesh::post_ready", [st.mctx, st.blk, oi, c, tag])))
    view = _slot_view("cm_out", op.src.buffer.dtype, st.slot_bytes // op.src.buffer.dtype.bytes)
    send = [L.CallStmt("tl::mesh::wait_ready", [st.mctx, st.blk, oi, d, tag]),
            L.PtrDeclStmt(lw.ctx.flat_of(view), _ext("tl::mesh::slot", [st.mctx, d, st.blk, oi, st.rank], _dt.handle)),
            _write_nest(lw, op.src, view, op.size),
            L.CallStmt("tl::mesh::publish", [st.mctx, st.blk, oi, d, tag])]
    out.append(S.IfStmt(binop("==", st.rank, c), _scoped(send)))
    view2 = _slot_view("cm_in", op.src.buffer.dtype, st.slot_bytes // op.src.buffer.dtype.bytes)
    recv = [L.CallStmt("tl::mesh::wait_data", [st.mctx, st.blk, oi, c, tag]),
            L.PtrDeclStmt(lw.ctx.flat_of(view2), _ext("tl::mesh::slot", [st.mctx, st.rank, st.blk, oi, c],
                                                     _dt.handle)),
            _read_nest(lw, op.dst, view2, op.size)]
    out.append(S.IfStmt(is_dst, _scoped(recv)))
    return _scoped(out)


def _write_chunk_nest(lw, src: BufferRegion, slot: Buffer, lo, c: int):
    """slot[q - lo] = src[q] for the flat tile elements q in [lo, lo + c)."""

    def mk(idx, q, _):
        st = S.StoreStmt(slot, [binop("-", q, lo)], cast(BufferLoad(src.buffer, idx), slot.dtype))
        return S.IfStmt(binop("&&", binop(">=", q, lo), binop("<", q, binop("+", lo, c))), st)

    return _nest(lw, src, mk)


def _send_chunks_loop(lw, st, oi, tag, src: BufferRegion, c: int, dirn: int, count: int, slot_dt):
    """Reduce-scatter sends: member d (rotated from me) gets chunk group_index(d) of the tile."""
    k = Var("cmk")
    d = Var("cmdst", _dt.int32)
    ci = Var("cmci", _dt.int32)
    view = _slot_view("cm_out", slot_dt, st.slot_bytes // slot_dt.bytes)
    body = [S.LetStmt(d, _ext("tl::mesh::group_member_rot", [st.mctx, dirn, st.rank, k])),
            S.LetStmt(ci, _ext("tl::mesh::group_index", [st.mctx, dirn, d])),
            L.CallStmt("tl::mesh::wait_ready", [st.mctx, st.blk, oi, d, tag]),
            L.PtrDeclStmt(lw.ctx.flat_of(view), _ext("tl::mesh::slot", [st.mctx, d, st.blk, oi, st.rank], _dt.handle)),
            _write_chunk_nest(lw, src, view, binop("*", ci, c), c),
            L.CallStmt("tl::mesh::publish", [st.mctx, st.blk, oi, d, tag])]
    return S.ForStmt(k, 0, count, "serial", _scoped(body))


def _lower_all_reduce_two_shot(lw, st, op, part: BufferRegion, n: int, dirn: int, kind: str, out: List):
    """Reduce-scatter + all-gather.  Phase 1: member k receives chunk k of every partial and
    combines them in member order; phase 2: every member sends its reduced chunk to all.  Each
    chunk is reduced once, so every rank ends with bitwise identical values."""
    from ..ir.expr import Var as _V
    G = _group_size(st, dirn)
    c = n // G
    pdt = part.buffer.dtype
    oi1 = st.nops - 1
    tag1 = [x for x in out if isinstance(x, S.LetStmt)][-1].var
    out.append(_post_ready_loop(st, oi1, tag1, dirn, G))
    out.append(_send_chunks_loop(lw, st, oi1, tag1, part, c, dirn, G, pdt))
    out.append(_wait_data_loop(st, oi1, tag1, dirn, G))
    oi2, tag2, pre2 = _begin(st, "all_reduce (all-gather phase)")
    out += pre2
    out.append(_post_ready_loop(st, oi2, tag2, dirn, G))
    k = _V("cmk")
    out.append(S.ForStmt(k, 0, G, "serial", L.CallStmt("tl::mesh::wait_ready", [
        st.mctx, st.blk, oi2, _ext("tl::mesh::group_member", [st.mctx, dirn, st.rank, k]), tag2])))
    # my chunk: combine the G received partial chunks, store it into every member's slot
    mine, decl1, stride1 = _gathered_view(lw, st, oi1, dirn, pdt)
    decls = [decl1]
    outs = []
    for m in range(G):
        v = _slot_view(f"cm_ag{m}", pdt, st.slot_bytes // pdt.bytes)
        decls.append(L.PtrDeclStmt(lw.ctx.flat_of(v), _ext("tl::mesh::slot", [
            st.mctx, _ext("tl::mesh::group_member", [st.mctx, dirn, st.rank, m]), st.blk, oi2, st.rank], _dt.handle)))
        outs.append(v)
    j = _V("cmj")
    acc = BufferLoad(mine, [j])
    for m in range(1, G):
        from ..transform.lower_tile_op import _combine
        acc = _combine(kind, acc, BufferLoad(mine, [binop("+", j, m * stride1)]))
    rv = _V("cmv", pdt)
    body = S.seq(S.LetStmt(rv, acc), *[S.StoreStmt(v, [j], rv) for v in outs])
    decls.append(lw.lower_nest(S.ForStmt(j, 0, c, "parallel", body), None))
    out.append(_scoped(decls))
    kk = _V("cmk")
    out.append(S.ForStmt(kk, 0, G, "serial", L.CallStmt("tl::mesh::publish", [
        st.mctx, st.blk, oi2, _ext("tl::mesh::group_member", [st.mctx, dirn, st.rank, kk]), tag2])))
    out.append(_wait_data_loop(st, oi2, tag2, dirn, G))
    # every chunk, reduced by its owner, gathered into dst
    allv, decl2, stride2 = _gathered_view(lw, st, oi2, dirn, pdt)
    dst = op.dst
    ddt = dst.buffer.dtype

    def mk(idx, q, _):
        val = BufferLoad(allv, [binop("+", binop("*", binop("//", q, c), stride2), binop("%", q, c))])
        if not op.clear:
            val = _combine2(kind, BufferLoad(dst.buffer, idx), val)
        return S.StoreStmt(dst.buffer, idx, cast(val, ddt))

    out.append(_scoped([decl2, _nest(lw, dst, mk)]))
    return _scoped(out)


def _combine2(kind, a, b):
    from ..transform.lower_tile_op import _combine
    return _combine(kind, a, b)


def _gather_phases(lw, st, oi, tag, src: BufferRegion, size: int, dirn: int):
    G = _group_size(st, dirn)
    return [_post_ready_loop(st, oi, tag, dirn, G),
            _send_loop(lw, st, oi, tag, src, size, st.rank, dirn, G, src.buffer.dtype),
            _wait_data_loop(st, oi, tag, dirn, G)]


def _gathered_view(lw, st, oi, dirn, dtype):
    """Flat view whose element ``k*stride + i`` is element i of group member k's slot."""
    G = _group_size(st, dirn)
    per = st.slot_bytes // dtype.bytes
    stride = _member_stride(st, dirn) * per
    view = _slot_view("cm_all", dtype, stride * (G - 1) + per)
    first = _ext("tl::mesh::group_member", [st.mctx, dirn, st.rank, 0])
    decl = L.PtrDeclStmt(lw.ctx.flat_of(view), _ext("tl::mesh::slot", [st.mctx, st.rank, st.blk, oi, first],
                                                    _dt.handle))
    return view, decl, stride


def lower_all_gather(lw, op: O.CommAllGatherOp):
    st = mesh_state(lw.ctx, op.mesh)
    cpu = lw.ctx.is_cpu
    _check_region(op.send, "all_gather", cpu)
    _check_region(op.recv, "all_gather", cpu)
    dirn = DIR[op.direction]
    oi, tag, out = _begin(st, "all_gather")
    out += _gather_phases(lw, st, oi, tag, op.send, op.size, dirn)
    view, decl, stride = _gathered_view(lw, st, oi, dirn, op.send.buffer.dtype)
    out.append(_scoped([decl, _read_nest(lw, op.recv, view, op.size, lead_stride=stride)]))
    return _scoped(out)


_COMBINE = {"sum": "sum", "abssum": "sum", "max": "max", "absmax": "max", "min": "min", "bitand": "bitand",
            "bitor": "bitor", "bitxor": "bitxor"}


def lower_all_reduce(lw, op: O.CommAllReduceOp):
    from ..transform.lower_tile_op import _combine
    st = mesh_state(lw.ctx, op.mesh)
    cpu = lw.ctx.is_cpu
    tile = op.dim is None  # all_reduce_tile: element-wise across cores, no local reduce
    if op.tmp is None and not tile:
        raise CommLoweringError("T.comm.all_reduce without a partial buffer")
    _check_region(op.src, "all_reduce", cpu)
    _check_region(op.dst, "all_reduce", cpu)
    dirn = DIR[op.direction]
    oi, tag, out = _begin(st, "all_reduce_tile" if tile else "all_reduce")
    part = op.src if tile else op.tmp
    if not tile:
        # 1) local reduce along dim into the partial
        out.append(lw.lower_ReduceOp(O.ReduceOp(op.src, op.tmp, op.reduce_type, op.dim, True)))
    n = 1
    for e in part.static_extents():
        n *= e
    G = _group_size(st, dirn)
    if _two_shot(op, n, G):
        return _lower_all_reduce_two_shot(lw, st, op, part, n, dirn, _COMBINE[op.reduce_type], out)
    # 2) all-gather the partials into the workspace
    out += _gather_phases(lw, st, oi, tag, part, n, dirn)
    # 3) combine in member (core-id) order — identical on every rank
    view, decl, stride = _gathered_view(lw, st, oi, dirn, op.dst.buffer.dtype)
    G = _group_size(st, dirn)
    kind = _COMBINE[op.reduce_type]
    dst = op.dst
    ddt = dst.buffer.dtype

    def mk(idx, q, _):
        acc = BufferLoad(view, [q])
        for k in range(1, G):
            acc = _combine(kind, acc, BufferLoad(view, [binop("+", q, k * stride)]))
        if not op.clear:
            acc = _combine(kind, BufferLoad(dst.buffer, idx), acc)
        return S.StoreStmt(dst.buffer, idx, cast(acc, ddt))

    out.append(_scoped([decl, _nest(lw, dst, mk)]))
    return _scoped(out)


def lower_barrier(lw, op: O.CommBarrierOp):
    st = mesh_state(lw.ctx, op.mesh)
    members = list(op.group) if op.group is not None else list(range(st.nranks))
    oi, tag, out = _begin(st, "barrier")
    body = [L.CallStmt("tl::mesh::barrier_arrive", [])]
    body += [L.CallStmt("tl::mesh::barrier_post", [st.mctx, st.blk, oi, p, tag]) for p in members]
    body += [L.CallStmt("tl::mesh::barrier_wait", [st.mctx, st.blk, oi, p, tag]) for p in members]
    if op.group is None:
        out += body
    else:
        cond = None
        for p in members:
            c = binop("==", st.rank, p)
            cond = c if cond is None else binop("||", cond, c)
        out.append(S.IfStmt(cond, _scoped(body)))
    return _scoped(out)


def lower_fence(lw, op: O.CommFenceOp):
    mesh_state(lw.ctx, op.mesh)
    return L.CallStmt("tl::mesh::fence", [])


def lower_comm(lw, op):
    fn = {O.CommBroadcastOp: lower_broadcast, O.CommPutOp: lower_put, O.CommAllGatherOp: lower_all_gather,
          O.CommAllReduceOp: lower_all_reduce, O.CommBarrierOp: lower_barrier, O.CommFenceOp: lower_fence}[type(op)]
    return fn(lw, op)
