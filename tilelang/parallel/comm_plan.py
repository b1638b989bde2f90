"""Communication schedules of the T.comm ops.

Two views of the same op:

``reference_schedule(op)`` — the routing the reference fork emits for a 2-D mesh (chains of
    ``broadcast_(src, dst, size, src_core, direction[, mask...])`` along rows/columns,
    ``src/op/comm.cc`` :121-218 broadcast, :259-385 put, :479-598 all_gather, :783-919
    all_reduce).  Kept for inspection, for parity tests against the reference's lowering
    tests, and as documentation of what a mesh-routed fabric would do.  It reproduces the
    reference faithfully, including its two-hop ``put`` whose intermediate core is
    ``src_row*ncol + dst_col`` although hop 1 travels vertically.

``xgmi_transfers(op)`` — what this framework executes on MI355X: every GPU pair has its own
    xGMI link, so each op is a set of direct ``src -> dst`` tile transfers (no hops), with the
    destination slot each lands in.  ``comm_lower`` generates exactly these.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple

from ..ir import tileop as O

H, V, ALL = 0, 1, 2
_DIR = {"h": H, "v": V, "all": ALL}


@dataclass
class Broadcast_:
    """One reference ``tl.broadcast_`` call."""
    src: str                 # "src" / "dst" / "partial" / "gather": which buffer is read
    src_offset: int          # element offset into the read buffer
    dst: str
    dst_offset: int
    size: int                # elements
    core: int                # broadcasting core
    direction: int           # 0 horizontal, 1 vertical
    mask: List[int] = field(default_factory=list)  # excluded row/col indices (put)

    def as_tuple(self):
        return (self.src, self.src_offset, self.dst, self.dst_offset, self.size, self.core, self.direction,
                tuple(self.mask))


def _numel(region) -> int:
    n = 1
    for e in region.static_extents():
        n *= e
    return n


def reference_schedule(op, nrow: int, ncol: int) -> List[Broadcast_]:
    if isinstance(op, O.CommBroadcastOp):
        n = _numel(op.src)
        size = op.size
        d = _DIR[op.direction]
        if d in (H, V):
            return [Broadcast_("src", 0, "dst", 0, size, op.src_core, d)]
        out = [Broadcast_("src", 0, "dst", 0, size, op.src_core, V)]
        col = op.src_core % ncol
        out += [Broadcast_("dst", 0, "dst", 0, size, i * ncol + col, H) for i in range(nrow)]
        return out
    if isinstance(op, O.CommPutOp):
        s, t = op.src_core, op.dst_core
        sx, sy, tx, ty = s // ncol, s % ncol, t // ncol, t % ncol
        if sx == tx:
            return [Broadcast_("src", 0, "dst", 0, op.size, s, H, [j for j in range(ncol) if j != ty])]
        if sy == ty:
            return [Broadcast_("src", 0, "dst", 0, op.size, s, V, [i for i in range(nrow) if i != tx])]
        inter = sx * ncol + ty
        return [Broadcast_("src", 0, "dst", 0, op.size, s, V, [i for i in range(nrow) if i != tx]),
                Broadcast_("dst", 0, "dst", 0, op.size, inter, H, [j for j in range(ncol) if j != ty])]
    if isinstance(op, O.CommAllGatherOp):
        n = _numel(op.send)
        size = op.size
        d = _DIR[op.direction]
        out = []
        if d == H:
            for i in range(nrow):
                for j in range(ncol):
                    out.append(Broadcast_("send", 0, "recv", j * n, size, i * ncol + j, H))
        elif d == V:
            for j in range(ncol):
                for i in range(nrow):
                    out.append(Broadcast_("send", 0, "recv", i * n, size, i * ncol + j, V))
        else:
            for i in range(nrow):
                for j in range(ncol):
                    out.append(Broadcast_("send", 0, "recv", (i * ncol + j) * n, size, i * ncol + j, H))
            for j in range(ncol):
                for i in range(nrow):
                    out.append(Broadcast_("recv", i * ncol * n, "recv", i * ncol * n, size * ncol, i * ncol + j, V))
        return out
    if isinstance(op, O.CommAllReduceOp):
        n = _numel(op.dst)
        d = _DIR[op.direction]
        out = []
        if d in (H, ALL):
            for i in range(nrow):
                for j in range(ncol):
                    out.append(Broadcast_("partial", 0, "row_gather", j * n, n, i * ncol + j, H))
        if d in (V, ALL):
            src = "row_reduced" if d == ALL else "partial"
            for j in range(ncol):
                for i in range(nrow):
                    out.append(Broadcast_(src, 0, "col_gather", i * n, n, i * ncol + j, V))
        return out
    return []


@dataclass
class Transfer:
    src: int
    dst: int
    slot: int          # destination slot (== src core); all_gather slice index is the member rank
    elements: int


def _group(d: int, anchor: int, nrow: int, ncol: int) -> List[int]:
    if d == H:
        r = anchor // ncol
        return [r * ncol + j for j in range(ncol)]
    if d == V:
        c = anchor % ncol
        return [i * ncol + c for i in range(nrow)]
    return list(range(nrow * ncol))


def xgmi_transfers(op, nrow: int, ncol: int) -> List[Transfer]:
    if isinstance(op, O.CommBroadcastOp):
        return [Transfer(op.src_core, m, op.src_core, op.size)
                for m in _group(_DIR[op.direction], op.src_core, nrow, ncol)]
    if isinstance(op, O.CommPutOp):
        return [Transfer(op.src_core, op.dst_core, op.src_core, op.size)]
    if isinstance(op, (O.CommAllGatherOp, O.CommAllReduceOp)):
        d = _DIR[op.direction]
        n = op.size if isinstance(op, O.CommAllGatherOp) else _numel(op.dst)
        out = []
        for s in range(nrow * ncol):
            for m in _group(d, s, nrow, ncol):
                out.append(Transfer(s, m, s, n))
        return out
    return []


def transfer_bytes(op, nrow: int, ncol: int, elem_bytes: int) -> Tuple[int, int]:
    """(bytes over xGMI links, bytes copied locally) for one block instance of the op."""
    remote = local = 0
    for t in xgmi_transfers(op, nrow, ncol):
        if t.src == t.dst:
            local += t.elements * elem_bytes
        else:
            remote += t.elements * elem_bytes
    return remote, local
