"""Compute analysis of an arbitrary loop-nest program (reference ``tilelang/carver/roller/node.py``
``PrimFuncNode``, ``tilelang/carver/matmul_analysis.py``, ``roller/shape_inference``).

The templates (``carver/template.py``) know their operator; this module looks at a user program
instead -- a naive ``T.prim_func`` whose body is a loop nest of scalar stores, e.g.

    for i, j, k in T.grid(M, N, K):
        C[i, j] += A[i, k] * B[j, k]

and recovers what the roller policies need:

* ``PrimFuncNode``: the compute statement, its loop nest (extents), the output buffer and index,
  every input access; axes are SPATIAL (they index the output) or REDUCE (they do not, and the
  store accumulates: ``C[..] = C[..] + ...`` or a max/min fold); ``infer_shapes`` gives each
  buffer's extent per axis (the reference's shape inference, for the affine single-variable
  indices these nests use);
* ``gemm_info``: whether the nest is a (batched) GEMM -- two multiplied inputs, one reduce axis,
  each input indexed by the reduce axis plus its own spatial axis (and a shared batch axis) --
  with M / N / K / batch extents and the operand orientations (``trans_A`` / ``trans_B``);
* ``recommend(func, arch, topk)``: GEMM-like nests go to ``TensorCorePolicy`` (MFMA tilings),
  everything else to ``DefaultPolicy`` (elementwise / reduction tiles, ``reduce_len`` from the
  reduce axes).  Convolutions written as a direct nest have more than one reduce axis and are
  reported as such (``conv_like``); their implicit-GEMM extents come from ``implicit_gemm``.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from ..ir import stmt as S
from ..ir.expr import BinOp, BufferLoad, Call, Cast, Var, as_int, free_vars, post_order


class AnalysisError(ValueError):
    pass


@dataclass
class Access:
    buffer: object
    indices: list
    is_write: bool = False

    @property
    def name(self) -> str:
        return self.buffer.name

    def axes(self) -> List[Optional[Var]]:
        """The single loop variable of each index position (None: constant or compound)."""
        out = []
        for i in self.indices:
            fv = free_vars(i)
            out.append(fv[0] if len(fv) == 1 else None)
        return out


@dataclass
class PrimFuncNode:
    func: object
    loops: List[Tuple[Var, int]] = field(default_factory=list)
    output: Optional[Access] = None
    inputs: List[Access] = field(default_factory=list)
    spatial: List[Var] = field(default_factory=list)
    reduce: List[Var] = field(default_factory=list)
    reduce_kind: Optional[str] = None   # "sum" / "max" / "min" / None (elementwise)
    store: Optional[S.StoreStmt] = None

    # -- construction ------------------------------------------------------------------------
    @staticmethod
    def from_func(func) -> "PrimFuncNode":
        node = PrimFuncNode(func)
        found = []

        def visit(s, loops):
            if s is None:
                return
            if isinstance(s, S.ForStmt):
                ext = as_int(s.extent)
                if ext is None:
                    raise AnalysisError(f"loop {s.var.name} has a non-constant extent: not analysable")
                visit(s.body, loops + [(s.var, ext)])
                return
            if isinstance(s, S.StoreStmt):
                found.append((s, loops))
                return
            for c in S.stmt_children(s):
                visit(c, loops)

        visit(func.body, [])
        stores = [(s, lp) for s, lp in found if s.buffer.scope == "global"]
        if len(stores) != 1:
            raise AnalysisError(f"expected one compute statement storing a global buffer, found {len(stores)}")
        st, loops = stores[0]
        node.store, node.loops = st, loops
        node.output = Access(st.buffer, list(st.indices), True)
        out_vars = []
        for i in st.indices:
            out_vars += free_vars(i)
        loop_vars = [v for v, _ in loops]
        node.spatial = [v for v in loop_vars if _has(out_vars, v)]
        node.reduce = [v for v in loop_vars if not _has(out_vars, v)]
        loads = [n for n in post_order(st.value) if isinstance(n, BufferLoad)]
        self_load = [ld for ld in loads if ld.buffer is st.buffer]
        node.inputs = [Access(ld.buffer, list(ld.indices)) for ld in loads if ld.buffer is not st.buffer]
        if node.reduce:
            if not self_load:
                raise AnalysisError("the nest has loop axes that do not index the output but the store does not "
                                    "accumulate (each iteration would overwrite the previous one)")
            node.reduce_kind = _fold_kind(st.value, st.buffer)
        return node

    # -- queries -----------------------------------------------------------------------------
    def extent(self, v: Var) -> int:
        for lv, e in self.loops:
            if lv is v:
                return e
        raise KeyError(v.name)

    def get_space_dim(self) -> List[int]:
        return [self.extent(v) for v in self.spatial]

    def get_reduce_dim(self) -> List[int]:
        return [self.extent(v) for v in self.reduce]

    def is_reduction(self) -> bool:
        return bool(self.reduce)

    def infer_shapes(self) -> Dict[str, List[Optional[int]]]:
        """Per buffer: the extent its index positions span over the loop nest (affine indices of one
        loop variable; None where an index is compound)."""
        out = {}
        for acc in [self.output] + self.inputs:
            dims = []
            for idx in acc.indices:
                fv = free_vars(idx)
                if not fv:
                    dims.append(1)
                elif len(fv) == 1:
                    dims.append(self.extent(fv[0]))
                else:
                    dims.append(None)
            out[acc.name] = dims
        return out

    def flops(self) -> int:
        n = 1
        for _, e in self.loops:
            n *= e
        ops = sum(1 for x in post_order(self.store.value) if isinstance(x, BinOp) and x.op in ("+", "-", "*", "/"))
        return n * max(1, ops)


def _fold_kind(value, out_buf) -> str:
    for n in post_order(value):
        if isinstance(n, BinOp) and n.op in ("+", "-") and any(isinstance(c, BufferLoad) and c.buffer is out_buf
                                                                for c in (n.a, n.b)):
            return "sum"
        if isinstance(n, Call) and n.op in ("max", "min") and any(
                isinstance(c, BufferLoad) and c.buffer is out_buf for c in n.args):
            return n.op
        if isinstance(n, BinOp) and n.op in ("max", "min") and any(
                isinstance(c, BufferLoad) and c.buffer is out_buf for c in (n.a, n.b)):
            return n.op
    return "sum"


@dataclass
class GemmInfo:
    M: int
    N: int
    K: int
    batch: int
    trans_A: bool
    trans_B: bool
    A: str
    B: str
    C: str
    in_dtype: str
    out_dtype: str


def _has(seq, v) -> bool:
    return any(x is v for x in seq)


def _index(seq, v) -> int:
    for i, x in enumerate(seq):
        if x is v:
            return i
    raise ValueError(v)


def _uniq(seq) -> list:
    out = []
    for x in seq:
        if not _has(out, x):
            out.append(x)
    return out


def _strip(e):
    while isinstance(e, Cast):
        e = e.value
    return e


def gemm_info(node: PrimFuncNode) -> Optional[GemmInfo]:
    """GEMM / batched GEMM recognition (reference ``matmul_analysis.py`` ``get_index_map`` /
    ``is_gemm_like``).  None when the nest is not one."""
    if len(node.reduce) != 1 or node.reduce_kind != "sum" or len(node.inputs) != 2:
        return None
    k = node.reduce[0]
    # the accumulated term must be a product of the two loads
    prod = None
    for n in post_order(node.store.value):
        if isinstance(n, BinOp) and n.op == "*":
            a, b = _strip(n.a), _strip(n.b)
            if isinstance(a, BufferLoad) and isinstance(b, BufferLoad):
                prod = (a, b)
    if prod is None:
        return None
    A, B = (Access(x.buffer, list(x.indices)) for x in prod)
    ax_a, ax_b, ax_c = A.axes(), B.axes(), node.output.axes()
    if any(x is None for x in ax_a + ax_b + ax_c) or not _has(ax_a, k) or not _has(ax_b, k):
        return None
    sa = [v for v in _uniq(ax_a) if v is not k]
    sb = [v for v in _uniq(ax_b) if v is not k]
    shared = [v for v in sa if _has(sb, v)]
    m_ax = [v for v in sa if not _has(shared, v)]
    n_ax = [v for v in sb if not _has(shared, v)]
    if len(m_ax) != 1 or len(n_ax) != 1:
        return None
    m, n = m_ax[0], n_ax[0]
    want = shared + [m, n]
    got = _uniq(ax_c)
    if len(got) != len(want) or not all(_has(want, v) for v in got):
        return None
    batch = 1
    for v in shared:
        batch *= node.extent(v)
    # orientation from the index positions: A [.., M, K] is "not transposed"
    trans_a = _index(ax_a, k) < _index(ax_a, m)
    trans_b = _index(ax_b, k) > _index(ax_b, n)  # B [.., N, K] = transpose_B (the MFMA-friendly layout)
    return GemmInfo(M=node.extent(m), N=node.extent(n), K=node.extent(k), batch=batch, trans_A=trans_a,
                    trans_B=trans_b, A=A.name, B=B.name, C=node.output.name, in_dtype=str(A.buffer.dtype),
                    out_dtype=str(node.output.buffer.dtype))


def implicit_gemm(node: PrimFuncNode) -> Optional[Tuple[int, int, int]]:
    """(M, N, K) of a multi-reduce-axis product nest (a direct convolution) read as an implicit GEMM:
    K = product of the reduce extents; N = the spatial axes that index the product's second
    operand (the filter); M = the other spatial axes."""
    if len(node.reduce) < 2 or node.reduce_kind != "sum" or len(node.inputs) != 2:
        return None
    K = 1
    for e in node.get_reduce_dim():
        K *= e
    w = node.inputs[1]
    w_vars = []
    for i in w.indices:
        w_vars += free_vars(i)
    N = 1
    M = 1
    for v in node.spatial:
        if _has(w_vars, v):
            N *= node.extent(v)
        else:
            M *= node.extent(v)
    return M, N, K


def recommend(func, arch=None, topk: int = 10):
    """Ranked ``Hint``s for an arbitrary loop-nest program; also returns what was recognised:
    (hints, {"kind": "gemm" | "conv_like" | "reduction" | "elementwise", ...})."""
    from .arch import CDNA
    from .roller.policy import DefaultPolicy, TensorCorePolicy
    arch = arch or CDNA("hip")
    node = PrimFuncNode.from_func(func)
    g = gemm_info(node)
    if g is not None:
        M = g.M * g.batch if g.batch > 1 else g.M
        hints = TensorCorePolicy(arch, M, g.N, g.K, g.in_dtype, g.trans_B).emit_config(topk)
        return hints, {"kind": "gemm", "gemm": g}
    ig = implicit_gemm(node)
    if ig is not None:
        M, N, K = ig
        dt = str(node.inputs[0].buffer.dtype)
        return TensorCorePolicy(arch, M, N, K, dt, True).emit_config(topk), {"kind": "conv_like", "mnk": ig}
    dt = str(node.output.buffer.dtype)
    space = node.get_space_dim() or [1]
    if node.is_reduction():
        red = 1
        for e in node.get_reduce_dim():
            red *= e
        return DefaultPolicy(arch, space, dt, reduce_len=red).emit_config(topk), {"kind": "reduction",
                                                                                 "reduce_len": red}
    return DefaultPolicy(arch, space, dt).emit_config(topk), {"kind": "elementwise", "shape": space}
