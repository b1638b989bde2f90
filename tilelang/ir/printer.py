"""Deterministic text printer for the tile IR (used by golden tests and the cache key).

Plays the role of TVM's ``func.script()`` that the reference's IR tests compare
against (e.g. ``testing/python/language/test_tilelang_language_comm.py:48``).
"""
from __future__ import annotations

from .expr import (BinOp, BufferLoad, Call, Cast, FloatImm, IntImm, PrimExpr, Select, StringImm, UnOp, Var)
from . import stmt as S
from .buffer import Buffer, BufferRegion

_PREC = {
    "||": 1, "&&": 2, "|": 3, "^": 4, "&": 5, "==": 6, "!=": 6, "<": 7, "<=": 7, ">": 7, ">=": 7,
    "<<": 8, ">>": 8, "+": 9, "-": 9, "*": 10, "/": 10, "//": 10, "%": 10
}


class _Names:

    def __init__(self):
        self.map = {}
        self.used = {}

    def __call__(self, obj, base):
        k = id(obj)
        if k in self.map:
            return self.map[k][1]
        n = self.used.get(base, 0)
        self.used[base] = n + 1
        name = base if n == 0 else f"{base}_{n}"
        self.map[k] = (obj, name)  # keep obj alive so ids are not reused
        return name


class Printer:

    def __init__(self):
        self.names = _Names()
        self.lines = []
        self.indent = 0

    # -- expressions --------------------------------------------------------------
    def e(self, x, prec=0) -> str:
        if isinstance(x, bool):
            return "True" if x else "False"
        if isinstance(x, (int, float)):
            return repr(x)
        if isinstance(x, Buffer):
            return self.names(x, x.name)
        if isinstance(x, BufferRegion):
            return self.region(x)
        if isinstance(x, str):
            return repr(x)
        if isinstance(x, (list, tuple)):
            return "[" + ", ".join(self.e(i) for i in x) + "]"
        if not isinstance(x, PrimExpr):
            return repr(x)
        if isinstance(x, IntImm):
            if x.dtype.is_bool:
                return "True" if x.value else "False"
            return str(x.value) if x.dtype.name in ("int32", "int64") else f"T.{x.dtype.name}({x.value})"
        if isinstance(x, FloatImm):
            return repr(x.value) if x.dtype.name == "float32" else f"T.{x.dtype.name}({x.value!r})"
        if isinstance(x, StringImm):
            return repr(x.value)
        if isinstance(x, Var):
            return self.names(x, x.name)
        if isinstance(x, BinOp):
            if x.op in ("min", "max"):
                return f"T.{x.op}({self.e(x.a)}, {self.e(x.b)})"
            p = _PREC[x.op]
            op = {"&&": "and", "||": "or"}.get(x.op, x.op)
            s = f"{self.e(x.a, p)} {op} {self.e(x.b, p + 1)}"
            return f"({s})" if p < prec else s
        if isinstance(x, UnOp):
            return f"not {self.e(x.a, 11)}" if x.op == "!" else f"~{self.e(x.a, 11)}"
        if isinstance(x, Cast):
            return f"T.Cast({x.dtype.name!r}, {self.e(x.value)})"
        if isinstance(x, Select):
            return f"T.if_then_else({self.e(x.cond)}, {self.e(x.t)}, {self.e(x.f)})"
        if isinstance(x, Call):
            args = ", ".join(self.e(a) for a in x.args)
            if x.attrs.get("memory_order"):
                args += f", memory_order={x.attrs['memory_order']!r}"
            return f"T.{x.op}({args})"
        if isinstance(x, BufferLoad):
            return f"{self.names(x.buffer, x.buffer.name)}[{', '.join(self.e(i) for i in x.indices)}]"
        return repr(x)

    def region(self, r: BufferRegion) -> str:
        parts = []
        for m, ext in r.region:
            if isinstance(ext, int) and ext == 1:
                parts.append(self.e(m))
            else:
                parts.append(f"{self.e(m)}:{self.e(m + ext)}")
        return f"{self.names(r.buffer, r.buffer.name)}[{', '.join(parts)}]"

    # -- statements ----------------------------------------------------------------
    def w(self, line):
        self.lines.append("    " * self.indent + line)

    def body(self, s):
        self.indent += 1
        if s is None or (isinstance(s, S.SeqStmt) and not s.stmts):
            self.w("pass")
        else:
            self.s(s)
        self.indent -= 1

    def s(self, s):
        if isinstance(s, S.SeqStmt):
            for c in s.stmts:
                self.s(c)
        elif isinstance(s, S.KernelStmt):
            grid = ", ".join(self.e(g) for g in s.grid)
            bv = ", ".join(self.e(v) for v in s.block_vars)
            thr = s.threads[0] if len(s.threads) == 1 else list(s.threads)
            extra = ", is_cpu=True" if s.is_cpu else ""
            self.w(f"with T.Kernel({grid}, threads={thr}{extra}) as ({bv}):")
            self.body(s.body)
        elif isinstance(s, S.ForStmt):
            kind = {"serial": "T.serial", "parallel": "T.Parallel", "pipelined": "T.Pipelined",
                    "unroll": "T.unroll", "vectorized": "T.vectorized", "persistent": "T.Persistent"}[s.kind]
            ann = ""
            for k in sorted(s.annotations):
                v = s.annotations[k]
                if k.startswith("_"):
                    continue
                ann += f", {k}={self.e(v) if isinstance(v, (PrimExpr, list, tuple)) else v!r}"
            rng = self.e(s.extent) if (isinstance(s.min, IntImm) and s.min.value == 0) else \
                f"{self.e(s.min)}, {self.e(s.min + s.extent)}"
            self.w(f"for {self.e(s.var)} in {kind}({rng}{ann}):")
            self.body(s.body)
        elif isinstance(s, S.WhileStmt):
            self.w(f"while {self.e(s.cond)}:")
            self.body(s.body)
        elif isinstance(s, S.IfStmt):
            self.w(f"if {self.e(s.cond)}:")
            self.body(s.then_body)
            if s.else_body is not None:
                self.w("else:")
                self.body(s.else_body)
        elif isinstance(s, S.StoreStmt):
            idx = ", ".join(self.e(i) for i in s.indices)
            self.w(f"{self.names(s.buffer, s.buffer.name)}[{idx}] = {self.e(s.value)}")
        elif isinstance(s, S.EvaluateStmt):
            self.w(f"T.evaluate({self.e(s.expr)})")
        elif isinstance(s, S.LetStmt):
            self.w(f"{self.e(s.var)}: T.{s.var.dtype.name} = {self.e(s.value)}")
        elif isinstance(s, S.AllocStmt):
            b = s.buffer
            shape = "[" + ", ".join(self.e(x) for x in b.shape) + "]"
            fn = {"shared": "alloc_shared", "fragment": "alloc_fragment", "local": "alloc_local",
                  "var": "alloc_var"}.get(b.scope, "alloc_buffer")
            if b.scope == "var":
                self.w(f"{self.names(b, b.name)} = T.alloc_var({b.dtype.name!r})")
            else:
                self.w(f"{self.names(b, b.name)} = T.{fn}({shape}, {b.dtype.name!r})")
            if getattr(b, "layout_annotated", False) and b.layout is not None:
                # user layouts change the generated code: they belong in the printed program
                # (and therefore in the kernel-cache key)
                self.w(f"T.annotate_layout({{{self.names(b, b.name)}: {_layout_key(b.layout)}}})")
        elif isinstance(s, S.TileOpStmt):
            self.w(self.tileop(s.op))
        elif isinstance(s, S.BreakStmt):
            self.w("T.loop_break()")
        elif isinstance(s, S.ContinueStmt):
            self.w("continue")
        elif isinstance(s, S.AssertStmt):
            self.w(f"T.device_assert({self.e(s.cond)}, {s.msg!r})")
        elif isinstance(s, S.AttrStmt):
            self.w(f"T.attr({s.key!r}, {self.e(s.value)})")
            if s.body is not None:
                self.s(s.body)
        elif isinstance(s, S.RawStmt):
            for ln in s.code.splitlines():
                self.w(f"# raw: {ln}")
        else:
            self.w(f"<{type(s).__name__}>")

    def tileop(self, op) -> str:
        k = op.kind
        from . import tileop as O
        if isinstance(op, O.CopyOp):
            return f"T.copy({self.region(op.src)}, {self.region(op.dst)})"
        if isinstance(op, O.GemmOp):
            extra = ""
            if op.trans_A:
                extra += ", transpose_A=True"
            if op.trans_B:
                extra += ", transpose_B=True"
            if op.policy:
                extra += f", policy={op.policy}"
            if op.clear_accum is not False:
                extra += f", clear_accum={self.e(op.clear_accum)}"
            if op.k_pack != 1:
                extra += f", k_pack={op.k_pack}"
            if getattr(op, "mfma_shape", None):
                extra += f", mfma_shape={op.mfma_shape!r}"
            if getattr(op, "valid_m", None) is not None:
                extra += f", valid_m={self.e(op.valid_m)}"
            if getattr(op, "valid_m_min", None) is not None:
                extra += f", valid_m_min={self.e(op.valid_m_min)}"
            if getattr(op, "is_mx", False):
                return (f"T.gemm_scaled({self.region(op.A)}, {self.region(op.B)}, {self.region(op.C)}, "
                        f"{self.region(op.scale_A)}, {self.region(op.scale_B)}{extra}, a_format={op.a_fmt!r}, "
                        f"b_format={op.b_fmt!r})")
            if getattr(op, "is_sp", False):
                return (f"T.gemm_sp({self.region(op.A)}, {self.region(op.E)}, {self.region(op.B)}, "
                        f"{self.region(op.C)}{extra})")
            return f"T.gemm({self.region(op.A)}, {self.region(op.B)}, {self.region(op.C)}{extra})"
        if isinstance(op, O.FillOp):
            return f"T.fill({self.region(op.dst)}, {self.e(op.value)})"
        if isinstance(op, O.ReduceOp):
            return (f"T.reduce_{op.reduce_type}({self.region(op.src)}, {self.region(op.dst)}, dim={op.dim}, "
                    f"clear={op.clear})")
        if isinstance(op, O.CumSumOp):
            return f"T.cumsum({self.region(op.src)}, {self.region(op.dst)}, dim={op.dim}, reverse={op.reverse})"
        if isinstance(op, O.AtomicOp):
            src = self.region(op.src) if isinstance(op.src, BufferRegion) else self.e(op.src)
            return f"T.atomic_{op.op}({self.region(op.dst)}, {src})"
        if isinstance(op, O.FinalizeReducerOp):
            return f"T.finalize_reducer({self.region(op.buf)})"
        if isinstance(op, O.CommOp):
            # the mesh shape an op was traced for changes its lowering (group sizes, two-shot
            # chunking): part of the printed IR, i.e. of the kernel-cache key
            txt = self._comm(op)
            return txt[:-1] + f", mesh={op.mesh!r})"
        if isinstance(op, O.GatherRowsOp):
            return (f"T.gather_rows({self.region(op.src)}, {self.region(op.idx)}, {self.region(op.dst)}, "
                    f"row_dim={op.row_dim})")
        return f"T.{k}({self._generic_args(op)})"

    def _comm(self, op) -> str:
        from . import tileop as O
        if isinstance(op, O.CommBroadcastOp):
            return (f"T.comm.broadcast({self.region(op.src)}, {self.region(op.dst)}, {self.e(op.src_core)}, "
                    f"direction={op.direction!r}, size={op.size})")
        if isinstance(op, O.CommPutOp):
            return (f"T.comm.put({self.region(op.src)}, {self.region(op.dst)}, {self.e(op.src_core)}, "
                    f"{self.e(op.dst_core)}, size={op.size})")
        if isinstance(op, O.CommAllGatherOp):
            return (f"T.comm.all_gather({self.region(op.send)}, {self.region(op.recv)}, "
                    f"direction={op.direction!r}, size={op.size})")
        if isinstance(op, O.CommAllReduceOp):
            return (f"T.comm.all_reduce({self.region(op.src)}, {self.region(op.dst)}, {op.reduce_type!r}, "
                    f"direction={op.direction!r}, dim={op.dim}, clear={op.clear})")
        if isinstance(op, O.CommBarrierOp):
            return f"T.comm.barrier({op.group!r})"
        if isinstance(op, O.CommFenceOp):
            return "T.comm.fence()"
        return f"T.comm.{op.kind}({self._generic_args(op)})"

    def _generic_args(self, op) -> str:
        """Every attribute of a tile op (regions, expressions, constants): the printed IR is the
        kernel-cache key, so nothing that changes the generated code may be left out."""
        parts = []
        for name in sorted(vars(op)):
            if name.startswith("_") or name == "plan":
                continue
            v = getattr(op, name)
            if isinstance(v, BufferRegion):
                parts.append(f"{name}={self.region(v)}")
            elif hasattr(v, "dtype") and not isinstance(v, (int, float, str)):
                try:
                    parts.append(f"{name}={self.e(v)}")
                except Exception:  # noqa: BLE001
                    parts.append(f"{name}={v!r}")
            elif isinstance(v, (int, float, str, bool, tuple, list, type(None))):
                parts.append(f"{name}={v!r}")
            else:
                parts.append(f"{name}={type(v).__name__}")
        return ", ".join(parts)

    def func(self, f: S.PrimFunc) -> str:
        params = []
        for p in f.params:
            if isinstance(p, Buffer):
                shape = "(" + ", ".join(self.e(x) for x in p.shape) + ("," if len(p.shape) == 1 else "") + ")"
                if p.strides is not None:  # T.StridedTensor: the strides are part of the program
                    st = "(" + ", ".join(self.e(x) for x in p.strides) + ("," if len(p.strides) == 1 else "") + ")"
                    params.append(f"{self.names(p, p.name)}: T.StridedTensor({shape}, {st}, {p.dtype.name!r})")
                else:
                    params.append(f"{self.names(p, p.name)}: T.Tensor({shape}, {p.dtype.name!r})")
            else:
                params.append(f"{self.e(p)}: T.{p.dtype.name}")
        self.w("@T.prim_func")
        self.w(f"def {f.name}({', '.join(params)}):")
        self.body(f.body)
        return "\n".join(self.lines)


def expr_str(e) -> str:
    return Printer().e(e)


def stmt_str(s) -> str:
    p = Printer()
    p.s(s)
    return "\n".join(p.lines)


def func_str(f) -> str:
    return Printer().func(f)


def _layout_key(layout) -> str:
    """Printable identity of a layout.  Subclasses carry a complete ``signature()``; a generic
    callable-defined ``Layout`` is identified by its index map sampled over (a prefix of) its
    domain, since two lambdas of the same shape would otherwise print alike."""
    from ..layout.layout import Layout
    sig = layout.signature() if hasattr(layout, "signature") else repr(layout)
    if type(layout) is not Layout:
        return repr(sig)
    import hashlib
    import itertools
    shape = [int(x) for x in layout.shape]
    h = hashlib.sha1()
    for idx in itertools.islice(itertools.product(*(range(n) for n in shape)), 8192):
        try:
            h.update(repr(layout.forward(*idx)).encode())
        except Exception:
            h.update(b"?")
    return repr(sig + (h.hexdigest()[:16],))
