"""Strength-reduce the global source addresses of LDS-DMA issues in pipelined loops.

The pipeline lowers each ``T.copy`` stage into ``tl::glds16(&A[idx], &A_s[...])`` calls whose
global index ``idx`` is an affine function of the loop variable plus a per-thread part (tile
row/column of the lane, the inverse LDS swizzle XOR-ed into the column chunk, block offsets).
hipcc does not reliably hoist that per-thread part out of the loop: in the 256x256 fp16 GEMM
it recomputed it every iteration (73 VALU per main-loop iteration against 22 in a hand-written
kernel of the same schedule; the gap cost ~4 % of the GEMM, profiles/r3/gemm_dsl_prefetch_ab.log,
VERDICT r2 "hoist the swizzled glds16 addresses").

This pass splits ``idx = c * k + rest`` for every such call inside a serial loop ``k``
(``rest`` free of ``k`` and of everything the loop body binds) and emits, before the loop,

    T* A_src0 = &A[rest];                    // once per (buffer, rest)
    ... loop: tl::glds16(&A_src0[c * k + c0], ...)

so the per-iteration cost is one scalar multiply and one 64-bit add per issue.
"""
from __future__ import annotations

from typing import Dict, List

from ..ir import stmt as S
from ..ir import lowered as L
from ..ir.buffer import Buffer
from ..ir.expr import IntImm, Var, _linear_form, binop, cast, const, free_vars, uses_var
from .utils import Mutator

_DMA = ("tl::glds16", "tl::glds4", "tl::glds16_nt")


def _bound_vars(body) -> set:
    out = set()
    for x in S.walk(body):
        if isinstance(x, S.ForStmt):
            out.add(x.var)
        elif isinstance(x, S.LetStmt):
            out.add(x.var)
        elif isinstance(x, L.AutoLetStmt):
            out.add(x.var)
    return out


class _Hoister(Mutator):

    def __init__(self):
        self.n = 0

    def visit_ForStmt(self, s):
        body = self.stmt(s.body)
        if s.kind != "serial":
            return S.ForStmt(s.var, s.min, s.extent, s.kind, body, s.annotations)
        k = s.var
        inner = _bound_vars(body)
        decls: List[S.Stmt] = []
        cache: Dict[tuple, Buffer] = {}

        def fix_call(c: L.CallStmt):
            p = c.args[0] if c.args else None
            if not isinstance(p, L.BufferPtr) or getattr(p.buffer, "scope", "") != "global":
                return c
            off = p.offset
            lf = _linear_form(off)
            if lf is None:
                return c
            coef, rest, c0 = 0, None, 0
            for key, (t, cf) in lf.items():
                if key == "__const__":
                    c0 = cf  # stays in the loop: copies that differ only by a constant share a base
                    continue
                elif t is k:
                    coef += cf
                    continue
                else:
                    if uses_var(t, k) or any(v in inner for v in free_vars(t)):
                        return c
                    term = t if cf == 1 else binop("*", t, const(cf, t.dtype))
                if term is not None:
                    rest = term if rest is None else binop("+", rest, term)
            if rest is None or isinstance(rest, (IntImm, Var)):
                return c  # nothing per-thread to hoist
            key = (id(p.buffer), repr(rest))
            nb = cache.get(key)
            if nb is None:
                self.n += 1
                nb = Buffer(f"{p.buffer.name}_src{self.n}", [1], p.buffer.dtype, "global")
                cache[key] = nb
                decls.append(L.PtrDeclStmt(nb, L.BufferPtr(p.buffer, rest)))
            kd = k if k.dtype == off.dtype else cast(k, off.dtype)
            new_off = binop("*", kd, const(coef, off.dtype)) if coef != 0 else const(0, off.dtype)
            if c0:
                new_off = binop("+", new_off, const(c0, off.dtype))
            return L.CallStmt(c.name, [L.BufferPtr(nb, new_off)] + list(c.args[1:]), c.targs)

        def walk(x):
            # calls of THIS loop's body (nested loops were handled by their own visit)
            if isinstance(x, L.CallStmt) and x.name in _DMA:
                return fix_call(x)
            if isinstance(x, S.SeqStmt):
                y = S.SeqStmt([walk(c) for c in x.stmts])
                if getattr(x, "scoped", False):
                    y.scoped = True
                return y
            if isinstance(x, S.IfStmt):
                return S.IfStmt(x.cond, walk(x.then_body), walk(x.else_body) if x.else_body is not None else None)
            return x

        body = walk(body)
        loop = S.ForStmt(s.var, s.min, s.extent, s.kind, body, s.annotations)
        return S.SeqStmt(decls + [loop]) if decls else loop


def hoist_dma_sources(kernel: S.KernelStmt) -> S.KernelStmt:
    return _Hoister().stmt(kernel)
