"""``tl.force_let_inline``: substitute every kernel-level let binding into its uses
(reference ``tilelang/transform/simplify.py`` ``LetInline``, enabled by the same pass config).

A ``LetStmt`` binds ``var = value`` for the rest of its enclosing block; the pass walks each
statement sequence, drops the binding and rewrites the following statements with the value
substituted (transitively, so a let that uses an earlier let is expanded too)."""
from __future__ import annotations

from ..ir import stmt as S
from ..ir.expr import substitute
from .utils import Mutator, subst_stmt


class _LetInliner(Mutator):

    def visit_SeqStmt(self, s: S.SeqStmt):
        out = []
        vmap = {}
        for c in s.stmts:
            if vmap:
                c = subst_stmt(c, vmap)
            if isinstance(c, S.LetStmt):
                vmap[c.var] = substitute(c.value, vmap) if vmap else c.value
                continue
            out.append(self.stmt(c))
        ns = S.SeqStmt(out)
        if getattr(s, "scoped", False):
            ns.scoped = True
        return ns


def inline_lets(kernel: S.KernelStmt) -> S.KernelStmt:
    return _LetInliner().stmt(kernel)
