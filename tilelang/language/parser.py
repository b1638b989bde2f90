"""``@T.prim_func`` / ``@T.macro``: AST rewrite + traced execution.

The reference parses kernel bodies with TVMScript (``tilelang/language/parser``)
or rewrites them with ``DSLMutator`` (``tilelang/language/v2/ast.py:251-575``).
This frontend does the latter for every kernel: the body's AST is rewritten so
that control flow over *symbolic* values becomes IR frames, while Python-level
meta-programming (static ``if``, list iteration, helper calls) still runs as
Python.  The rewritten function is then executed once under a ``Builder``.

Rewrites:
  ``if c:``            -> static branch when ``c`` is a Python value, else ``T.If``/``T.Else``
  ``while c:``         -> static Python loop, else ``T.While``
  ``for i in range()`` -> ``T.serial`` loop
  ``a and b`` / ``not`` -> IR logical ops when symbolic (short-circuit kept for static)
  ``x = v``            -> store when ``x`` is a ``T.alloc_var``; ``LetStmt`` for loaded values
  ``break/continue``   -> ``T.loop_break`` / continue inside IR loops
"""
from __future__ import annotations

import ast
import functools
import inspect
import sys
import textwrap
from typing import Any, Dict, List, Optional

from ..ir import stmt as S
from ..ir.buffer import Buffer
from ..ir.expr import Var, PrimExpr
from ..ir import dtypes as _dt
from .builder import HELPERS, building

_IR_LOOP_FUNCS = {"range", "serial", "Parallel", "Pipelined", "unroll", "Serial", "Unroll", "Persistent",
                  "vectorized", "grid", "Vectorized"}


class _Rewriter(ast.NodeTransformer):

    def __init__(self):
        self.counter = 0
        self.loop_kinds: List[bool] = []  # True if IR loop

    def _tmp(self):
        self.counter += 1
        return f"__tl_c{self.counter}"

    # do not descend into nested function definitions (macros rewrite themselves)
    def visit_FunctionDef(self, node):
        return node

    visit_AsyncFunctionDef = visit_FunctionDef

    def visit_Lambda(self, node):
        return node

    def visit_ClassDef(self, node):
        return node

    @staticmethod
    def _call(func_attr: str, args, keywords=None):
        return ast.Call(func=ast.Attribute(value=ast.Name(id="__tl__", ctx=ast.Load()), attr=func_attr,
                                           ctx=ast.Load()), args=args, keywords=keywords or [])

    def visit_If(self, node: ast.If):
        test = self.visit(node.test)
        body = [self.visit(s) for s in node.body]
        orelse = [self.visit(s) for s in node.orelse]
        body = _flatten(body)
        orelse = _flatten(orelse)
        tmp = self._tmp()
        assign = ast.Assign(targets=[ast.Name(id=tmp, ctx=ast.Store())], value=test)
        static_if = ast.If(test=ast.Name(id=tmp, ctx=ast.Load()), body=body or [ast.Pass()], orelse=orelse)
        dyn = [
            ast.With(items=[ast.withitem(context_expr=self._call("If", [ast.Name(id=tmp, ctx=ast.Load())]))],
                     body=_copy_stmts(body) or [ast.Pass()])
        ]
        if orelse:
            dyn.append(ast.With(items=[ast.withitem(context_expr=self._call("Else", []))],
                                body=_copy_stmts(orelse)))
        outer = ast.If(test=self._call("is_static", [ast.Name(id=tmp, ctx=ast.Load())]),
                       body=[static_if], orelse=dyn)
        return [assign, outer]

    def visit_While(self, node: ast.While):
        import copy
        orig_body = _copy_stmts(node.body)
        py_test = self.visit(copy.deepcopy(node.test))
        test = self.visit(node.test)
        self.loop_kinds.append(True)
        body = _flatten([self.visit(s) for s in node.body])
        self.loop_kinds.pop()
        # python-level while loops over static conditions keep Python semantics
        self.loop_kinds.append(False)
        py_body = _flatten([self.visit(s) for s in orig_body])
        self.loop_kinds.pop()
        tmp = self._tmp()
        assign = ast.Assign(targets=[ast.Name(id=tmp, ctx=ast.Store())], value=test)
        py_loop = ast.While(test=py_test, body=py_body, orelse=[])
        dyn = ast.With(items=[ast.withitem(context_expr=self._call("While", [ast.Name(id=tmp, ctx=ast.Load())]))],
                       body=body or [ast.Pass()])
        outer = ast.If(test=self._call("is_static", [ast.Name(id=tmp, ctx=ast.Load())]),
                       body=[ast.If(test=ast.Name(id=tmp, ctx=ast.Load()), body=[py_loop], orelse=[])],
                       orelse=[dyn])
        return [assign, outer]

    def visit_For(self, node: ast.For):
        is_ir = False
        it = node.iter
        if isinstance(it, ast.Call):
            f = it.func
            name = f.id if isinstance(f, ast.Name) else (f.attr if isinstance(f, ast.Attribute) else None)
            if name in _IR_LOOP_FUNCS:
                is_ir = True
            if isinstance(f, ast.Name) and f.id == "range":
                it = ast.Call(func=ast.Attribute(value=ast.Name(id="__tl__", ctx=ast.Load()), attr="range",
                                                 ctx=ast.Load()), args=it.args, keywords=it.keywords)
        node.iter = self.visit(it)
        self.loop_kinds.append(is_ir)
        node.body = _flatten([self.visit(s) for s in node.body])
        self.loop_kinds.pop()
        node.orelse = _flatten([self.visit(s) for s in node.orelse])
        return node

    def visit_Break(self, node):
        if self.loop_kinds and self.loop_kinds[-1]:
            return ast.Expr(value=self._call("loop_break", []))
        return node

    def visit_Continue(self, node):
        if self.loop_kinds and self.loop_kinds[-1]:
            return ast.Expr(value=self._call("loop_continue", []))
        return node

    def visit_BoolOp(self, node: ast.BoolOp):
        values = [self.visit(v) for v in node.values]
        fn = "land" if isinstance(node.op, ast.And) else "lor"
        acc = values[0]
        for v in values[1:]:
            acc = self._call(fn, [acc, ast.Lambda(args=_no_args(), body=v)])
        return acc

    def visit_IfExp(self, node: ast.IfExp):
        # ``a if c else b``: a select when c is symbolic, Python's own choice when static
        test = self.visit(node.test)
        body = self.visit(node.body)
        orelse = self.visit(node.orelse)
        return self._call("ifexp", [test, ast.Lambda(args=_no_args(), body=body),
                                    ast.Lambda(args=_no_args(), body=orelse)])

    def visit_Compare(self, node: ast.Compare):
        # chained ``a < b < c`` -> ``(a < b) and (b < c)`` (Python would ask bool(a < b))
        node = self.generic_visit(node)
        if len(node.ops) == 1:
            return node
        import copy
        parts = []
        left = node.left
        for op, right in zip(node.ops, node.comparators):
            parts.append(ast.Compare(left=copy.deepcopy(left), ops=[op], comparators=[copy.deepcopy(right)]))
            left = right
        acc = parts[0]
        for p in parts[1:]:
            acc = self._call("land", [acc, ast.Lambda(args=_no_args(), body=p)])
        return acc

    def visit_UnaryOp(self, node: ast.UnaryOp):
        operand = self.visit(node.operand)
        if isinstance(node.op, ast.Not):
            return self._call("lnot", [operand])
        node.operand = operand
        return node

    def visit_Assign(self, node: ast.Assign):
        if len(node.targets) == 1 and isinstance(node.targets[0], ast.Tuple) and isinstance(node.value, ast.Tuple) \
                and len(node.targets[0].elts) == len(node.value.elts):
            # ``a, b = b, a`` / ``A[0], A[1] = A[1], A[0]``: every right-hand value is bound to a
            # temporary first (loads are let-bound there), so no target sees an earlier store
            tmps = [self._tmp() for _ in node.value.elts]
            out = []
            for t, v in zip(tmps, node.value.elts):
                out.append(self.visit_Assign(ast.Assign(targets=[ast.Name(id=t, ctx=ast.Store())], value=v)))
            for tgt, t in zip(node.targets[0].elts, tmps):
                out.append(self.visit_Assign(ast.Assign(targets=[tgt], value=ast.Name(id=t, ctx=ast.Load()))))
            return _flatten(out)
        node.value = self.visit(node.value)
        if len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            node.value = self._call("assign", [
                ast.Constant(value=name), node.value,
                ast.Lambda(args=_no_args(), body=ast.Name(id=name, ctx=ast.Load()))
            ])
        else:
            node.targets = [self.visit(t) for t in node.targets]
        return node

    def visit_AnnAssign(self, node: ast.AnnAssign):
        # ``x: T.int32 = v`` behaves like an assignment
        if node.value is not None and isinstance(node.target, ast.Name):
            return self.visit_Assign(ast.Assign(targets=[node.target], value=node.value))
        return node

    def visit_AugAssign(self, node: ast.AugAssign):
        if isinstance(node.target, ast.Name):
            name = node.target.id
            value = ast.BinOp(left=ast.Name(id=name, ctx=ast.Load()), op=node.op, right=node.value)
            return self.visit_Assign(ast.Assign(targets=[ast.Name(id=name, ctx=ast.Store())], value=value))
        node.value = self.visit(node.value)
        return node


def _no_args():
    return ast.arguments(posonlyargs=[], args=[], vararg=None, kwonlyargs=[], kw_defaults=[], kwarg=None,
                         defaults=[])


def _flatten(stmts):
    out = []
    for s in stmts:
        if isinstance(s, list):
            out.extend(s)
        elif s is not None:
            out.append(s)
    return out


def _copy_stmts(stmts):
    import copy
    return [copy.deepcopy(s) for s in stmts]


# ---------------------------------------------------------------------------


def _closure_namespace(fn) -> Dict[str, Any]:
    ns = dict(fn.__globals__)
    if fn.__closure__:
        for name, cell in zip(fn.__code__.co_freevars, fn.__closure__):
            try:
                ns[name] = cell.cell_contents
            except ValueError:  # empty cell
                pass
    ns["__tl__"] = HELPERS
    return ns


@functools.lru_cache(maxsize=None)
def _parse_source(filename: str, firstlineno: int, src: str):
    tree = ast.parse(src)
    ast.increment_lineno(tree, firstlineno - 1)
    return tree


def rewrite_function(fn):
    """Return a new Python function whose body has been rewritten for IR tracing."""
    try:
        src = textwrap.dedent(inspect.getsource(fn))
    except (OSError, TypeError) as e:  # pragma: no cover - interactive definitions
        raise RuntimeError(f"cannot read the source of {fn.__name__}; define kernels in a file") from e
    filename = inspect.getsourcefile(fn) or "<tilelang>"
    firstlineno = fn.__code__.co_firstlineno
    tree = _parse_source(filename, firstlineno, src)
    import copy
    tree = copy.deepcopy(tree)
    fdef = tree.body[0]
    while not isinstance(fdef, (ast.FunctionDef, ast.AsyncFunctionDef)):
        raise RuntimeError("prim_func must decorate a function definition")
    fdef.decorator_list = []
    fdef.returns = None
    # strip annotations (they were already evaluated by Python)
    for a in fdef.args.args + fdef.args.kwonlyargs + fdef.args.posonlyargs:
        a.annotation = None
    rw = _Rewriter()
    fdef.body = _flatten([rw.visit(s) for s in fdef.body])
    ast.fix_missing_locations(tree)
    ns = _closure_namespace(fn)
    code = compile(tree, filename, "exec")
    exec(code, ns)  # noqa: S102 - executing the user's own (rewritten) kernel source
    new_fn = ns[fdef.name]
    new_fn.__tl_original__ = fn
    return new_fn


# ---------------------------------------------------------------------------
# parameter annotations
# ---------------------------------------------------------------------------


class TensorAnnot:
    """``T.Tensor(shape, dtype)`` / ``T.Tensor[shape, dtype]`` kernel parameter annotation."""

    def __init__(self, shape, dtype="float32", strides=None, scope="global", meta=None):
        if isinstance(shape, (int, PrimExpr)):
            shape = (shape, )
        self.shape = list(shape)
        self.dtype = _dt.as_dtype(dtype)
        self.strides = strides
        self.scope = scope
        self.meta = meta  # MeshTensor metadata

    @staticmethod
    def _construct_strides(shape):
        strides = []
        acc = 1
        for s in reversed(list(shape)):
            strides.append(acc)
            acc = acc * s
        return tuple(reversed(strides))

    def make_buffer(self, name: str) -> Buffer:
        b = Buffer(name, self.shape, self.dtype, self.scope, strides=self.strides)
        if self.meta is not None:
            b.mesh_meta = self.meta
        return b


class ScalarAnnot:

    def __init__(self, dtype):
        self.dtype = _dt.as_dtype(dtype)


def _param_from_annotation(name: str, ann):
    if isinstance(ann, TensorAnnot):
        return ann.make_buffer(name)
    if isinstance(ann, Buffer):
        # an already built buffer (e.g. T.Buffer(...) object); rename it
        b = Buffer(name, ann.shape, ann.dtype, ann.scope, strides=ann.strides)
        return b
    if isinstance(ann, _dt.DType):
        return Var(name, ann, nonneg=ann.is_int)
    if isinstance(ann, ScalarAnnot):
        return Var(name, ann.dtype, nonneg=ann.dtype.is_int)
    if isinstance(ann, str):
        try:
            return Var(name, _dt.as_dtype(ann))
        except ValueError:
            pass
    if ann is int:
        return Var(name, _dt.int32)
    if ann is float:
        return Var(name, _dt.float32)
    if isinstance(ann, type) and issubclass(ann, PrimExpr):
        return Var(name, _dt.int32)
    raise TypeError(f"parameter {name!r}: unsupported annotation {ann!r}")


def _resolve_annotations(fn) -> Dict[str, Any]:
    anns = dict(getattr(fn, "__annotations__", {}))
    ns = None
    for k, v in list(anns.items()):
        if isinstance(v, str):  # from __future__ import annotations
            if ns is None:
                ns = _closure_namespace(fn)
                # names used only in annotations are not captured by the closure: use the
                # locals of the frame that applied the decorator
                for name, val in (getattr(fn, "__tl_def_locals__", None) or {}).items():
                    ns.setdefault(name, val)
            anns[k] = eval(v, ns)  # noqa: S307 - user annotation
    return anns


def prim_func(fn=None, *, private: bool = False, generator: bool = False):
    """Decorator turning a kernel definition into a ``PrimFunc`` (eagerly traced)."""

    def deco(f, depth=1):
        try:
            f.__tl_def_locals__ = dict(sys._getframe(depth).f_locals)
        except (AttributeError, ValueError):
            pass
        if generator:
            return _PrimFuncGenerator(f)
        return trace_prim_func(f)

    if fn is None:
        return deco
    return deco(fn, depth=2)


def trace_prim_func(f, arg_overrides: Optional[Dict[str, Any]] = None) -> S.PrimFunc:
    anns = _resolve_annotations(f)
    sig = inspect.signature(f)
    params = []
    args = []
    for name, p in sig.parameters.items():
        ann = (arg_overrides or {}).get(name, anns.get(name, p.annotation))
        if ann is inspect.Parameter.empty:
            raise TypeError(f"kernel parameter {name!r} needs a T.Tensor / dtype annotation")
        obj = _param_from_annotation(name, ann)
        obj_param = obj
        params.append(obj_param)
        args.append(obj)
    new_fn = rewrite_function(f)
    with building() as b:
        new_fn(*args)
        body = b.pop() if len(b.frames) == 1 else None
        if body is None:
            raise RuntimeError("unbalanced frames while building the kernel")
    for i, p in enumerate(params):
        if isinstance(p, Buffer):
            p.param_index = i
    func = S.PrimFunc(f.__name__, params, body)
    func.attrs.update(b.attrs)
    metas = {p.name: p.mesh_meta for p in params if isinstance(p, Buffer) and getattr(p, "mesh_meta", None)}
    if metas:
        func.attrs["tensor_meta"] = metas
    func.source_fn = f
    return func


class _PrimFuncGenerator:
    """``T.prim_func(generator=True)``: re-traced per call (used by lazy_jit)."""

    def __init__(self, f):
        self.f = f
        functools.update_wrapper(self, f)

    def __call__(self, **overrides):
        return trace_prim_func(self.f, overrides)


def macro(fn=None, *, hygienic: bool = True):
    """``@T.macro``: a helper whose body is inlined (traced) into the calling kernel."""

    def deco(f):
        rewritten = {}

        @functools.wraps(f)
        def wrapper(*args, **kwargs):
            if "fn" not in rewritten:
                rewritten["fn"] = rewrite_function(f)
            return rewritten["fn"](*args, **kwargs)

        wrapper.__tl_macro__ = True
        return wrapper

    if fn is None:
        return deco
    return deco(fn)
