"""``@tilelang.lazy_jit``: kernels specialised from their call-site arguments.

Reference: ``tilelang/jit/__init__.py`` (``lazy_jit``) + ``tilelang/language/v2/annot.py``; tests
``testing/python/language/test_tilelang_language_lazy_jit.py``.  The decorated function is the
kernel body itself; calling it with torch tensors (or ``par_compile`` with ``T.Tensor(shape,
dtype)`` / ``T.ptr()`` specs) binds every parameter by its annotation:

=====================================  ===============================================  ===========
annotation                             parameter of the compiled kernel                 cache key
=====================================  ===============================================  ===========
``T.Tensor[[int, T.dyn, 64], Any]``    global buffer; ``int`` dims static, ``T.dyn``    dtype, static
                                       dims runtime symbols, literal dims checked       dims/strides
``T.StridedTensor[[..], [..], dt]``    same, with explicit strides (views)
``T.Tensor((M, N), dt)``               fixed-shape buffer (promoted as is)
``T.ptr``                              raw pointer bound by ``T.make_tensor(p, shape)``  —
``T.dyn`` / ``T.dyn[int, 'X']``        runtime int32 scalar                             —
``T.dtype``, ``int``, anything else    compile-time constant                            the value
=====================================  ===============================================  ===========

Tensors created with ``T.empty(...)`` in the body become outputs the launcher allocates; the call
returns whatever the body returns (one of them, a tuple, or None for in-place kernels).  Every
specialisation is compiled once (memory, then the whole-kernel disk cache) and reused.
"""
from __future__ import annotations

import functools
import inspect
from typing import Any, Dict, List, Tuple

from ..ir import dtypes as _dt
from ..ir import stmt as S
from ..ir.buffer import Buffer
from ..ir.expr import Var
from ..language import annot as A
from ..language.parser import TensorAnnot, ScalarAnnot, _resolve_annotations, rewrite_function
from ..language.builder import building


def _is_tensor(x):
    return hasattr(x, "shape") and hasattr(x, "dtype") and hasattr(x, "data_ptr")


class _Spec:
    """How one parameter is bound for one call."""

    def __init__(self, kind, key, build):
        self.kind = kind      # "tensor" | "ptr" | "dyn" | "const"
        self.key = key
        self.build = build    # () -> traced object (Buffer / PtrParam / Var / python value)


def _tensor_spec(name, ann, arg, symbols):
    """Bind a tensor parameter: static dims/dtype go into the key, dyn dims become symbols."""
    if isinstance(arg, TensorAnnot):   # par_compile spec: T.Tensor((M, N), dtype)
        shape = [int(s) for s in arg.shape]
        strides = list(arg.strides) if arg.strides else None
        dtype = arg.dtype
    elif _is_tensor(arg):
        shape = list(arg.shape)
        strides = list(arg.stride())
        dtype = _dt.from_torch(arg.dtype)
    else:
        raise TypeError(f"parameter {name!r} expects a tensor, got {type(arg).__name__}")
    if isinstance(ann, TensorAnnot):   # fully static annotation: must match
        want = [int(s) for s in ann.shape]
        if want != shape or ann.dtype != dtype:
            raise TypeError(f"parameter {name!r}: expected {tuple(want)} {ann.dtype}, got {tuple(shape)} {dtype}")
        return _Spec("tensor", ("T", tuple(shape), dtype.name), lambda: ann.make_buffer(name))
    if ann is None:
        ann = A.TensorTemplate([int] * len(shape), Any)
    if len(ann.shape) != len(shape):
        raise TypeError(f"parameter {name!r}: rank {len(shape)} does not match annotation {ann.shape}")
    if ann.dtype is not None and ann.dtype != dtype:
        raise TypeError(f"parameter {name!r}: dtype {dtype} does not match annotation {ann.dtype}")
    key_dims, dims = [], []
    for i, (d, v) in enumerate(zip(ann.shape, shape)):
        if d is int:
            key_dims.append(v)
            dims.append(("static", v))
        elif d is A.dyn or isinstance(d, A.DynAnnot):
            sym = d.name if isinstance(d, A.DynAnnot) and d.name else f"{name}_dim{i}"
            key_dims.append("?")
            dims.append(("dyn", sym))
        elif isinstance(d, int):
            if d != v:
                raise TypeError(f"parameter {name!r}: dim {i} is {v}, annotation requires {d}")
            key_dims.append(v)
            dims.append(("static", v))
        else:
            raise TypeError(f"parameter {name!r}: unsupported dim annotation {d!r}")
    sdims = None
    if ann.strides is not None:
        if strides is None:
            strides = _row_major(shape)
        if len(ann.strides) != len(strides):
            raise TypeError(f"parameter {name!r}: strides rank mismatch")
        sdims = []
        for i, (d, v) in enumerate(zip(ann.strides, strides)):
            if d is int or (isinstance(d, int) and d == v):
                sdims.append(("static", v))
                key_dims.append(("s", v))
            elif d is A.dyn or isinstance(d, A.DynAnnot):
                sym = d.name if isinstance(d, A.DynAnnot) and d.name else f"{name}_stride{i}"
                sdims.append(("dyn", sym))
                key_dims.append(("s", "?"))
            else:
                raise TypeError(f"parameter {name!r}: stride {i} is {v}, annotation requires {d}")
    elif strides is not None and list(strides) != _row_major(shape) and _is_tensor(arg):
        raise TypeError(f"parameter {name!r} is not contiguous: annotate it with T.StridedTensor")

    def build():
        sh = [v if k == "static" else symbols.setdefault(v, Var(v, _dt.int32, nonneg=True)) for k, v in dims]
        st = None
        if sdims is not None:
            st = [v if k == "static" else symbols.setdefault(v, Var(v, _dt.int32, nonneg=True)) for k, v in sdims]
        return Buffer(name, sh, dtype, "global", strides=st)

    return _Spec("tensor", ("T", tuple(key_dims), dtype.name), build)


def _row_major(shape):
    out, acc = [], 1
    for s in reversed(list(shape)):
        out.append(acc)
        acc *= int(s)
    return list(reversed(out))


class LazyJITImpl:
    """Kernel body with parameter annotations; specialised, compiled and run per call."""

    def __init__(self, fn, out_idx=None, target="auto", pass_configs=None, compile_flags=None, verbose=False):
        self.fn = fn
        self.out_idx = out_idx
        self.target = target
        self.pass_configs = pass_configs
        self.compile_flags = compile_flags
        self.verbose = verbose
        self.signature = inspect.signature(fn)
        self._cache: Dict[Any, Tuple] = {}
        self._anns = None
        functools.update_wrapper(self, fn)

    # -- binding ---------------------------------------------------------------------------
    def _annotations(self):
        if self._anns is None:
            self._anns = _resolve_annotations(self.fn)
        return self._anns

    def _bind(self, args, kwargs):
        bound = self.signature.bind(*args, **kwargs)
        bound.apply_defaults()
        anns = self._annotations()
        symbols: Dict[str, Var] = {}
        specs = []
        for name, value in bound.arguments.items():
            ann = anns.get(name, inspect.Parameter.empty)
            if isinstance(ann, (A.TensorTemplate, TensorAnnot)) or \
                    (ann is inspect.Parameter.empty and (_is_tensor(value) or isinstance(value, TensorAnnot))):
                specs.append((name, _tensor_spec(name, None if ann is inspect.Parameter.empty else ann, value,
                                                 symbols)))
            elif ann is A.ptr:
                if not (_is_tensor(value) or isinstance(value, A.PtrSpec)):
                    raise TypeError(f"parameter {name!r} (T.ptr) expects a tensor")
                specs.append((name, _Spec("ptr", ("P", ), (lambda n=name: A.PtrParam(n)))))
            elif ann is A.dyn or isinstance(ann, (A.DynAnnot, ScalarAnnot)):
                dt = _dt.int32 if ann is A.dyn else ann.dtype
                specs.append((name, _Spec("dyn", ("D", dt.name),
                                          (lambda n=name, d=dt: symbols.setdefault(n, Var(n, d, nonneg=d.is_int))))))
            else:
                v = value
                if ann is A.dtype or isinstance(v, _dt.DType):
                    v = _dt.as_dtype(v)
                key = ("C", v.name if isinstance(v, _dt.DType) else _freeze(v))
                specs.append((name, _Spec("const", key, (lambda x=v: x))))
        return bound, specs

    # -- tracing ---------------------------------------------------------------------------
    def _trace(self, specs):
        objs = [(name, sp.kind, sp.build()) for name, sp in specs]
        new_fn = rewrite_function(self.fn)
        ctx = A.LazyTrace()
        A.LAZY_STACK.append(ctx)
        try:
            with building() as b:
                ret = new_fn(*[o for _, _, o in objs])
                body = b.pop() if len(b.frames) == 1 else None
                if body is None:
                    raise RuntimeError("unbalanced frames while tracing the lazy_jit kernel")
        finally:
            A.LAZY_STACK.pop()
        params, call_plan = [], []
        for name, kind, o in objs:
            if kind == "tensor":
                params.append(o)
                call_plan.append(("arg", name, None))
            elif kind == "ptr":
                buf = ctx.ptr_buffers.get(o)
                if buf is None:
                    raise ValueError(f"T.ptr parameter {name!r} is never bound with T.make_tensor")
                params.append(buf)
                call_plan.append(("ptr", name, [int(s) if not isinstance(s, Var) else None for s in buf.shape]))
            elif kind == "dyn":
                params.append(o)
                call_plan.append(("arg", name, None))
        outs = list(ctx.outputs)
        out_idx = list(range(len(params), len(params) + len(outs))) or None
        params += outs
        for i, p in enumerate(params):
            if isinstance(p, Buffer):
                p.param_index = i
        func = S.PrimFunc(self.fn.__name__, params, body)
        func.attrs.update(b.attrs)
        func.source_fn = self.fn
        rets = ret if isinstance(ret, (tuple, list)) else ([] if ret is None else [ret])
        ret_plan = []
        for r in rets:
            if not isinstance(r, Buffer) or r not in outs:
                raise TypeError("a lazy_jit kernel may only return tensors created with T.empty")
            ret_plan.append(outs.index(r))
        ret_kind = "tuple" if isinstance(ret, (tuple, list)) else ("one" if ret is not None else "none")
        if self.out_idx is not None:
            out_idx = self.out_idx
        return func, out_idx, call_plan, ret_plan, ret_kind

    def _get(self, args, kwargs):
        bound, specs = self._bind(args, kwargs)
        key = tuple(sp.key for _, sp in specs)
        hit = self._cache.get(key)
        if hit is None:
            func, out_idx, call_plan, ret_plan, ret_kind = self._trace(specs)
            from . import compile as _compile
            k = _compile(func, out_idx, "auto", self.target, None, self.verbose, self.pass_configs,
                         self.compile_flags)
            hit = (k, call_plan, ret_plan, ret_kind)
            self._cache[key] = hit
        return bound, hit

    # -- public API --------------------------------------------------------------------------
    def get_tir(self, *args, **kwargs) -> S.PrimFunc:
        _, specs = self._bind(args, kwargs)
        return self._trace(specs)[0]

    def compile(self, *args, **kwargs):
        return self._get(args, kwargs)[1][0]

    get_kernel = compile

    def par_compile(self, configs: List[Dict[str, Any]], num_workers=None, ignore_error=False):
        from concurrent.futures import ThreadPoolExecutor
        import os

        def one(c):
            try:
                return self.compile(**c)
            except Exception:
                if ignore_error:
                    return None
                raise

        with ThreadPoolExecutor(num_workers or min(16, os.cpu_count() or 4)) as ex:
            return list(ex.map(one, configs))

    def __call__(self, *args, **kwargs):
        bound, (k, call_plan, ret_plan, ret_kind) = self._get(args, kwargs)
        inputs = []
        for kind, name, shape in call_plan:
            v = bound.arguments[name]
            if kind == "ptr" and _is_tensor(v) and None not in shape and list(v.shape) != shape:
                v = v.view(shape)
            inputs.append(v)
        out = k(*inputs)
        if ret_kind == "none":
            return None
        outs = list(out) if isinstance(out, tuple) else [out]
        picked = [outs[i] for i in ret_plan]
        return picked[0] if ret_kind == "one" else tuple(picked)


def _freeze(x):
    if isinstance(x, (list, tuple)):
        return tuple(_freeze(i) for i in x)
    if isinstance(x, dict):
        return tuple(sorted((k, _freeze(v)) for k, v in x.items()))
    try:
        hash(x)
        return x
    except TypeError:
        return repr(x)


def lazy_jit(func=None, *, out_idx=None, target="auto", pass_configs=None, compile_flags=None, verbose=False):

    def deco(fn):
        return LazyJITImpl(fn, out_idx, target, pass_configs, compile_flags, verbose)

    if func is not None and callable(func):
        return deco(func)
    return deco
