"""Source post-processing and compiler hooks (reference ``tilelang/engine/callback.py:7-92`` and the
``tilelang_callback_hip_postproc`` / ``tilelang_callback_hip_compile`` globals consulted by
``src/target/rt_mod_hip.cc:56-90``).

* ``register_hip_postproc(func)``: ``func(code: str, target) -> str`` rewrites every generated
  gfx950 kernel source before it is compiled (inject pragmas, ``__builtin_amdgcn_*`` tweaks,
  instrumentation).  The rewritten source is what ``JITKernel.get_kernel_source()`` shows.
* ``register_hip_compile(func)``: ``func(code: str, target) -> bytes`` replaces the built-in
  clang++ ``--offload-device-only`` step; it must return a gfx950 code object (ELF) that
  ``hipModuleLoadData`` accepts.
* decorator forms ``@register_hip_postproc_callback`` / ``@register_hip_compile_callback`` (with
  or without parentheses, ``override=`` as in the reference).

The hooks' bytecode is part of the whole-kernel cache key (``hook_fingerprint``), so a changed or
removed hook never serves a kernel compiled under another.  This framework has no CUDA target:
``register_cuda_postproc`` raises instead of silently registering a hook nothing would call.
"""
from __future__ import annotations

import hashlib
from typing import Callable, Optional

_HOOKS = {}


def _register(name: str, func: Callable, override: bool):
    if not callable(func):
        raise TypeError(f"{name}: expected a callable, got {type(func).__name__}")
    if name in _HOOKS and not override:
        raise ValueError(f"{name} is already registered (pass override=True to replace it)")
    _HOOKS[name] = func


def register_hip_postproc(func: Callable[[str, object], str], override: bool = True):
    _register("tilelang_callback_hip_postproc", func, override)


def register_hip_compile(func: Callable[[str, object], bytes], override: bool = True):
    _register("tilelang_callback_hip_compile", func, override)


def _decorator(register):

    def deco(func=None, override: bool = True):
        if callable(func):
            register(func, override)
            return func
        if func is None or isinstance(func, bool):
            ov = func if isinstance(func, bool) else override

            def _reg(fn):
                register(fn, ov)
                return fn

            return _reg
        raise TypeError("Invalid decorator usage")

    return deco


register_hip_postproc_callback = _decorator(register_hip_postproc)
register_hip_compile_callback = _decorator(register_hip_compile)


def unregister(name: Optional[str] = None):
    """Remove one hook (by its global name) or all of them."""
    if name is None:
        _HOOKS.clear()
    else:
        _HOOKS.pop(name, None)


def get(name: str) -> Optional[Callable]:
    return _HOOKS.get(name)


def hook_fingerprint() -> str:
    """Identity of the registered hooks for cache keys ('' when none is registered)."""
    if not _HOOKS:
        return ""
    h = hashlib.sha256()
    for name in sorted(_HOOKS):
        h.update(name.encode())
        _hash_callable(h, _HOOKS[name], depth=0)
    return h.hexdigest()


def _hash_value(h, v, depth):
    """Hash what a hook can read besides its bytecode: closure cells, defaults and the module
    globals it names.  Two hooks with one body but different captured values (a lambda built in
    a loop over variants) must not share a cache key."""
    if isinstance(v, (str, bytes, int, float, bool, type(None))):
        h.update(repr(v).encode())
    elif isinstance(v, (list, tuple, set, frozenset)):
        h.update(type(v).__name__.encode())
        for x in (sorted(v, key=repr) if isinstance(v, (set, frozenset)) else v):
            _hash_value(h, x, depth)
    elif isinstance(v, dict):
        for k in sorted(v, key=repr):
            _hash_value(h, k, depth)
            _hash_value(h, v[k], depth)
    elif callable(v) and hasattr(v, "__code__") and depth < 3:
        _hash_callable(h, v, depth + 1)
    else:
        # objects without a stable value: their type only (a mutable object is the user's business)
        h.update(type(v).__qualname__.encode())


def _hash_callable(h, f, depth):
    code = getattr(f, "__code__", None)
    h.update(getattr(f, "__qualname__", repr(f)).encode())
    if code is None:
        h.update(repr(f).encode())
        return
    h.update(code.co_code)
    h.update(repr(code.co_consts).encode())
    for cell in (getattr(f, "__closure__", None) or ()):
        try:
            _hash_value(h, cell.cell_contents, depth)
        except ValueError:  # empty cell
            h.update(b"<empty>")
    _hash_value(h, getattr(f, "__defaults__", None), depth)
    _hash_value(h, getattr(f, "__kwdefaults__", None), depth)
    g = getattr(f, "__globals__", {})
    for n in code.co_names:
        if n in g and not isinstance(g[n], type(hashlib)):
            h.update(n.encode())
            _hash_value(h, g[n], depth)


def apply_hip_postproc(code: str, target) -> str:
    f = _HOOKS.get("tilelang_callback_hip_postproc")
    if f is None:
        return code
    out = f(code, target)
    if not isinstance(out, str):
        raise TypeError(f"HIP postproc callback returned {type(out).__name__}, expected str")
    return out


def hip_compile_override(code: str, target) -> Optional[bytes]:
    f = _HOOKS.get("tilelang_callback_hip_compile")
    if f is None:
        return None
    out = f(code, target)
    if not isinstance(out, (bytes, bytearray)) or not bytes(out[:4]) == b"\x7fELF":
        raise TypeError("HIP compile callback must return a gfx950 code object (ELF bytes)")
    return bytes(out)


def _no_cuda(*_a, **_k):
    raise NotImplementedError("this framework targets gfx950 only: there is no CUDA code generation to post-process "
                              "(use register_hip_postproc)")


register_cuda_postproc = _no_cuda
register_cuda_postproc_callback = _no_cuda
