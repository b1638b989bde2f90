"""Kernel cache (reference ``tilelang/cache/kernel_cache.py``): memory + disk.

Two levels:
  * compiled code objects keyed by sha256(kernel source, flags, arch, toolchain) under
    ``$TILELANG_CACHE_DIR/obj/<key>.hsaco`` (or ``.so`` for CPU);
  * whole JIT kernels keyed by the printed IR + target + pass configs + out_idx + compiler
    fingerprint, in-process and on disk (``kernel_cache.py``: a new process skips lowering).
Writes are atomic (temp file + rename), so concurrent compiles (autotuner pools, several ranks)
never observe partial files.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import tempfile
import threading
from pathlib import Path

from ..env import env, INCLUDE_DIR
from ..contrib import hipcc

_mem = {}
_lock = threading.Lock()
_toolchain = None


def _tc():
    global _toolchain
    if _toolchain is None:
        _toolchain = hipcc.toolchain_version()
    return _toolchain


def cache_dir() -> Path:
    p = Path(env.TILELANG_CACHE_DIR)
    p.mkdir(parents=True, exist_ok=True)
    return p


def _atomic_write(path: Path, data: bytes):
    path.parent.mkdir(parents=True, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=str(path.parent), prefix=".tmp_")
    with os.fdopen(fd, "wb") as f:
        f.write(data)
    os.replace(tmp, path)


def _key(source: str, flags, kind: str) -> str:
    from .. import env as _e
    inc = ""
    for h in sorted((INCLUDE_DIR / "tl").glob("*.h")):
        inc += h.read_text()
    return hashlib.sha256("\0".join([kind, source, " ".join(flags or []), _tc(), inc]).encode()).hexdigest()


def compile_hip_cached(source: str, flags=None, verbose=False) -> bytes:
    from ..engine.callback import hip_compile_override
    data = hip_compile_override(source, "hip")  # register_hip_compile hook: never cached
    if data is not None:
        return data
    key = _key(source, flags, "hip-gfx950")
    with _lock:
        if key in _mem:
            return _mem[key]
    path = cache_dir() / "obj" / f"{key}.hsaco"
    if env.is_cache_enabled() and path.exists():
        data = path.read_bytes()
    else:
        if env.is_print_on_compilation_enabled():
            print(f"[tilelang] compiling gfx950 kernel {key[:12]}")
        data = hipcc.compile_hip(source, options=flags, verbose=verbose)
        if env.is_cache_enabled():
            _atomic_write(path, data)
    with _lock:
        _mem[key] = data
    return data


def compile_cpu_cached(source: str, flags=None, verbose=False) -> str:
    key = _key(source, flags, "cpu")
    path = cache_dir() / "obj" / f"{key}.so"
    if env.is_cache_enabled() and path.exists():
        return str(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=str(path.parent), prefix=".tmp_", suffix=".so")
    os.close(fd)
    hipcc.compile_cpu(source, tmp, options=flags, verbose=verbose)
    if env.is_cache_enabled():
        os.replace(tmp, path)
        return str(path)
    return tmp


def clear_cache():
    with _lock:
        _mem.clear()
    from ..jit import _GLOBAL_JIT_CACHE
    _GLOBAL_JIT_CACHE.clear()
    p = Path(env.TILELANG_CACHE_DIR)
    if p.exists():
        shutil.rmtree(p, ignore_errors=True)


def disable_cache():
    env.disable_cache()


def enable_cache():
    env.enable_cache()
