"""Whole-kernel disk cache (reference ``tilelang/cache/kernel_cache.py:250-452``).

A second process compiling the same program skips lowering AND code generation: the entry holds
everything ``JITKernel`` needs to launch — the device sources, code objects (``.hsaco`` bytes for
gfx950, a shared object for the CPU target), the launcher's parameter specs and grid programs, block
size and LDS bytes.  Key = sha256 of

  * the printed program (``PrimFunc.script()``: every tile-op attribute is printed, so two programs
    that lower differently never share a key — ``ir/printer.py``),
  * target, pass configs, ``out_idx``, compile flags,
  * a fingerprint of the compiler itself (every ``tilelang/**/*.py`` that lowers/generates code, the
    ``tl/*.h`` device headers, the built native core/runtime extensions and the hipcc version), so
    editing or rebuilding the compiler invalidates entries,
  * the registered compile hooks, closures and referenced globals included (``hook_fingerprint``).

Layout: ``$TILELANG_CACHE_DIR/kernels/<key>/{meta.json, kernel_<i>.hip, code_<i>.{hsaco,so}}``,
written into a temp directory and renamed into place (concurrent writers — autotuner threads,
several ranks — never expose a partial entry).  Programs that use the Mesh (``T.comm``) are not
disk-cached: their launch arguments depend on the live mesh.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import tempfile
import threading
from pathlib import Path

from ..env import env, INCLUDE_DIR

_FP = None
_FP_LOCK = threading.Lock()
_COMPILER_DIRS = ("analysis", "codegen", "engine", "ir", "jit", "language", "layout", "transform", "utils",
                  "contrib", "cache")


def compiler_fingerprint() -> str:
    """Hash of the compiler's own sources + device headers + toolchain (memoised per process)."""
    global _FP
    if _FP is None:
        with _FP_LOCK:
            if _FP is None:
                from . import _tc
                h = hashlib.sha256(_tc().encode())
                root = Path(__file__).resolve().parent.parent
                files = []
                for d in _COMPILER_DIRS:
                    files += sorted((root / d).rglob("*.py"))
                files += sorted((INCLUDE_DIR / "tl").rglob("*.h"))
                files += [root / "_native.py", root / "__init__.py"]
                # the native compiler core (reduce_owners, plan_arena, fragment inverses) and the
                # runtime: a rebuilt extension must not be served entries lowered by the old one
                files += sorted(root.glob("_tl_*.so"))
                for f in files:
                    if not f.exists():
                        continue
                    h.update(str(f.relative_to(root.parent) if root.parent in f.parents else f.name).encode())
                    h.update(f.read_bytes())
                _FP = h.hexdigest()
    return _FP


def _freeze(x):
    if isinstance(x, dict):
        return {str(k): _freeze(v) for k, v in sorted(x.items(), key=lambda kv: str(kv[0]))}
    if isinstance(x, (list, tuple)):
        return [_freeze(v) for v in x]
    return x if isinstance(x, (int, float, str, bool, type(None))) else repr(x)


def kernel_key(func, target, out_idx, pass_configs, compile_flags) -> str:
    from ..engine.callback import hook_fingerprint
    import os
    blob = json.dumps({"hooks": hook_fingerprint(), "ir": func.script(), "target": str(target),
                       "env": {"TL_GEMM_QUAD": os.environ.get("TL_GEMM_QUAD", "1"),
                               "TL_PIPELINE_UNROLL": os.environ.get("TL_PIPELINE_UNROLL", "0"),
                               "TL_ATOMIC_STAGE": os.environ.get("TL_ATOMIC_STAGE", "1"),
                               "TL_GEMM_RS_PIPE": os.environ.get("TL_GEMM_RS_PIPE", "")},  # lower.py A/B switches
                       "out_idx": _freeze(out_idx),
                       "pass_configs": _freeze(pass_configs or {}), "flags": _freeze(compile_flags or []),
                       "compiler": compiler_fingerprint()}, sort_keys=True)
    return hashlib.sha256(blob.encode()).hexdigest()


def _root() -> Path:
    p = Path(env.TILELANG_CACHE_DIR) / "kernels"
    p.mkdir(parents=True, exist_ok=True)
    return p


def _json_specs(specs):
    out = []
    for d in specs:
        d = dict(d)
        d["shape"] = [list(s) for s in d["shape"]]
        d["strides"] = [list(s) for s in d["strides"]]
        out.append(d)
    return out


def _tuple_specs(specs):
    out = []
    for d in specs:
        d = dict(d)
        d["shape"] = [tuple(s) for s in d["shape"]]
        d["strides"] = [tuple(s) for s in d["strides"]]
        out.append(d)
    return out


def save(key: str, kernel) -> bool:
    """Store a compiled ``JITKernel``; returns False when the program is not cacheable."""
    a = kernel.artifact
    if not env.is_cache_enabled() or any(dk.mesh is not None for dk in a.kernels):
        return False
    dest = _root() / key
    if dest.exists():
        return True
    tmp = Path(tempfile.mkdtemp(dir=str(_root()), prefix=".tmp_"))
    try:
        meta = {"version": 1, "is_cpu": a.is_cpu, "kernels": []}
        for i, (dk, code) in enumerate(zip(a.kernels, kernel.code)):
            specs, nsyms, grid = kernel._param_specs(dk, with_outputs=(i == 0))
            (tmp / f"kernel_{i}.hip").write_text(dk.source)
            ext = "so" if a.is_cpu else "hsaco"
            if a.is_cpu:
                shutil.copy(code, tmp / f"code_{i}.{ext}")
            else:
                (tmp / f"code_{i}.{ext}").write_bytes(code)
            meta["kernels"].append({
                "name": dk.name, "block": [int(b) for b in dk.block], "lds_bytes": int(dk.lds_bytes),
                "grid_exprs": [str(g) for g in dk.grid], "cooperative": bool(getattr(dk, "cooperative", False)),
                "params": [{"kind": p["kind"], "name": p["name"], "dtype": str(p.get("dtype", ""))}
                           for p in dk.params],
                "specs": _json_specs(specs), "nsyms": nsyms, "grid": grid,
                "narrow_index": sorted(getattr(dk, "narrow_index", ()) or ()),
                "layout_info": dict(getattr(dk, "layout_info", {}) or {})})
        (tmp / "meta.json").write_text(json.dumps(meta))
        try:
            os.replace(tmp, dest)
        except OSError:  # another writer won the race
            shutil.rmtree(tmp, ignore_errors=True)
        return True
    except Exception:
        shutil.rmtree(tmp, ignore_errors=True)
        raise


def load(key: str):
    """(artifact, code, launch specs) for a cached entry, or None."""
    if not env.is_cache_enabled():
        return None
    d = _root() / key
    mf = d / "meta.json"
    if not mf.exists():
        return None
    try:
        meta = json.loads(mf.read_text())
    except (OSError, ValueError):
        return None
    from ..engine.lower import DeviceKernel
    kernels, code, launch = [], [], []
    for i, k in enumerate(meta["kernels"]):
        src = (d / f"kernel_{i}.hip").read_text()
        dk = DeviceKernel(src, k["name"], k["grid_exprs"], k["block"], k["lds_bytes"], k["params"])
        dk.cooperative = k["cooperative"]
        dk.narrow_index = set(k.get("narrow_index", ()))  # int32-addressed params (launcher overflow check)
        dk.layout_info = dict(k.get("layout_info", {}))
        kernels.append(dk)
        path = d / f"code_{i}.{'so' if meta['is_cpu'] else 'hsaco'}"
        code.append(str(path) if meta["is_cpu"] else path.read_bytes())
        launch.append((_tuple_specs(k["specs"]), k["nsyms"], k["grid"]))
    return meta["is_cpu"], kernels, code, launch


def clear():
    p = Path(env.TILELANG_CACHE_DIR) / "kernels"
    if p.exists():
        shutil.rmtree(p, ignore_errors=True)


def entries() -> int:
    p = Path(env.TILELANG_CACHE_DIR) / "kernels"
    return sum(1 for x in p.iterdir() if not x.name.startswith(".")) if p.exists() else 0
