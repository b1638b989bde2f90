"""Device/host compilers (reference ``tilelang/contrib/hipcc.py:19-100``, ``jit/adapter/libgen.py``).

gfx950 kernels are compiled straight to a raw code object (no host stub, no fat binary):
``clang++ -x hip --offload-arch=gfx950 --offload-device-only --no-gpu-bundle-output -O3``.
CPU kernels are compiled by host clang++ into a shared object.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import tempfile
from pathlib import Path
from typing import List, Optional

from ..env import INCLUDE_DIR, env

ARCH = "gfx950"


class CompileError(RuntimeError):
    pass


def rocm_path() -> str:
    return env.ROCM_PATH


def clang_path() -> str:
    for p in (os.path.join(rocm_path(), "lib", "llvm", "bin", "clang++"), os.path.join(rocm_path(), "llvm", "bin",
                                                                                       "clang++")):
        if os.path.exists(p):
            return p
    return "clang++"


def get_rocm_arch() -> str:
    return ARCH


def toolchain_version() -> str:
    try:
        out = subprocess.run([clang_path(), "--version"], capture_output=True, text=True, timeout=60).stdout
        return out.splitlines()[0] if out else "unknown"
    except Exception:  # noqa: BLE001
        return "unknown"


DEFAULT_HIP_FLAGS = ["-O3", "-std=c++17", "-ffp-contract=fast-honor-pragmas", "-Wno-unused-variable",
                     "-Wno-unused-value",
                     "-Wno-unused-but-set-variable", "-Wno-pass-failed"]


def compile_hip(source: str, arch: str = ARCH, options: Optional[List[str]] = None, verbose: bool = False,
                keep_dir: Optional[str] = None, asm: bool = False) -> bytes:
    """Compile HIP source to a gfx950 code object (bytes)."""
    if arch != ARCH:
        raise CompileError(f"only gfx950 is supported, got {arch}")
    with tempfile.TemporaryDirectory(prefix="tl_hip_") as d:
        src = Path(d) / "kernel.hip"
        out = Path(d) / ("kernel.s" if asm else "kernel.hsaco")
        src.write_text(source)
        cmd = [clang_path(), "-x", "hip", f"--offload-arch={arch}", "--offload-device-only", "--no-gpu-bundle-output",
               "-I", str(INCLUDE_DIR)] + DEFAULT_HIP_FLAGS + list(options or [])
        if asm:
            cmd += ["-S"]
        cmd += ["-o", str(out), str(src)]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            numbered = "\n".join(f"{i + 1:4d}  {ln}" for i, ln in enumerate(source.splitlines()))
            raise CompileError(f"hipcc failed ({' '.join(cmd)}):\n{r.stderr}\n--- source ---\n{numbered}")
        if keep_dir:
            Path(keep_dir).mkdir(parents=True, exist_ok=True)
            (Path(keep_dir) / src.name).write_text(source)
        return out.read_bytes()


def compile_cpu(source: str, out_path: str, options: Optional[List[str]] = None, verbose: bool = False) -> str:
    with tempfile.TemporaryDirectory(prefix="tl_cpu_") as d:
        src = Path(d) / "kernel.cpp"
        src.write_text(source)
        cmd = [clang_path(), "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-I", str(INCLUDE_DIR), "-w"] + \
            list(options or []) + ["-o", out_path, str(src)]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            numbered = "\n".join(f"{i + 1:4d}  {ln}" for i, ln in enumerate(source.splitlines()))
            raise CompileError(f"host compile failed:\n{r.stderr}\n--- source ---\n{numbered}")
    return out_path


def source_hash(source: str, extra: str = "") -> str:
    h = hashlib.sha256()
    h.update(source.encode())
    h.update(extra.encode())
    return h.hexdigest()
