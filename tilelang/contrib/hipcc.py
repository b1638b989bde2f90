"""Device/host compilers (reference ``tilelang/contrib/hipcc.py:19-100``, ``jit/adapter/libgen.py``).

gfx950 kernels are compiled straight to a raw code object (no host stub, no fat binary):
``clang++ -x hip --offload-arch=gfx950 --offload-device-only --no-gpu-bundle-output -O3``.
CPU kernels are compiled by host clang++ into a shared object.
"""
from __future__ import annotations

import hashlib
import os
import shlex
import subprocess
import tempfile
import threading
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


# ---------------------------------------------------------------------------------------------
# Precompiled tl/tl.h.  Parsing the HIP runtime wrapper + the tile templates is ~1.1 s of the
# ~1.6 s device compile of a typical kernel; every generated kernel starts with the same
# ``#include "tl/tl.h"``, so that prefix is parsed once per (toolchain, headers, flags) into a
# clang PCH under $TILELANG_CACHE_DIR/pch and the kernel compile loads it (GEMM 256x256 kernel:
# 1.61 -> 0.65 s, identical ISA).  The key covers the header text, so the PCH is used with
# -fno-validate-pch (a checkout that only touches mtimes does not invalidate it).  Any failure
# falls back to the plain compile; TL_HIP_PCH=0 disables.
# ---------------------------------------------------------------------------------------------
_TL_INCLUDE_LINE = '#include "tl/tl.h"'
_pch_lock = threading.Lock()
_pch_paths = {}
_hdr_digest = None


def _headers_digest() -> str:
    global _hdr_digest
    if _hdr_digest is None:
        h = hashlib.sha256(toolchain_version().encode())
        for f in sorted(Path(INCLUDE_DIR).rglob("*.h")):
            h.update(str(f.relative_to(INCLUDE_DIR)).encode())
            h.update(f.read_bytes())
        # the ROCm HIP headers and clang's HIP wrappers that tl.h pulls in: a ROCm update that
        # keeps the clang version line must not reuse a stale PCH (-fno-validate-pch below)
        for d in _system_header_dirs():
            for f in sorted(Path(d).rglob("*.h")):
                st = f.stat()
                h.update(f"{f}\0{st.st_size}\0{st.st_mtime_ns}".encode())
        _hdr_digest = h.hexdigest()
    return _hdr_digest


def _system_header_dirs() -> List[str]:
    """The HIP include dir and clang's resource include dir (HIP wrapper headers)."""
    dirs = []
    try:
        rd = subprocess.run([clang_path(), "-print-resource-dir"], capture_output=True, text=True,
                            timeout=60).stdout.strip()
        if rd and os.path.isdir(os.path.join(rd, "include")):
            dirs.append(os.path.join(rd, "include"))
    except Exception:  # noqa: BLE001
        pass
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    if os.path.isdir(os.path.join(rocm, "include", "hip")):
        dirs.append(os.path.join(rocm, "include", "hip"))
    return dirs


def _base_cmd(arch: str) -> List[str]:
    return [clang_path(), "-x", "hip", f"--offload-arch={arch}", "--offload-device-only", "--no-gpu-bundle-output",
            "-I", str(INCLUDE_DIR)]


def precompiled_header(flags: List[str], arch: str = ARCH, verbose: bool = False) -> Optional[str]:
    """Path of the tl/tl.h PCH for these compile flags (built on first use), or None."""
    if os.environ.get("TL_HIP_PCH", "1") == "0":
        return None
    key = hashlib.sha256((_headers_digest() + "\0" + arch + "\0" + "\0".join(flags)).encode()).hexdigest()[:24]
    with _pch_lock:
        if key in _pch_paths:
            return _pch_paths[key]
    d = Path(env.TILELANG_CACHE_DIR) / "pch"
    path = d / f"tl_{key}.pch"
    if not path.exists():
        try:
            d.mkdir(parents=True, exist_ok=True)
            hdr = d / "tl_pch.h"
            if not hdr.exists():
                tmp_h = d / f"tl_pch.h.{os.getpid()}"
                tmp_h.write_text(_TL_INCLUDE_LINE + "\n")
                os.replace(tmp_h, hdr)
            # the driver links device code objects even with -c: take its cc1 job and make it
            # emit the PCH instead of an object
            probe = subprocess.run(_base_cmd(arch) + list(flags) + ["-c", str(hdr), "-o", str(d / "probe.o"), "-###"],
                                   capture_output=True, text=True)
            cc1 = [ln for ln in probe.stderr.splitlines() if '"-cc1"' in ln]
            if probe.returncode != 0 or len(cc1) != 1:
                raise CompileError(probe.stderr[-500:])
            args = shlex.split(cc1[0])
            args[args.index("-emit-obj")] = "-emit-pch"
            tmp = d / f"tl_{key}.pch.{os.getpid()}.{threading.get_ident()}"
            args[args.index("-o") + 1] = str(tmp)
            if verbose:
                print(" ".join(args))
            r = subprocess.run(args, capture_output=True, text=True)
            if r.returncode != 0:
                raise CompileError(r.stderr[-500:])
            os.replace(tmp, path)
        except Exception as e:  # noqa: BLE001 -- the plain compile still works
            if verbose:
                print(f"tl/tl.h PCH unavailable ({e}); compiling without it")
            path = None
    with _pch_lock:
        _pch_paths[key] = str(path) if path else None
    return _pch_paths[key]


def compile_hip(source: str, arch: str = ARCH, options: Optional[List[str]] = None, verbose: bool = False,
                keep_dir: Optional[str] = None, asm: bool = False) -> bytes:
    """Compile HIP source to a gfx950 code object (bytes)."""
    if arch != ARCH:
        raise CompileError(f"only gfx950 is supported, got {arch}")
    flags = DEFAULT_HIP_FLAGS + list(options or [])
    pch = None
    first, _, rest = source.partition("\n")
    if first.strip() == _TL_INCLUDE_LINE:
        pch = precompiled_header(flags, arch, verbose)
    with tempfile.TemporaryDirectory(prefix="tl_hip_") as d:
        src = Path(d) / "kernel.hip"
        out = Path(d) / ("kernel.s" if asm else "kernel.hsaco")

        def run(use_pch):
            # the PCH replaces line 1; the blank line keeps the diagnostics' line numbers
            src.write_text(("\n" + rest) if use_pch else source)
            cmd = _base_cmd(arch) + flags
            if use_pch:
                cmd += ["-Xclang", "-include-pch", "-Xclang", use_pch, "-Xclang", "-fno-validate-pch"]
            if asm:
                cmd += ["-S"]
            cmd += ["-o", str(out), str(src)]
            if verbose:
                print(" ".join(cmd))
            return cmd, subprocess.run(cmd, capture_output=True, text=True)

        cmd, r = run(pch)
        if r.returncode != 0 and pch:
            cmd, r = run(None)
            if r.returncode == 0:
                # only the PCH compile failed: the toolchain rejects the PCH, drop it for this
                # process.  A kernel that fails both ways has an error of its own (an autotune
                # config that does not compile) and keeps the PCH for every later kernel
                with _pch_lock:
                    for k, v in list(_pch_paths.items()):
                        if v == pch:
                            _pch_paths[k] = None
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
