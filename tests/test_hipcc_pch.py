"""Precompiled tl/tl.h (contrib/hipcc.py precompiled_header): the PCH compile emits the same gfx950
code as the plain compile, is built once per flag set, and a PCH the toolchain rejects falls
back to the plain compile."""
import os
import subprocess

import pytest

from tilelang.contrib import hipcc

SRC = '''#include "tl/tl.h"

extern "C" __global__ void __launch_bounds__(256) add_kernel(float* __restrict__ A, float* __restrict__ B) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  B[i] = A[i] * 2.0f + tl::quad::uni(i);
}
'''


def _text(code: bytes, tmp_path, name):
    p = tmp_path / name
    p.write_bytes(code)
    objdump = os.path.join(os.path.dirname(hipcc.clang_path()), "llvm-objdump")
    out = subprocess.run([objdump, "-d", str(p)], capture_output=True, text=True, check=True).stdout
    return [ln for ln in out.splitlines() if "file format" not in ln]


@pytest.fixture
def fresh_cache(tmp_path, monkeypatch):
    monkeypatch.setenv("TILELANG_CACHE_DIR", str(tmp_path / "cache"))
    monkeypatch.setattr(hipcc, "_pch_paths", {})
    return tmp_path


def test_pch_same_code(fresh_cache, monkeypatch):
    tmp = fresh_cache
    monkeypatch.setenv("TL_HIP_PCH", "1")
    with_pch = hipcc.compile_hip(SRC)
    pchs = [p for p in hipcc._pch_paths.values() if p]
    assert len(pchs) == 1 and os.path.exists(pchs[0])
    again = hipcc.compile_hip(SRC)  # reuses it
    assert [p for p in hipcc._pch_paths.values() if p] == pchs
    monkeypatch.setenv("TL_HIP_PCH", "0")
    plain = hipcc.compile_hip(SRC)
    assert _text(with_pch, tmp, "a.co") == _text(plain, tmp, "b.co") == _text(again, tmp, "c.co")


def test_pch_rejected_falls_back(fresh_cache, monkeypatch):
    monkeypatch.setenv("TL_HIP_PCH", "1")
    hipcc.compile_hip(SRC)
    (pch, ) = [p for p in hipcc._pch_paths.values() if p]
    with open(pch, "wb") as f:
        f.write(b"not a pch")
    code = hipcc.compile_hip(SRC)  # the broken PCH is dropped, the plain compile runs
    assert code and all(v is None for v in hipcc._pch_paths.values())


def test_no_pch_for_other_sources(fresh_cache, monkeypatch):
    monkeypatch.setenv("TL_HIP_PCH", "1")
    hipcc.compile_hip("#include <hip/hip_runtime.h>\nextern \"C\" __global__ void k(float* a) { a[0] = 1.f; }\n")
    assert hipcc._pch_paths == {}


def _compile_in_child(cache):
    os.environ["TILELANG_CACHE_DIR"] = cache
    os.environ["TL_HIP_PCH"] = "1"
    from tilelang.contrib import hipcc as h
    return len(h.compile_hip(SRC)), [p for p in h._pch_paths.values() if p]


def test_pch_concurrent_builders(tmp_path):
    """Several processes building the same PCH at once: each writes a private temp file and
    renames it into place, so every compile succeeds and one PCH file remains."""
    import multiprocessing as mp
    cache = str(tmp_path / "cache")
    with mp.get_context("spawn").Pool(3) as pool:
        res = pool.map(_compile_in_child, [cache] * 3)
    assert all(n > 0 for n, _ in res)
    pchs = {p for _, ps in res for p in ps}
    assert len(pchs) == 1 and os.path.exists(pchs.pop())
    assert sorted(os.listdir(os.path.join(cache, "pch"))) == sorted(
        [os.path.basename(p) for _, ps in res for p in ps][:1] + ["tl_pch.h"])
