"""Whole-kernel disk cache (tilelang/cache/kernel_cache.py)."""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm"))

import tilelang  # noqa: E402
from tilelang.cache import kernel_cache  # noqa: E402
from tilelang.jit import JITKernel, _GLOBAL_JIT_CACHE  # noqa: E402
from example_gemm import matmul  # noqa: E402


def test_disk_cache_roundtrip(tmp_path, monkeypatch):
    monkeypatch.setenv("TILELANG_CACHE_DIR", str(tmp_path))
    _GLOBAL_JIT_CACHE.clear()
    f = matmul.get_tir(128, 128, 128, 64, 64, 32, 128, 2, "float16")
    assert JITKernel.from_database(f, out_idx=[-1], target="cpu") is None
    k1 = tilelang.compile(f, out_idx=[-1], target="cpu")
    assert not k1.from_disk_cache and kernel_cache.entries() == 1
    _GLOBAL_JIT_CACHE.clear()
    k2 = tilelang.compile(f, out_idx=[-1], target="cpu")
    assert k2.from_disk_cache
    assert k2.get_kernel_source() == k1.get_kernel_source()
    a = torch.randn(128, 128, dtype=torch.float16)
    b = torch.randn(128, 128, dtype=torch.float16)
    torch.testing.assert_close(k2(a, b), k1(a, b))
    k3 = JITKernel.from_database(f, out_idx=[-1], target="cpu")
    assert k3 is not None and k3.from_disk_cache
    # any option change is a different entry
    _GLOBAL_JIT_CACHE.clear()
    k4 = tilelang.compile(f, out_idx=[-1], target="cpu", pass_configs={"tir.disable_vectorize": True})
    assert not k4.from_disk_cache and kernel_cache.entries() == 2
    tilelang.disable_cache()
    try:
        assert kernel_cache.load(kernel_cache.kernel_key(f, k1.target, [-1], {}, [])) is None
    finally:
        tilelang.enable_cache()


def test_disk_cache_across_processes(tmp_path):
    code = ("import sys; sys.path.insert(0, %r); import tilelang; from example_gemm import matmul; "
            "f = matmul.get_tir(128, 128, 64, 64, 64, 32, 128, 2, 'float16'); "
            "k = tilelang.compile(f, out_idx=[-1], target='cpu'); print('HIT' if k.from_disk_cache else 'MISS')"
            % os.path.join(ROOT, "examples", "gemm"))
    env = dict(os.environ, TILELANG_CACHE_DIR=str(tmp_path), PYTHONPATH=ROOT)
    outs = [subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            for _ in range(2)]
    assert [o.stdout.strip().splitlines()[-1] for o in outs] == ["MISS", "HIT"], [o.stderr[-2000:] for o in outs]


def test_annotated_layout_changes_cache_key():
    """A user layout (T.annotate_layout) changes the generated code, so it must change the key."""
    f0 = matmul.get_tir(256, 256, 256, 256, 256, 64, 512, 2, "float16", staged_epilogue=True)
    import tilelang.language as T  # noqa: F401
    from tilelang.layout import PaddedLayout
    k0 = kernel_cache.kernel_key(f0, "hip", [-1], {}, [])
    f1 = matmul.get_tir(256, 256, 256, 256, 256, 64, 512, 2, "float16", staged_epilogue=True)
    bufs = [s.buffer for s in __import__("tilelang.ir.stmt", fromlist=["walk"]).walk(f1.body)
            if type(s).__name__ == "AllocStmt" and s.buffer.name == "C_shared"]
    bufs[0].layout = PaddedLayout((256, 256), 16)
    assert kernel_cache.kernel_key(f1, "hip", [-1], {}, []) != k0
