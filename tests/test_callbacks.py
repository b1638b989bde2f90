"""Source post-processing / compile hooks (reference tilelang/engine/callback.py)."""
import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang.engine import callback


@pytest.fixture(autouse=True)
def _fresh_cache(tmp_path, monkeypatch):
    """Hooks run at compile time: a kernel found in the on-disk cache (same program and hook
    fingerprint from an earlier run) would skip them, so every test compiles into an empty cache."""
    from tilelang import env
    monkeypatch.setattr(env, "TILELANG_CACHE_DIR", str(tmp_path))


def _prog(n=256):

    @T.prim_func
    def main(A: T.Tensor((n, ), "float32"), B: T.Tensor((n, ), "float32")):
        with T.Kernel(n // 64, threads=64) as bx:
            for i in T.Parallel(64):
                B[bx * 64 + i] = A[bx * 64 + i] * 2.0

    return main


def test_hip_postproc_rewrites_source_and_keys_cache():
    seen = []

    @callback.register_hip_postproc_callback
    def tag(code, target):
        seen.append(target)
        return "// postproc-was-here\n" + code

    try:
        k = tilelang.compile(_prog(), out_idx=[1], target="hip")
        assert k.get_kernel_source().startswith("// postproc-was-here") and seen
        assert len(k.code[0]) > 0
    finally:
        callback.unregister()
    k2 = tilelang.compile(_prog(), out_idx=[1], target="hip")
    assert "postproc-was-here" not in k2.get_kernel_source()  # the hook is part of the cache key


def test_hip_compile_hook_and_validation():
    from tilelang.contrib import hipcc
    calls = []

    @callback.register_hip_compile_callback(override=True)
    def comp(code, target):
        calls.append(len(code))
        return hipcc.compile_hip(code)

    try:
        k = tilelang.compile(_prog(512), out_idx=[1], target="hip")
        assert calls and k.code[0][:4] == b"\x7fELF"
        with pytest.raises(ValueError):
            callback.register_hip_compile(comp, override=False)
        callback.register_hip_compile(lambda c, t: b"not-elf")
        with pytest.raises(TypeError):
            tilelang.compile(_prog(1024), out_idx=[1], target="hip")
    finally:
        callback.unregister()


def test_cuda_postproc_is_refused():
    with pytest.raises(NotImplementedError):
        callback.register_cuda_postproc(lambda c, t: c)


def test_cpu_target_unaffected():
    callback.register_hip_postproc(lambda c, t: c + "\n#error must not reach the cpu compiler\n")
    try:
        k = tilelang.compile(_prog(), out_idx=[1], target="cpu")
        a = torch.randn(256)
        torch.testing.assert_close(k(a), a * 2)
    finally:
        callback.unregister()
