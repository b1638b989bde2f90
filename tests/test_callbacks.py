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


def test_hooks_with_same_body_different_closures_get_different_keys():
    """A hook built in a loop (same bytecode, different captured values) must not be served
    the kernel compiled under its sibling (hook_fingerprint hashed only co_code)."""
    srcs = []
    for tag in ("// variant-a", "// variant-b"):
        callback.register_hip_postproc(lambda code, target: tag + "\n" + code)
        try:
            srcs.append(tilelang.compile(_prog(2048), out_idx=[1], target="hip").get_kernel_source())
        finally:
            callback.unregister()
    assert srcs[0].startswith("// variant-a") and srcs[1].startswith("// variant-b")


def test_compiler_fingerprint_covers_native_core():
    from tilelang.cache import kernel_cache
    import hashlib
    from pathlib import Path
    import tilelang as tl
    sos = sorted(Path(tl.__file__).parent.glob("_tl_*.so"))
    assert sos, "native extensions must be built in-tree"
    fp = kernel_cache.compiler_fingerprint()
    assert isinstance(fp, str) and len(fp) == 64
