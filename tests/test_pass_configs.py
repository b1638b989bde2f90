"""Every PassConfigKey either changes the compile or is rejected (never silently ignored)."""
import os

import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang.transform.pass_config import PassConfigKey, EFFECT, SATISFIED, UNSUPPORTED, validate_pass_configs


def add_kernel(M=256, N=256, dyn=False):
    m = T.dynamic("m") if dyn else M

    @T.prim_func
    def main(A: T.Tensor((m, N), "float32"), B: T.Tensor((m, N), "float32"), C: T.Tensor((m, N), "float32")):
        with T.Kernel(T.ceildiv(m, 32), threads=128) as bx:
            for i, j in T.Parallel(32, N):
                C[bx * 32 + i, j] = T.exp(A[bx * 32 + i, j]) + B[bx * 32 + i, j]

    return main


def test_every_key_is_classified():
    for k in PassConfigKey:
        assert k.value in EFFECT or k.value in SATISFIED or k.value in UNSUPPORTED, k


def test_unknown_and_unsupported_keys_raise():
    with pytest.raises(ValueError, match="unknown pass config"):
        validate_pass_configs({"tl.no_such_key": True})
    with pytest.raises(NotImplementedError):
        validate_pass_configs({"tl.ptxas_register_usage_level": 10})
    assert validate_pass_configs({"tl.storage_rewrite_detect_inplace": True})
    with pytest.raises(ValueError):
        validate_pass_configs({"tl.config_index_bitwidth": 16})
    assert validate_pass_configs({"tl.disable_tma_lower": True, "tl.disable_warp_specialized": True})


def _src(**cfg):
    return tilelang.compile(add_kernel(), target="hip", pass_configs=cfg).get_kernel_source()


def test_fast_math_and_vectorize_keys_change_code():
    base = _src()
    assert "fast_exp" in _src(**{"tl.enable_fast_math": True})
    assert "fast_exp" not in _src(**{"tl.enable_fast_math": True, "tl.disable_fast_math": True})
    assert "load_vec" in base or "store_vec" in base
    nv = _src(**{"tir.disable_vectorize": True})
    assert "load_vec" not in nv and "store_vec" not in nv


def test_disable_safe_memory_and_thread_sync():
    dyn = tilelang.compile(add_kernel(dyn=True), target="hip").get_kernel_source()
    nodyn = tilelang.compile(add_kernel(dyn=True), target="hip",
                             pass_configs={"tl.disable_safe_memory_legalize": True}).get_kernel_source()
    assert dyn != nodyn


def test_dynamic_alignment_enables_vector_access():
    n = T.dynamic("n")

    @T.prim_func
    def f(A: T.Tensor((64, n), "float32"), B: T.Tensor((64, n), "float32")):
        with T.Kernel(T.ceildiv(n, 128), threads=128) as bx:
            for i, j in T.Parallel(64, 128):
                B[i, bx * 128 + j] = A[i, bx * 128 + j] * 2.0

    plain = tilelang.compile(f, target="hip").get_kernel_source()
    al = tilelang.compile(f, target="hip", pass_configs={"tl.dynamic_alignment": 8}).get_kernel_source()
    assert "load_vec" not in plain and "load_vec" in al


def test_force_let_inline_numerics():

    @T.prim_func
    def f(A: T.Tensor((64, ), "float32"), B: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=64):
            for i in T.Parallel(64):
                x = A[i] * 2.0
                B[i] = x + 1.0

    k = tilelang.compile(f, target="cpu", pass_configs={"tl.force_let_inline": True})
    a = torch.randn(64)
    b = torch.zeros(64)
    k(a, b)
    torch.testing.assert_close(b, a * 2 + 1)


def test_layout_visualization_dump(tmp_path, monkeypatch):
    monkeypatch.setenv("TILELANG_LAYOUT_DIR", str(tmp_path))
    import example_gemm
    f = example_gemm.matmul.get_tir(128, 128, 128, 64, 64, 32, 128, 2)
    tilelang.compile(f, out_idx=[-1], target="hip", pass_configs={"tl.layout_visualization_enable": True,
                                                                  "tl.layout_visualization_formats": "txt,svg"})
    files = os.listdir(tmp_path)
    assert any(x.endswith(".layouts.txt") for x in files)
    assert any(x.endswith(".svg") for x in files)
    txt = open(os.path.join(tmp_path, [x for x in files if x.endswith(".layouts.txt")][0])).read()
    assert "C_local" in txt and "A_shared" in txt


def test_use_async_copy_false_disables_lds_dma():
    import example_gemm
    f = example_gemm.matmul.get_tir(256, 256, 256, 128, 128, 32, 256, 2)
    on = tilelang.compile(f, out_idx=[-1], target="hip").get_kernel_source()
    off = tilelang.compile(f, out_idx=[-1], target="hip",
                           pass_configs={"tir.use_async_copy": False}).get_kernel_source()
    assert "glds16" in on and "glds16" not in off


def test_lds_reuse_shares_bytes():

    @T.prim_func
    def f(A: T.Tensor((64, 64), "float32"), B: T.Tensor((64, 64), "float32")):
        with T.Kernel(1, threads=256):
            S1 = T.alloc_shared((64, 64), "float32")
            S2 = T.alloc_shared((64, 64), "float32")
            T.copy(A, S1)
            T.copy(S1, B)
            T.copy(B, S2)
            T.copy(S2, A)

    on = tilelang.compile(f, target="hip")
    off = tilelang.compile(f, target="hip", pass_configs={"tl.lds_reuse": False})
    assert on.artifact.lds_bytes == 16384 and off.artifact.lds_bytes == 32768
    k = tilelang.compile(f, target="cpu")
    a = torch.randn(64, 64)
    b = torch.zeros(64, 64)
    a0 = a.clone()
    k(a, b)
    torch.testing.assert_close(b, a0)
    torch.testing.assert_close(a, a0)
