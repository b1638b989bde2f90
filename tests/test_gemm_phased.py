"""K-half phased GEMM main loop (transform/gemm_ksplit.py + pipeline.py ``_phased_schedule``)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "gemm"))

import tilelang  # noqa: E402
from example_gemm import matmul  # noqa: E402


def _src(M, N, K, phased=None, bk=64, stages=2, prefetch=None):
    f = matmul.get_tir(M, N, K, 256, 256, bk, 512, stages, "float16")
    cfg = {} if phased is None else {"tl.gemm_phased": phased}
    if prefetch is not None:
        cfg["tl.gemm_prefetch"] = prefetch
    return tilelang.lower(f, target="hip", pass_configs=cfg).kernel_source


def test_phased_structure():
    src = _src(4096, 4096, 4096, prefetch=False)
    body = src[src.index("for (int k"):]
    # two K-half GEMMs (K = 32 each) per iteration, counted waits, vmcnt(0) only on the last iteration
    assert body.count("tl::gemm_ss<half_t, 256, 256, 32,") == 2
    assert "wait_vmcnt<8>" in body and body.count("tl::barrier_raw") >= 2
    assert "A_shared_k0" in src and "B_shared_k1" in src


def test_prefetch_structure():
    """Default: fragments of the next K half are read one phase ahead of their MFMAs, from the
    bank the phase does not refill; the 256x256 tile runs 2x4 waves (fewer LDS reads)."""
    src = _src(4096, 4096, 4096)
    pre, body = src[:src.index("for (int k")], src[src.index("for (int k"):]
    assert pre.count("tl::ss_frags<half_t, 256, 256, 32, 2, 4>") == 2
    assert "tl::gemm_ss_load" in pre and "wait_vmcnt<12>" in pre
    assert body.count("tl::gemm_ss_load<") == 2 and body.count("tl::gemm_ss_mma<half_t, 256, 256, 32, 2, 4, 16>") == 2
    # the even phase refills bank 0 and reads bank 1; the odd phase the other way round
    even, odd = body.split("tl::gemm_ss_mma", 1)
    assert "&A_shared_k0" in even.split("gemm_ss_load")[0] and "A_shared_k1" in even.split("gemm_ss_load")[1]
    assert "tl::gemm_ss<" not in body


def test_prefetch_valid_m_structure():
    """T.gemm(valid_m=) in the prefetched schedule: one uniform branch per phase around the
    fragment load AND the MFMAs (same basic block, so the 1:1 interleave still applies)."""
    from tilelang.ops.moe import expert_gemm_sk_kernel, max_padded_rows
    mr = max_padded_rows(4096, 8, 256)
    k = expert_gemm_sk_kernel(mr, 2048, 4096, 8, "bfloat16", "hip", 256, phased=True, skip_padding=True,
                              block_N=256, block_K=64, num_stages=2, threads=512, quad=False)
    src = k.get_kernel_source()
    body = src[src.index("for (int k"):]
    guard = "if ((((wave_ / 2) * 64) < nrows[0])) {"
    assert body.count(guard) >= 2
    for part in body.split(guard)[1:3]:
        head = part[:part.index("}")]
        assert "tl::gemm_ss_load<" in head and "tl::gemm_ss_mma<" in head


def test_phased_opt_out_and_shape_gate():
    src = _src(4096, 4096, 4096, phased=False)
    assert "A_shared_k0" not in src and "gemm_ss<half_t, 256, 256, 64," in src
    # BK != 64 or 3-stage rings keep the plain schedule
    assert "A_shared_k0" not in _src(4096, 4096, 4096, bk=32, stages=4)


def test_phased_config_validation():
    f = matmul.get_tir(256, 256, 256, 256, 256, 64, 512, 2, "float16")
    with pytest.raises(ValueError):
        tilelang.lower(f, target="hip", pass_configs={"tl.gemm_phased": "fast"})
    assert "setprio" in tilelang.lower(f, target="hip", pass_configs={"tl.gemm_phased": "prio"}).kernel_source


@pytest.mark.gpu
@pytest.mark.parametrize("K", [64, 128, 192, 1024])
@pytest.mark.parametrize("phased", [True, "prio", "noprefetch", "noilv"])
def test_phased_numerics(K, phased):
    """1, 2, 3 and 16 K-tiles: the prologue / last-iteration waits of the phased ring (with and
    without the register-prefetched fragments)."""
    M, N = 512, 768
    f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, "float16")
    cfg = {"tl.gemm_phased": phased} if phased in (True, "prio") else {
        "tl.gemm_prefetch": False} if phased == "noprefetch" else {"tl.gemm_interleave": False}
    k = tilelang.compile(f, out_idx=[-1], target="hip", pass_configs=cfg)
    assert "A_shared_k0" in k.get_kernel_source()
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(K, N, device="cuda", dtype=torch.float16)
    c = k(a, b)
    torch.testing.assert_close(c.float(), a.float() @ b.float(), rtol=1e-2, atol=1e-2 * K ** 0.5)


def _nt_src(M, N, K, threads=512, dtype="float16", **cfg):
    f = matmul.get_tir(M, N, K, 256, 256, 64, threads, 2, dtype, trans_B=True, staged_epilogue=True)
    return tilelang.lower(f, target="hip", pass_configs=cfg).kernel_source


def test_quad_structure():
    """The 256x256x64 NT tile on 512 threads runs the whole K loop as tl::gemm_quad_nt
    (tl/gemm_quad.h); tl.gemm_quad=False, NN layouts and other block sizes keep the K-half
    schedule."""
    src = _nt_src(4096, 4096, 4096)
    assert src.count("tl::gemm_quad_nt_x<half_t, false, 0>(") == 1 and "gemm_ss_load" not in src
    assert "for (int k" not in src
    assert "tl::gemm_quad_nt_x<bfloat16_t, false, 0>(" in _nt_src(512, 768, 192, dtype="bfloat16")
    off = _nt_src(4096, 4096, 4096, **{"tl.gemm_quad": False})
    assert "gemm_quad" not in off and "A_shared_k0" in off
    assert "gemm_quad" not in _src(4096, 4096, 4096)  # NN
    assert "gemm_quad" not in _nt_src(4096, 4096, 4096, threads=256)


def test_quad_moe_structure():
    """The MoE expert GEMMs (row gather + 32-row extension GEMM + valid_m; dense A with an
    unprovable row range) take the quad loop with the range-checked row modes."""
    from tilelang.ops.moe import expert_gemm_sk_kernel, max_padded_rows
    mr = max_padded_rows(4096, 8, 288)
    g1 = expert_gemm_sk_kernel(mr, 4096, 4096, 8, "bfloat16", "hip", 256, n_src=2048, swiglu=True, ext_M=32,
                               block_N=256, block_K=64, num_stages=2, threads=512).get_kernel_source()
    assert "tl::gemm_quad_nt_x<bfloat16_t, true, 32>((&A[0]), 4096, (&row_src[" in g1
    g2 = expert_gemm_sk_kernel(mr, 2048, 4096, 8, "bfloat16", "hip", 256, ext_M=32, block_N=256, block_K=64,
                               num_stages=2, threads=512).get_kernel_source()
    assert "tl::gemm_quad_nt_x<bfloat16_t, true, 32>((&A[0]), 2048, tl::quad::no_rows()," in g2
    # the narrow tail tiles (256 x 64) keep the generic pipeline
    assert "for (int k" in g2


def _fp8_src(K, dtype="float8_e4m3fn", **cfg):
    sys.path.insert(0, os.path.join(ROOT, "examples", "gemm_fp8"))
    from example_tilelang_gemm_fp8 import matmul as mm8
    f = mm8.get_tir(512, 768, K, dtype=dtype, staged_epilogue=True)
    return tilelang.lower(f, target="hip", pass_configs=cfg).kernel_source


def test_quad_fp8_structure():
    """fp8 256x256x128 (128-byte K tiles, the same LDS bytes as fp16 x 64) runs on the quad loop
    with the 16x16x128 f8f6f4 MFMA; tl.gemm_quad=False keeps the generic pipeline."""
    assert "tl::gemm_quad_nt_x<fp8_e4_t, false, 0>(" in _fp8_src(4096)
    assert "tl::gemm_quad_nt_x<fp8_e5_t, false, 0>(" in _fp8_src(256, dtype="float8_e5m2")
    assert "gemm_quad" not in _fp8_src(4096, **{"tl.gemm_quad": False})


@pytest.mark.gpu
@pytest.mark.parametrize("K", [128, 256, 384, 2048, 8320])
@pytest.mark.parametrize("dtype", ["float8_e4m3fn", "float8_e5m2"])
def test_quad_fp8_numerics(K, dtype):
    """fp8 quad loop (1, 2, 3, 16, 65 K tiles) against the fp32 product of the same fp8 values."""
    sys.path.insert(0, os.path.join(ROOT, "examples", "gemm_fp8"))
    from example_tilelang_gemm_fp8 import matmul as mm8
    M, N = 512, 768
    k = tilelang.compile(mm8.get_tir(M, N, K, dtype=dtype, staged_epilogue=True), out_idx=[-1], target="hip")
    assert "gemm_quad_nt_x<fp8_e" in k.get_kernel_source()
    td = getattr(torch, dtype)
    for _ in range(2):
        a = torch.randn(M, K, device="cuda").to(td)
        b = torch.randn(N, K, device="cuda").to(td)
        c = k(a, b)
        ref = a.float() @ b.float().T
        torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=2e-2 * K ** 0.5)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [64, 128, 192, 1024, 4160])
@pytest.mark.parametrize("dtype", ["float16", "bfloat16"])
def test_quad_numerics(K, dtype):
    """1, 2, 3, 16 and 65 K tiles (odd counts end on a half iteration) against fp32 torch."""
    M, N = 512, 768
    f = matmul.get_tir(M, N, K, 256, 256, 64, 512, 2, dtype, trans_B=True, staged_epilogue=True)
    k = tilelang.compile(f, out_idx=[-1], target="hip")
    assert "gemm_quad_nt" in k.get_kernel_source()
    td = getattr(torch, dtype)
    a = torch.randn(M, K, device="cuda", dtype=td)
    b = torch.randn(N, K, device="cuda", dtype=td)
    for _ in range(2):  # a rerun with new data: stale LDS would show here
        c = k(a, b)
        ref = a.float() @ b.float().T
        torch.testing.assert_close(c.float(), ref, rtol=2e-2, atol=2e-2 * K ** 0.5)
        a = torch.randn_like(a)
