"""Carver (config recommender), static analyzer, layout plotting and quantisation helpers (CPU)."""
import os

import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang import quantize as Q
from tilelang.carver.arch import CDNA
from tilelang.carver.template import (ElementwiseTemplate, FlashAttentionTemplate, GEMVTemplate, MatmulTemplate)


def test_carver_matmul_hints_fit_hardware():
    arch = CDNA("hip")
    hints = MatmulTemplate(M=4096, N=4096, K=4096).with_arch(arch).recommend_hints(topk=8)
    assert hints and all(h.estimated_us > 0 for h in hints)
    for h in hints:
        cfg = h.to_config()
        eb = 2
        assert cfg["num_stages"] * (cfg["block_M"] + cfg["block_N"]) * cfg["block_K"] * eb <= 160 * 1024
        assert cfg["threads"] % 64 == 0
    assert hints == sorted(hints, key=lambda h: h.estimated_us)
    # big square GEMMs want big tiles and rasterisation
    assert hints[0].block[0] * hints[0].block[1] >= 128 * 128
    small = MatmulTemplate(M=16, N=8192, K=8192).with_arch(arch).recommend_hints(topk=3)
    assert small[0].block[0] <= 64


def test_carver_other_templates():
    arch = CDNA("hip")
    assert FlashAttentionTemplate(heads=64, seq_len=4096).with_arch(arch).recommend_hints(3)
    g = GEMVTemplate(N=16384, K=16384).with_arch(arch).recommend_hints(3)
    assert set(g[0].to_config()) >= {"block_N", "block_K", "threads"}
    e = ElementwiseTemplate(shape=[8192, 8192], dtype="float32").with_arch(arch).recommend_hints(3)
    assert e and e[0].threads in (128, 256, 512)


def test_carver_hints_drive_a_kernel_factory():
    from example_gemm import matmul
    hint = MatmulTemplate(M=256, N=256, K=256).with_arch(CDNA()).recommend_hints(topk=1)[0]
    c = hint.to_config()
    f = matmul.get_tir(256, 256, 256, c["block_M"], c["block_N"], c["block_K"], c["threads"], c["num_stages"])
    k = tilelang.compile(f, out_idx=[-1], target="cpu")
    a, b = torch.randn(256, 256).half(), torch.randn(256, 256).half()
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float(), rtol=1e-2, atol=1e-2)


def test_static_analyzer_counts_gemm_flops_and_bytes():
    from tilelang.tools import Analyzer
    from example_gemm import matmul
    f = matmul.get_tir(1024, 1024, 1024, 128, 128, 32, 256, 2)
    r = Analyzer.analysis(f, "MI355X")
    assert r.total_flops == pytest.approx(2 * 1024**3)
    # A and B tiles are re-read once per output tile; C written once
    assert r.total_global_bytes == pytest.approx((1024 * 1024 * 2) * (1024 // 128) * 2 + 1024 * 1024 * 2)
    assert r.bound == "memory" and r.estimated_time_us > 0  # tile re-reads counted as HBM traffic (no L2 model)


def test_plot_layout_writes_grid(tmp_path):
    from tilelang.layout import mfma as MF
    from tilelang.tools import plot_layout, layout_text
    frag = MF.mfma_c_fragment(16, 16, 1, 1)
    txt = layout_text(frag)
    assert txt.count("T") == 16 * 16
    p = plot_layout(frag, str(tmp_path), "c16", "txt,svg")
    assert os.path.exists(p) and os.path.exists(os.path.join(tmp_path, "c16.svg"))


def test_int4_and_mxfp4_roundtrip():
    W = torch.randn(64, 256)
    packed, s = Q.quantize_int4_groupwise(W, 128)
    assert packed.shape == (64, 128) and packed.dtype == torch.uint8
    assert (Q.dequantize_int4_groupwise(packed, s, 128) - W).abs().max() <= s.max() * 0.51
    pk, e = Q.quantize_mxfp4(W, 32)
    deq = Q.dequantize_mxfp4(pk, e, 32)
    rel = (deq - W).abs() / W.abs().clamp(min=1e-3)
    assert rel.median() < 0.15
    codes = torch.arange(16, dtype=torch.uint8)
    assert torch.equal(Q.float_to_e2m1(Q.e2m1_to_float_torch(codes)) & 0xF,
                       torch.where(codes == 8, 0, codes).to(torch.uint8))


@tilelang.jit(out_idx=[-1], target="cpu")
def _deq_kernel(N, K):

    @T.prim_func
    def main(P: T.Tensor((N, K // 2), "uint8"), E: T.Tensor((N, K // 32), "uint8"), O: T.Tensor((N, K), "float32")):
        with T.Kernel(1, is_cpu=True):
            for n, k in T.Parallel(N, K):
                O[n, k] = Q.fp4_to_float(P[n, k // 2], k % 2) * Q.e8m0_to_float(E[n, k // 32])

    return main


def test_dsl_dequant_expressions_match_host():
    W = torch.randn(8, 64)
    pk, e = Q.quantize_mxfp4(W, 32)
    out = _deq_kernel(8, 64)(pk, e)
    torch.testing.assert_close(out, Q.dequantize_mxfp4(pk, e, 32))


def test_math_testing_utils_libinfo():
    import torch

    import tilelang
    import tilelang.language as T
    from tilelang.utils.language import (is_fragment, is_global, is_shared, legalize_pairwise_extents,
                                         retrieve_shape)
    assert tilelang.cdiv(7, 2) == 4 and tilelang.math.next_power_of_2(33) == 64
    assert tilelang.math.next_power_of_2(1) == 1 and tilelang.math.prev_power_of_2(33) == 32
    tilelang.testing.set_random_seed(3)
    a = torch.rand(4)
    tilelang.testing.set_random_seed(3)
    assert torch.equal(a, torch.rand(4))
    tilelang.testing.torch_assert_close(a, a + 1e-4)
    try:
        tilelang.testing.torch_assert_close(a, a + 1)
        raise RuntimeError("expected a mismatch")
    except AssertionError as e:
        assert "mismatched" in str(e)
    assert tilelang.libinfo.find_lib_path("_tl_runtime")
    assert legalize_pairwise_extents([1, 64, 32], [64, 32]) == ([64, 32], [64, 32])

    @T.prim_func
    def f(A: T.Tensor((64, 64), "float16")):
        with T.Kernel(1, threads=64):
            s = T.alloc_shared((16, 64), "float16")
            r = T.alloc_fragment((16, 64), "float")
            assert is_global(A) and is_shared(s) and is_fragment(r)
            assert [int(x) for x in retrieve_shape(A[0:16, :])] == [16, 64]
            T.copy(A[0:16, :], s)
            T.copy(s, r)


def test_precision_probe_cpu():
    """maint/precision counterpart: the probe runs every op and reports float64-referenced errors."""
    from tilelang.tools import precision as P
    res = P.run("cpu", n=1 << 12, ops=["exp", "div", "log", "rsqrt"])
    for op, rows in res.items():
        assert set(rows) == {"TileLang (precise)", "TileLang (fast math)", "PyTorch"}
        assert rows["TileLang (precise)"]["max_ulp"] <= 4.0, (op, rows)
    md = P.to_markdown(res, "cpu")
    assert "### exp" in md and "Max ULP" in md


@pytest.mark.gpu
def test_precision_probe_gpu():
    """gfx950: precise OCML paths within a few ULP; the hardware fast-math transcendentals the
    attention kernels use stay within float32-softmax tolerance."""
    from tilelang.tools import precision as P
    res = P.run("cuda", n=1 << 16)
    for op, rows in res.items():
        assert rows["TileLang (precise)"]["max_ulp"] <= 4.0, (op, rows["TileLang (precise)"])
        assert rows["TileLang (precise)"]["nonfinite"] == 0
    assert res["exp"]["TileLang (fast math)"]["max_rel"] < 1e-5
    assert res["exp2"]["TileLang (fast math)"]["max_rel"] < 1e-5


def test_carver_bestfit_packing():
    from tilelang.carver.roller.bestfit import BestFit, pack, gemm_lds_bytes
    a = BestFit(16)
    x, y = a.malloc(100), a.malloc(50)
    assert (x.start, y.start) == (0, 112)
    a.free(x)
    z = a.malloc(40)  # best fit reuses the freed hole
    assert z.start == 0 and a.limit == 112 + 64
    # disjoint lifetimes share bytes; overlapping ones do not
    size, off = pack([("ring", 1024, 0, 2), ("epi", 512, 2, 3)])
    assert size == 1024 and off["epi"] == 0
    size, _ = pack([("a", 1024, 0, 2), ("b", 512, 1, 3)])
    assert size == 1536
    # the staged GEMM epilogue (256 x 264 fp16) reuses the 2-stage 256x256x64 ring: max, not sum
    assert gemm_lds_bytes(256, 256, 64, 2, 2) == 131072
    assert gemm_lds_bytes(256, 256, 64, 2, 2, staged_epilogue=True) == 256 * 264 * 2


def test_carver_conv_and_reduction_hints_drive_kernels():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "examples", "convolution"))
    sys.path.insert(0, os.path.join(root, "examples", "norm"))
    from tilelang.carver.template import ConvTemplate, GeneralReductionTemplate
    from example_convolution import convolution
    from rms_norm import rms_norm, ref_program as rms_ref
    arch = CDNA()
    # implicit-GEMM conv: N*OH*OW x F x KH*KW*C
    hints = ConvTemplate(N=2, C=64, H=16, W=16, F=64, K=3, S=1, D=1, P=1).with_arch(arch).recommend_hints(4)
    assert hints
    c = hints[0].to_config()
    f = convolution.get_tir(2, 64, 16, 16, 64, 3, 1, 1, 1, c["block_M"], c["block_N"], c["block_K"],
                            c["num_stages"], c["threads"])
    k = tilelang.compile(f, out_idx=[-1], target="cpu")
    x = torch.randn(2, 16, 16, 64).half()
    w = torch.randn(3, 3, 64, 64).half()
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(3, 2, 0, 1).float(), padding=1)
    torch.testing.assert_close(k(x, w).float(), ref.permute(0, 2, 3, 1), rtol=2e-2, atol=5e-1)
    # row reduction (RMS norm): whole rows in registers, blk_m rows per block
    r = GeneralReductionTemplate(shape=[8192, 8192], dtype="float32").with_arch(arch).recommend_hints(4)
    assert r and all(h.score["per_lane"] <= 64 for h in r)
    small = GeneralReductionTemplate(shape=[64, 256], dtype="float32").with_arch(arch).recommend_hints(1)[0]
    cfg = small.to_config()
    assert set(cfg) == {"blk_m", "threads"}
    kr = tilelang.compile(rms_norm.get_tir(64, 256, cfg["blk_m"], cfg["threads"]), out_idx=[-1], target="cpu")
    a = torch.randn(64, 256)
    torch.testing.assert_close(kr(a), rms_ref(a), rtol=1e-4, atol=1e-4)
