"""The carver's GEMM cost model is calibrated against measured MI355X kernels (carver/roller/policy.py
LOOP_EFF): it knows which tilings the compiler turns into the tl::gemm_quad_nt_x main loop, the
K-half phased loop or the generic pipeline, and ranks the measured-best tiling first (reference:
tilelang/carver/roller/policy/tensorcore.py, tilelang/carver/template/matmul.py)."""
import os
import sys

import pytest

from tilelang.carver.arch import CDNA
from tilelang.carver.roller.policy import gemm_cost, main_loop_kind, TensorCorePolicy
from tilelang.carver.template import MatmulTemplate

ARCH = CDNA("hip")

# measured on MI355X (docs/RESULTS.md): (M, N, K, dtype, tile (bm, bn, bk, threads, stages), trans_b, TFLOPS)
MEASURED = [
    (8192, 8192, 256, "float16", (256, 256, 64, 512, 2), True, 557),      # profiles/r5/benchmarks/matmul_fp16.md
    (8192, 8192, 1024, "float16", (256, 256, 64, 512, 2), True, 1031),
    (8192, 8192, 2048, "float16", (256, 256, 64, 512, 2), True, 1206),
    (8192, 8192, 4096, "float16", (256, 256, 64, 512, 2), True, 1309),
    (8192, 8192, 8192, "float16", (256, 256, 64, 512, 2), True, 1343),
    (4096, 4096, 4096, "float16", (256, 256, 64, 512, 2), True, 1311),     # RESULTS r5 (quad loop)
    (8192, 8192, 1024, "float8_e4m3fn", (256, 256, 128, 512, 2), True, 1650),  # RESULTS r5 fp8 table
    (8192, 8192, 4096, "float8_e4m3fn", (256, 256, 128, 512, 2), True, 2533),
    (8192, 8192, 8192, "float8_e4m3fn", (256, 256, 128, 512, 2), True, 2845),
    (4096, 4096, 4096, "float16", (256, 128, 64, 512, 2), True, 910),      # profiles/r3/s3/gemm/tile_shape_sweep.log
    (4096, 4096, 4096, "float16", (128, 256, 64, 512, 2), True, 1001),
    (4096, 4096, 4096, "float16", (256, 128, 64, 256, 2), True, 827),
    (4096, 4096, 4096, "float16", (256, 256, 64, 512, 2), False, 1210),    # NN: the phased K-half loop
]


@pytest.mark.parametrize("case", MEASURED, ids=[f"{c[0]}x{c[1]}x{c[2]}-{c[3]}-{c[4]}-{'NT' if c[5] else 'NN'}"
                                                 for c in MEASURED])
def test_model_within_10pct_of_measured(case):
    M, N, K, dt, (bm, bn, bk, th, st), tb, tf = case
    c = gemm_cost(ARCH, M, N, K, bm, bn, bk, th, st, dt, trans_b=tb)
    model_tf = 2.0 * M * N * K / c["us"] / 1e6
    assert abs(model_tf / tf - 1) < 0.10, (model_tf, tf, c)


def test_loop_kind_mirrors_the_compiler():
    assert main_loop_kind(256, 256, 64, 512, 2, "float16", True) == "quad"
    assert main_loop_kind(256, 256, 128, 512, 2, "float8_e4m3fn", True) == "quad_fp8"
    assert main_loop_kind(256, 256, 64, 512, 2, "float16", False) == "phased"
    assert main_loop_kind(256, 256, 32, 512, 2, "float16", True) == "generic"
    assert main_loop_kind(128, 256, 64, 512, 2, "float16", True) == "generic"
    assert main_loop_kind(256, 256, 64, 512, 3, "float16", True) == "generic"


# the measured-best tiling of each shape: the quad loop's 256 x 256 x (128 bytes) / 512 threads / 2 stages
BEST16, BEST8 = ([256, 256], [64], 512, 2), ([256, 256], [128], 512, 2)
SHAPES = [((4096, 4096, 4096), "float16", BEST16), ((8192, 8192, 8192), "float16", BEST16),
          ((8192, 8192, 4096), "float16", BEST16), ((8192, 8192, 8192), "float8_e4m3fn", BEST8),
          # the bench MoE's expert GEMMs as one grouped launch: 2048 tokens x top-2 rows over 8
          # experts; GEMM1 [rows, hidden 4096] x [2 ffn = 4096, 4096]^T, GEMM2 [rows, 2048] x [4096, 2048]^T
          ((4096, 4096, 4096), "bfloat16", BEST16), ((4096, 4096, 2048), "bfloat16", BEST16),
          ((4000, 4000, 4000), "float16", BEST16)]


@pytest.mark.parametrize("shape,dt,best", SHAPES, ids=[f"{s[0]}-{s[1]}" for s in SHAPES])
def test_top1_is_measured_best(shape, dt, best):
    h = TensorCorePolicy(ARCH, *shape, in_dtype=dt, trans_b=True).emit_config(4)[0]
    assert (h.block, h.rstep, h.threads, h.pipeline_stage) == best, h


def test_autotune_example_topk4_contains_quad_config():
    """examples/gemm/example_gemm_autotune.py with carver top-k 4 tries the quad tiling, and that
    tiling compiles to the tl::gemm_quad_nt_x main loop."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "examples", "gemm"))
    import tilelang
    from example_gemm_autotune import get_configs, kernel
    cfgs = get_configs(4096, 4096, 4096, with_roller=True, topk=4)
    quad = dict(block_M=256, block_N=256, block_K=64, num_stages=2, thread_num=512)
    hit = [c for c in cfgs if all(c[k] == v for k, v in quad.items())]
    assert hit, cfgs
    src = tilelang.lower(kernel(4096, 4096, 4096, **hit[0]), target="hip").kernel_source
    assert "tl::gemm_quad_nt_x" in src


def test_matmul_template_recommendation():
    hs = MatmulTemplate(M=8192, N=8192, K=8192, in_dtype="float16").with_arch(ARCH).recommend_hints(3)
    c = hs[0].to_config()
    assert (c["block_M"], c["block_N"], c["threads"]) == (256, 256, 512)


def test_rasterization_panel_from_l2_model():
    """The rasterisation plan of a hint carries the panel width of the per-XCD L2 model
    (roller/rasterization.py l2_panel_width) into to_config()['panel_size']."""
    from tilelang.carver.roller.rasterization import l2_panel_width, Rasterization2DRow
    assert l2_panel_width(8192, 8192, 4096, 256, 256, 2) == 8
    assert l2_panel_width(1024, 8192, 4096, 256, 256, 2) == 4  # 4 tile rows only
    assert l2_panel_width(256, 8192, 4096, 256, 256, 2) == 1
    h = TensorCorePolicy(ARCH, 8192, 8192, 8192, trans_b=True).emit_config(1)[0]
    assert isinstance(h.rasterization_plan, Rasterization2DRow) and h.to_config()["panel_size"] == 8
    assert h.rasterization_plan.get_code() == ['T.use_swizzle(panel_size=8, order="row")']
