"""Performance guard: the pipelined operand copies of the headline / hot kernels must be LDS-DMA
(``glds16`` / ``buffer_lds16``), never the register-staged fallback the compiler uses when it cannot
prove a tile in bounds (that fallback adds a vmcnt(0) + VGPR round trip to every K step)."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("gemm", "flash_attention", "flash_decoding", "deepseek_mla", "blocksparse_attention", "amd"):
    sys.path.insert(0, os.path.join(ROOT, "examples", d))

import tilelang  # noqa: E402


def _counts(src):
    return len(re.findall(r"tl::(?:glds16|buffer_lds16)\(", src)), len(re.findall(r"\bstage\d+\[", src))


def _hip(jf, *a, **kw):
    f = jf.get_tir(*a, **kw)
    return tilelang.compile(f, out_idx=jf.out_idx, target="hip", pass_configs=jf.pass_configs).get_kernel_source()


@pytest.mark.parametrize("name", ["gemm", "fa", "fa_causal", "fa_persistent", "gqa_paged", "mla_paged",
                                  "sparse_gqa_paged"])
def test_examples_use_lds_dma(name):
    if name == "gemm":
        from example_gemm import matmul
        src = _hip(matmul, 4096, 4096, 4096, 256, 256, 64, 512, 2)
    elif name == "fa":
        from example_mha_fwd_pipelined import flashattn_pipelined as fa
        src = _hip(fa, 1, 64, 4096, 128, False, 1, 256, 64, 512, 2, "bfloat16", True, True)
    elif name == "fa_causal":
        from example_mha_fwd_pipelined import flashattn_pipelined as fa
        src = _hip(fa, 1, 64, 4096, 128, True, 1, 256, 64, 512, 2, "bfloat16", True, True, mfma="32x32")
    elif name == "fa_persistent":  # the tile index comes from a while loop: clamped for the prover
        from example_amd_flash_attn_fwd import fast_flashattn
        src = _hip(fast_flashattn, 1, 64, 4096, 128, True, 1)
    elif name == "gqa_paged":
        import example_gqa_decode as d
        src = _hip(d.gqa_decode_paged, 4, 32, 8, 64, 64, 32, 128)
    elif name == "mla_paged":
        import example_mla_decode_paged as m
        src = _hip(m.mla_decode_paged, 8, 128, 4096, 128, 64)
    else:
        from sparse_gqa_decode import sparse_gqa_decode_paged
        src = _hip(sparse_gqa_decode_paged, 2, 32, 8, 128, 64, 64, 64, 32, 8)
    dma, staged = _counts(src)
    assert dma > 0 and staged == 0, (name, dma, staged)


@pytest.mark.parametrize("gather", [False, True])
def test_moe_expert_gemms_use_lds_dma(gather):
    from tilelang.ops.moe import expert_gemm_sk_kernel, expert_gemm_kernel, max_padded_rows
    mr = max_padded_rows(4096, 8, 256)
    kw = dict(n_src=2048, swiglu=True) if gather else {}
    for fn in (expert_gemm_sk_kernel, expert_gemm_kernel):
        src = fn(mr, 2048, 4096, 8, "bfloat16", "hip", 256, 256, 64, 2, 512, **kw).get_kernel_source()
        dma, staged = _counts(src)
        assert dma > 0 and staged == 0, (fn.__name__, gather, dma, staged)
