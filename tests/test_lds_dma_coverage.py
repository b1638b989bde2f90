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
    # tl::gemm_quad_nt_x (tl/gemm_quad.h) stages both operands by buffer LDS-DMA inside the template
    return len(re.findall(r"tl::(?:glds16|buffer_lds16|gemm_quad_nt_x<)", src)), len(re.findall(r"\bstage\d+\[", src))


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


def _small_tile_kernel(big_elems):
    import tilelang.language as T

    @T.prim_func
    def main(L: T.Tensor((64, 4096), "float32"), X: T.Tensor((64, 64), "float32"), O: T.Tensor((64, 64), "float32")):
        with T.Kernel(64, threads=256) as bx:
            big = T.alloc_shared((big_elems, ), "float32")
            l_s = T.alloc_shared((64, ), "float32")
            acc = T.alloc_fragment((64, ), "float32")
            T.clear(acc)
            T.copy(X[bx, :], big[0:64])
            for k in T.Pipelined(64, num_stages=3):
                T.copy(L[bx, k * 64:(k + 1) * 64], l_s)
                for i in T.Parallel(64):
                    acc[i] += l_s[i] * big[i]
            T.copy(acc, O[bx, :])

    return main


def test_small_tile_dma_and_lds_overflow_fallback():
    """A 256-byte per-step tile (an LSE row, an MX scale tile) becomes ONE 4-byte buffer LDS-DMA per
    wave (tl::buffer_lds4) instead of a register-staged copy; when the padded stage slots would push
    the arena past 160 KiB the kernel is lowered again with register staging."""
    src = tilelang.lower(_small_tile_kernel(1024), target="hip").kernel_source
    assert "tl::buffer_lds4(" in src and not re.search(r"\bstage\d+\[", src)
    # 158 KiB of other LDS: 3 padded 1 KiB slots (4 waves x 256 B) no longer fit
    src = tilelang.lower(_small_tile_kernel(158 * 256), target="hip").kernel_source
    assert "tl::buffer_lds4(" not in src and re.search(r"\bstage\d+\[", src)


def test_moe_ext_rows_gather_is_lds_dma():
    """The 32-row extension tile of ext_M (4 KiB: fewer 16-byte chunks than lanes) is a row-gather
    LDS-DMA whose extra waves re-fetch a covered piece -- not a synchronous SIMT gather (which put
    a global round trip and a barrier into every K step: GEMM1 147 -> 213 us)."""
    from tilelang.ops.moe import expert_gemm_sk_kernel, max_padded_rows
    mr = max_padded_rows(4096, 8, 288)
    for sw in (True, False):
        kw = dict(n_src=2048, swiglu=True) if sw else {}
        src = expert_gemm_sk_kernel(mr, 2048, 4096, 8, "bfloat16", "hip", 256, 256, 64, 2, 512, ext_M=32,
                                    **kw).get_kernel_source()
        dma, staged = _counts(src)
        assert staged == 0 and "% 4)" in src, (sw, dma)
        loop = src[src.index("for (int k"):]
        loop = loop[:loop.index("tl::gemm_ss<")]
        assert "tl::sync_threads()" not in loop  # no synchronous gather before the MFMAs


def test_gemm_rs_pipe_template_arg():
    """tl.gemm_rs_pipe reaches the register-A GEMM as its PIPE template argument."""
    from example_mha_fwd_pipelined import flashattn_pipelined as fa
    f = fa.get_tir(1, 8, 512, 128, False, 1, 256, 64, 512, 2, "bfloat16", True, True, sum_mfma=True, fold_max=True)
    for pipe in (0, 4):
        cfg = dict(fa.pass_configs)
        cfg["tl.gemm_rs_pipe"] = pipe
        src = tilelang.compile(f, out_idx=[3], target="hip", pass_configs=cfg).get_kernel_source()
        args = [m for m in re.findall(r"tl::gemm_rs<([^>]*)>", src)]
        assert args and all(a.split(",")[-1].strip() == str(pipe) for a in args), (pipe, args)


def test_pack_f32_pairs():
    """tl.pack_f32: fp32 register pairs of an unrolled fragment loop become floatx2 math."""
    import tilelang.language as T

    @T.prim_func
    def main(A: T.Tensor((256, 64), "float32"), B: T.Tensor((256, 64), "float32")):
        with T.Kernel(1, threads=256):
            a = T.alloc_fragment((256, 64), "float32")
            T.copy(A, a)
            for i, j in T.Parallel(256, 64):
                a[i, j] = a[i, j] * 0.5 + 1.0
            T.copy(a, B)

    plain = tilelang.lower(main, target="hip").kernel_source
    packed = tilelang.lower(main, target="hip", pass_configs={"tl.pack_f32": True}).kernel_source
    assert "tl::floatx2" not in plain and "tl::floatx2" in packed


def _persistent_kernel(iter_local):
    import tilelang.language as T

    @T.prim_func
    def main(A: T.Tensor((8, 256, 128), "float32"), O: T.Tensor((8, 256, 128), "float32")):
        with T.Kernel(2, threads=256) as bx:
            big = T.alloc_shared((256, 128), "float32")  # 128 KiB: two of them do not fit
            out = T.alloc_shared((256, 128), "float32")
            for it in T.serial(4, annotations={"lds_iteration_local": True} if iter_local else None):
                t = bx * 4 + it
                T.copy(A[t, :, :], big)
                for i, j in T.Parallel(256, 128):
                    big[i, j] = big[i, j] * 2.0
                T.copy(big, O[t, :, :])
                for i, j in T.Parallel(256, 128):
                    out[i, j] = O[t, i, j] + 1.0
                T.copy(out, O[t, :, :])

    return main


def test_lds_iteration_local_loops():
    """Loops annotated ``lds_iteration_local`` (transform/lds_plan.py): buffers confined to
    disjoint stretches of one iteration share bytes, with a barrier where the tenants switch and
    one at the top of the body (the late tenant of iteration i precedes the early one of i + 1);
    without the annotation the loop is one statement and the two 128 KiB tiles do not fit."""
    from tilelang.transform.lds_plan import LDSPlanError
    src = tilelang.lower(_persistent_kernel(True), target="hip").kernel_source
    assert "tl_smem[131072]" in src
    body = src[src.index("for (int i = 0; i < 4;"):]
    assert body.index("tl::sync_threads()") < body.index("big")
    with pytest.raises(LDSPlanError):
        tilelang.lower(_persistent_kernel(False), target="hip")


@pytest.mark.gpu
def test_lds_iteration_local_gpu():
    """The shared-bytes persistent kernel computes the right thing on the GPU (barriers at the
    tenant switches and at the top of every iteration)."""
    import torch
    k = tilelang.compile(_persistent_kernel(True), target="hip")
    a = torch.randn(8, 256, 128, device="cuda")
    o = torch.zeros_like(a)
    k(a, o)
    torch.testing.assert_close(o, a * 2.0 + 1.0)


def test_persistent_gemm_staged_epilogue_shares_lds():
    """T.Persistent(lds_iteration_local=True): the persistent GEMM's C staging tile takes the
    operand ring's bytes (135 KiB arena instead of 263 KiB)."""
    from example_gemm_persistent import matmul_persistent
    src = _hip(matmul_persistent, 8192, 8192, 1024, trans_B=True, staged_epilogue=True)
    assert "tl_smem[135168]" in src and "gemm_quad_nt_x<" in src


@pytest.mark.gpu
def test_persistent_gemm_staged_epilogue_gpu():
    import torch
    from example_gemm_persistent import matmul_persistent
    M, N, K = 1024, 1536, 512
    k = matmul_persistent(M, N, K, trans_B=True, staged_epilogue=True, num_cus=4)
    a = torch.randn(M, K, device="cuda", dtype=torch.float16)
    b = torch.randn(N, K, device="cuda", dtype=torch.float16)
    torch.testing.assert_close(k(a, b).float(), a.float() @ b.float().T, rtol=2e-2, atol=2e-1)
