"""T.Pipelined(order=, stage=, group=) schedules (transform/stage_schedule.py)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "flash_attention"))

import tilelang  # noqa: E402
import tilelang.language as T  # noqa: E402
from example_mha_fwd import ref_program  # noqa: E402
from example_mha_fwd_pipelined import flashattn_pipelined  # noqa: E402


def staged_chain(n, order, stage, group=None):
    """x_{t} = 2 * x_{t-1} + a[t] split into a stage-0 load and a stage-1 update."""

    @T.prim_func
    def main(A: T.Tensor((n, 64), "float32"), O: T.Tensor((64, ), "float32")):
        with T.Kernel(1, threads=64):
            acc = T.alloc_fragment((64, ), "float32")
            tmp = T.alloc_fragment((64, ), "float32")
            T.clear(acc)
            for k in T.Pipelined(n, num_stages=2, order=order, stage=stage, group=group):
                for i in T.Parallel(64):
                    tmp[i] = A[k, i] + 1.0
                for i in T.Parallel(64):
                    acc[i] = acc[i] * 2.0 + tmp[i]
            T.copy(acc, O)

    return main


def _chain_ref(a):
    acc = torch.zeros(a.shape[1])
    for t in range(a.shape[0]):
        acc = acc * 2 + a[t] + 1
    return acc


@pytest.mark.parametrize("n", [1, 2, 5])
def test_two_stage_chain(n):
    # the stage-1 reader is ordered before the stage-0 writer of the next iteration: legal
    k = tilelang.compile(staged_chain(n, order=[1, 0], stage=[0, 1]), out_idx=[1], target="cpu")
    a = torch.randn(n, 64)
    torch.testing.assert_close(k(a), _chain_ref(a))


def test_hazard_rejected():
    # reader after the writer that already overwrote tmp -> needs register versioning
    with pytest.raises(NotImplementedError):
        tilelang.lower(staged_chain(4, order=[0, 1], stage=[0, 1]), target="cpu")


def test_bad_group_rejected():
    with pytest.raises(ValueError):
        tilelang.lower(staged_chain(4, order=[0], stage=[0], group=[[0]]), target="cpu")


@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("lazy,sum_mfma", [(False, False), (True, False), (True, True)])
def test_fa_staged_cpu(causal, lazy, sum_mfma):
    f = flashattn_pipelined.get_tir(1, 2, 192, 64, causal, 1, 64, 32, 128, 2, "bfloat16", lazy, False,
                                    sum_mfma=sum_mfma)
    k = tilelang.compile(f, out_idx=[3], target="cpu")
    q = torch.randn(1, 192, 2, 64, dtype=torch.bfloat16)
    kk, v = torch.randn_like(q), torch.randn_like(q)
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, causal).float(), rtol=2e-2, atol=2e-2)


def test_fa_staged_hip_source():
    f = flashattn_pipelined.get_tir(1, 64, 4096, 128, False, 1, 256, 64, 512, 2)
    src = tilelang.lower(f, target="hip", pass_configs=flashattn_pipelined.pass_configs).kernel_source
    # Q in registers: QK(0) in the prologue, QK(t) + PV(t-1) in the main loop, PV(n-1) in the epilogue
    assert src.count("tl::gemm_rs") == 4
    assert "wait_vmcnt" in src


def test_fa_mfma32_hip_source():
    """32x32x16 tiles: Q (natural k order) and P (the accumulator's k order) as register A operands."""
    f = flashattn_pipelined.get_tir(1, 64, 4096, 128, False, 1, 256, 64, 512, 2, mfma="32x32")
    src = tilelang.lower(f, target="hip", pass_configs=flashattn_pipelined.pass_configs).kernel_source
    assert src.count("tl::gemm_rs_32<") == 4
    assert ", 0>((&Q_s[0])" in src and ", 1>((&acc_s_cast[0])" in src
    # one query row per lane: the row max / sum need only the lane^32 exchange
    assert "lane_allreduce<tl::MaxOp, 32>" in src


@pytest.mark.gpu
@pytest.mark.parametrize("mfma,sum_mfma", [("16x16", False), ("32x32", False), ("16x16", True), ("32x32", True)])
@pytest.mark.parametrize("causal", [False, True])
def test_fa_staged_gpu(causal, mfma, sum_mfma):
    k = flashattn_pipelined(2, 4, 1024, 128, causal, 2, 256, 64, 512, 2, mfma=mfma, sum_mfma=sum_mfma)
    q = torch.randn(2, 1024, 4, 128, device="cuda", dtype=torch.bfloat16)
    kk = torch.randn(2, 1024, 2, 128, device="cuda", dtype=torch.bfloat16)
    v = torch.randn_like(kk)
    torch.testing.assert_close(k(q, kk, v).float(), ref_program(q, kk, v, causal, 2).float(), rtol=2e-2,
                               atol=2e-2)


def alt_chain(cond_fn, n=4):
    """Two compute orders selected per wave by ``alt_cond`` (T.Pipelined(order_alt=, alt_cond=))."""

    @T.prim_func
    def main(A: T.Tensor((n, 128), "float32"), O: T.Tensor((128, ), "float32")):
        with T.Kernel(1, threads=128):
            acc = T.alloc_fragment((128, ), "float32")
            tmp = T.alloc_fragment((128, ), "float32")
            T.clear(acc)
            for k in T.Pipelined(n, num_stages=2, order=[1, 0], stage=[0, 1], order_alt=[1, 0],
                                 alt_cond=cond_fn()):
                for i in T.Parallel(128):
                    tmp[i] = A[k, i] + 1.0
                for i in T.Parallel(128):
                    acc[i] = acc[i] * 2.0 + tmp[i]
            T.copy(acc, O)

    return main


def test_alt_cond_must_be_wave_uniform():
    # wave-constant: one scalar branch per wave (readfirstlane) is exact
    src = tilelang.lower(alt_chain(lambda: T.get_thread_binding() >= 64), target="hip").kernel_source
    assert "__builtin_amdgcn_readfirstlane" in src
    # lane-varying: readfirstlane would silently give every lane lane 0's choice -> refused
    with pytest.raises(Exception, match="same for every lane"):
        tilelang.lower(alt_chain(lambda: T.get_thread_binding() % 2 == 0), target="hip")
