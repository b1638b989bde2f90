"""Autotuner: set_autotune_inputs capture and process isolation with a hard timeout (CPU target)."""
import time

import pytest
import torch

import tilelang
import tilelang.language as T
from tilelang.autotuner import set_autotune_inputs, get_autotune_inputs, AutoTuner


def _scale_factory(N, block=64, slow=0):
    if slow:
        time.sleep(slow)  # stands in for a config whose launch never returns

    @T.prim_func
    def main(A: T.Tensor((N, ), "float32"), B: T.Tensor((N, ), "float32")):
        with T.Kernel(T.ceildiv(N, block), threads=block) as bx:
            for i in T.Parallel(block):
                if bx * block + i < N:
                    B[bx * block + i] = A[bx * block + i] * 2.0

    return tilelang.compile(main, out_idx=[1], target="cpu")


def test_capture_stack_nests():
    a, b = torch.ones(3), torch.zeros(3)
    assert get_autotune_inputs() is None
    with set_autotune_inputs(a):
        with set_autotune_inputs([b]):
            assert get_autotune_inputs()[0] is b
        assert get_autotune_inputs()[0] is a
    assert get_autotune_inputs() is None


def test_captured_inputs_are_used(monkeypatch):
    monkeypatch.setenv("TILELANG_AUTO_TUNING_DISABLE_CACHE", "1")
    seen = []

    def check(out, a):
        seen.append(a)
        torch.testing.assert_close(out, a * 2)

    x = torch.arange(256, dtype=torch.float32)
    tuner = AutoTuner(_scale_factory, [{"block": 64}, {"block": 128}]).set_profile_args(
        warmup=1, rep=2, manual_check_prog=check)
    with set_autotune_inputs(x):
        res = tuner.run(256)
    assert res.config in ({"block": 64}, {"block": 128})
    assert len(seen) == 2 and all(s is x for s in seen)


@pytest.mark.timeout(300)
def test_isolated_config_is_killed_at_timeout(monkeypatch):
    """A config that hangs in its worker process is killed at the timeout; the others win."""
    monkeypatch.setenv("TILELANG_AUTO_TUNING_DISABLE_CACHE", "1")
    cfgs = [{"block": 64, "slow": 0}, {"block": 128, "slow": 0}, {"block": 32, "slow": 600}]
    tuner = AutoTuner(_scale_factory, cfgs).set_profile_args(
        warmup=1, rep=2, timeout=20, isolate=True, ref_prog=lambda a: a * 2)
    # the parent compiles every config first: keep the slow one fast here, slow in the worker
    orig = tuner._compile
    tuner._compile = lambda args, kwargs, cfg: orig(args, kwargs, dict(cfg, slow=0))
    t0 = time.time()
    res = tuner.run(256)
    assert time.time() - t0 < 200
    assert res.config["slow"] == 0
    errs = [r for r in res.all_results if "error" in r]
    assert len(errs) == 1 and errs[0]["config"]["slow"] == 600 and "killed" in errs[0]["error"]


@pytest.mark.timeout(300)
def test_process_compile_backend_fills_kernel_cache(monkeypatch, tmp_path):
    """compile_backend="process": worker processes lower + compile every config into the disk kernel
    cache; the parent's compiles are then cache hits, an invalid config's error still surfaces."""
    from tilelang.cache import kernel_cache
    monkeypatch.setenv("TILELANG_AUTO_TUNING_DISABLE_CACHE", "1")
    monkeypatch.setenv("TILELANG_CACHE_DIR", str(tmp_path))
    from tilelang.env import env
    monkeypatch.setattr(env, "TILELANG_CACHE_DIR", str(tmp_path), raising=False)
    cfgs = [{"block": 64}, {"block": 128}, {"block": 96}, {"block": 0}]  # block 0: invalid
    tuner = AutoTuner(_scale_factory, cfgs).set_profile_args(warmup=1, rep=2, ref_prog=lambda a: a * 2)
    tuner.set_compile_args(backend="process")
    errs = tuner._prefetch_compile((256, ), {})
    assert set(errs) == {3}
    assert kernel_cache.entries() == 3
    res = tuner.run(256)
    assert res.config in cfgs[:3]
    assert any(r.get("error") for r in res.all_results if r["config"] == {"block": 0})
