"""bench.py contract on the CPU target: --gpus N spawns N ranks (gloo) and reports n_gpus=N."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--steps", "2",
                        "--warmup", "1", *args], cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("n", [1, 2])
def test_bench_spawns_ranks(n):
    out = _run("--gpus", str(n))
    assert out["n_gpus"] == n
    assert out["steps"] == 2 and out["warmup"] == 1
    for k in ("metric", "value", "unit", "ms_per_step", "higher_is_better", "scaling", "vs_baseline", "dtype",
              "data", "config", "moe_tflops_per_gpu"):
        assert k in out
    assert out["config"]["parallelism"] == ("dp1" if n == 1 else f"dp{n}+ep{n}")
    assert "MoE" in out["config"]["model"]
