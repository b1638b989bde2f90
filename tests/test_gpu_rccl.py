"""RCCL at world size 1 on one MI355X (SURVEY §7.5 test tier "RCCL world size 1 (loopback)").

Every multi-GPU path that a single GPU can execute, under ``torchrun --nproc-per-node 1`` with
the ``nccl`` backend (= RCCL on ROCm): ProcessMesh + its row/column groups, the host collectives,
a T.comm kernel on the mesh workspace, the expert-parallel MoE (device exchange and the RCCL
all_to_all_v fallback) and the tensor-parallel MoE (tests/rccl_world1.py), plus ``bench.py
--dist`` forced through the mesh path with its result checks."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_rccl_world1_torchrun():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "tests", "rccl_world1.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-5000:])
    assert "RCCL_WORLD1_OK" in r.stdout


def test_bench_dist_world1():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--dist", "--steps", "2", "--warmup", "1", "--prewarm-ms",
           "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-5000:])
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["n_gpus"] == 1
    assert out["config"]["parallelism"] == "dp1+ep1"
    assert out["ep_exchange"].startswith("device") and out["ep_fallback_reason"] is None
    assert out["tp_moe"] is not None and "error" not in out["tp_moe"], out["tp_moe"]
