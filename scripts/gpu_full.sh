#!/bin/bash
# Full GPU validation + bench + MoE tail sweep (each step time-limited; stop at the first failure).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python scripts/prof_moe.py 20 --tail-sweep > gpurun_out/tail.log 2>&1 || { echo FAILED moe; tail -20 gpurun_out/tail.log; exit 1; }
grep -v amdgpu gpurun_out/tail.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
