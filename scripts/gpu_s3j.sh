#!/bin/bash
# session 3: full GPU suite after the small-tile DMA change, bench, low-precision numbers
set -u
mkdir -p gpurun_out/s3j
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 900 python -u -m pytest tests -v -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/s3j/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/s3j/pytest_gpu.log | tail -6
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/s3j/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/s3j/bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_lowp.py > gpurun_out/s3j/lowp.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/s3j/lowp.log
