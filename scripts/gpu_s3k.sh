#!/bin/bash
set -u
mkdir -p gpurun_out/s3k
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3k/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/s3k/pytest_gpu.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u scripts/bench_lowp.py > gpurun_out/s3k/lowp.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/s3k/lowp.log
timeout -k 10 600 python -u scripts/sweep_mx.py > gpurun_out/s3k/sweep_mx.log 2>&1; grep -v amdgpu gpurun_out/s3k/sweep_mx.log
