#!/bin/bash
# MX GEMM: GPU tests (row-major and pre-shuffled scales) + one-process bench
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3z
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_mx_gemm.py > gpurun_out/s3z/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/s3z/pytest.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/mx_bench.py > gpurun_out/s3z/mx_bench.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/s3z/mx_bench.log | tail -8; exit $rc
