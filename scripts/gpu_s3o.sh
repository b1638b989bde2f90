#!/bin/bash
set -u
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3o
timeout -k 10 300 python -u -m pytest tests -v -m gpu -k "mxfp4 or gemv or cast" --timeout 120 --timeout-method thread > gpurun_out/s3o/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/s3o/t.log | tail -4
[ $rc -eq 0 ] || { tail -30 gpurun_out/s3o/t.log; exit 1; }
timeout -k 10 500 python -u scripts/bench_lowp.py > gpurun_out/s3o/lowp.log 2>&1; grep -E "GEMV|decode" gpurun_out/s3o/lowp.log
(cd examples/cast && timeout -k 10 200 python example_per_token_cast_to_fp8.py 2>&1 | grep -v amdgpu | tail -2)
