#!/bin/bash
set -u
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3n
timeout -k 10 300 python -u -m pytest tests/test_moe.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3n/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/s3n/t.log | tail -6
[ $rc -eq 0 ] || { tail -30 gpurun_out/s3n/t.log; exit 1; }
timeout -k 10 600 python -u scripts/moe_gemm_probe.py > gpurun_out/s3n/probe2.log 2>&1; grep -v amdgpu gpurun_out/s3n/probe2.log | tail -12
