#!/bin/bash
set -u
mkdir -p gpurun_out/s3v
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -k sink --timeout 120 --timeout-method thread > gpurun_out/s3v/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/s3v/t.log | tail -3
[ $rc -eq 0 ] || { tail -30 gpurun_out/s3v/t.log; exit 1; }
timeout -k 10 400 python -u scripts/sink_ab.py > gpurun_out/s3v/sink_ab.log 2>&1; grep -v amdgpu gpurun_out/s3v/sink_ab.log
