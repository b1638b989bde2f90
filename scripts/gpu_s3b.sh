#!/bin/bash
# session 3: persistent FA A/B + FA / persistent GPU tests
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_stage_schedule.py tests/test_examples_amd.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3b_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s3b_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/fa_persistent_ab.py > gpurun_out/fa_persistent_ab.log 2>&1 || { grep -v amdgpu.ids gpurun_out/fa_persistent_ab.log | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_persistent_ab.log
