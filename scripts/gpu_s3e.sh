#!/bin/bash
# session 3: varlen bwd after the head clamp / interior fast path / pipelined LSE; FA bwd tile sweep
set -u
mkdir -p gpurun_out/s3e
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_backward_kernels.py -v -m gpu -k varlen --timeout 120 --timeout-method thread > gpurun_out/s3e/varlen_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s3e/varlen_tests.log | tail -5
[ $rc -le 1 ] || exit $rc
(cd examples/flash_attention && timeout -k 10 300 python -u example_mha_bwd_varlen.py) > gpurun_out/s3e/varlen.log 2>&1 || { tail -20 gpurun_out/s3e/varlen.log; exit 1; }
grep -v amdgpu gpurun_out/s3e/varlen.log | tail -2
timeout -k 10 600 python -u scripts/sweep_fa_bwd.py > gpurun_out/s3e/sweep_bwd.log 2>&1 || { tail -20 gpurun_out/s3e/sweep_bwd.log; exit 1; }
grep -v amdgpu gpurun_out/s3e/sweep_bwd.log
timeout -k 10 600 python -u scripts/sweep_fa_bwd.py --causal > gpurun_out/s3e/sweep_bwd_causal.log 2>&1 || { tail -20 gpurun_out/s3e/sweep_bwd_causal.log; exit 1; }
grep best gpurun_out/s3e/sweep_bwd_causal.log
