#!/bin/bash
# GEMM main-loop A/B (register-prefetch prototypes) + the new EP/TP 2-process MoE GPU tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u scripts/proto/gemm_rp_ab.py > gpurun_out/gemm_rp_ab2.log 2>&1; rc=$?
grep -v Warning gpurun_out/gemm_rp_ab2.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_moe.py tests/test_builtins.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/moe_gpu.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/moe_gpu.log | tail -20
exit $rc
