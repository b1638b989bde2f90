#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_mx_gemm.py tests/test_moe.py tests/test_index_bitwidth.py tests/test_builtins.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r2b bash scripts/gpu_prof_moe.sh
