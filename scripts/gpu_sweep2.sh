#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
: > gpurun_out/sweep2.log
timeout -k 10 300 python -u -m pytest tests/test_moe.py tests/test_gemm_phased.py -m gpu -x -v --timeout 120 --timeout-method thread >> gpurun_out/sweep2.log 2>&1 || { echo FAILED tests; tail -30 gpurun_out/sweep2.log; exit 1; }
timeout -k 10 300 python scripts/prof_moe.py 20 --tail-sweep >> gpurun_out/sweep2.log 2>&1 || { echo FAILED moe; tail -30 gpurun_out/sweep2.log; exit 1; }
timeout -k 10 300 python examples/flash_decoding/example_mha_inference.py --sweep >> gpurun_out/sweep2.log 2>&1 || { echo FAILED mhainf; tail -30 gpurun_out/sweep2.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/sweep2.log 2>&1 || { echo FAILED bench; tail -30 gpurun_out/sweep2.log; exit 1; }
grep -v "amdgpu.ids\|PASSED" gpurun_out/sweep2.log | tail -30
