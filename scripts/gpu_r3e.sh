#!/bin/bash
# Full GPU suite (no -x: collect every failure), precision table, fp8 paths, emitter GEMM, memory-bound sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m tilelang.tools.precision --out gpurun_out/PRECISION.md > gpurun_out/precision.log 2>&1 || { tail -20 gpurun_out/precision.log; exit 1; }
timeout -k 10 400 python -u scripts/bench_fp8_paths.py > gpurun_out/fp8_paths.log 2>&1 || { tail -20 gpurun_out/fp8_paths.log; exit 1; }
grep -v Warn gpurun_out/fp8_paths.log | tail -25
for a in "--micro 32" "--micro 16" "--micro 32 --preshuffle" "--dtype int8" "--dtype float8_e4m3fn"; do
  timeout -k 10 120 python -u examples/gemm/example_gemm_intrinsics.py $a >> gpurun_out/emitter.log 2>&1 || { tail -20 gpurun_out/emitter.log; exit 1; }
done
grep TFLOPS gpurun_out/emitter.log
timeout -k 10 400 python -u scripts/membound_sweep.py > gpurun_out/membound.log 2>&1; rc=$?
grep -v Warning gpurun_out/membound.log | tail -40
exit $rc
