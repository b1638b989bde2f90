#!/bin/bash
# session 3: NSA bwd (token lists + gathers), FA bwd with swept tiles and the two-stream overlap
set -u
mkdir -p gpurun_out/s3f
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_backward_kernels.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3f/bwd_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/s3f/bwd_tests.log | tail -9
[ $rc -le 1 ] || exit $rc
cd examples/deepseek_nsa
timeout -k 10 300 python -u example_nsa_bwd.py > ../../gpurun_out/s3f/nsa.log 2>&1 || { tail -20 ../../gpurun_out/s3f/nsa.log; exit 1; }
grep TFLOPS ../../gpurun_out/s3f/nsa.log
cd ../flash_attention
for c in "" "--causal"; do
  timeout -k 10 300 python -u -c "import sys, example_mha_bwd as E; E.BWD_OVERLAP=False; E.main(causal='$c'!='')" 2>&1 | grep TFLOPS | sed 's/^/no-overlap /'
  timeout -k 10 300 python -u example_mha_bwd.py $c 2>&1 | grep TFLOPS | sed 's/^/overlap /'
done
