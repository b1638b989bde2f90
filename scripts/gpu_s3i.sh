#!/bin/bash
set -u
mkdir -p gpurun_out/s3i
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_backward_kernels.py -v -m gpu -k nsa --timeout 120 --timeout-method thread > gpurun_out/s3i/t.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/s3i/t.log | tail -2
[ $rc -eq 0 ] || { tail -30 gpurun_out/s3i/t.log; exit 1; }
cd examples/deepseek_nsa
for cfg in "dict(block_T=32, threads=64)" "dict(block_T=64, threads=256)" "dict(block_T=32, threads=128)" "dict(block_T=64, threads=128)"; do
  timeout -k 10 200 python -u -c "import example_nsa_bwd as E; E.DQ_CFG=$cfg; E.main()" 2>&1 | grep TFLOPS | sed "s/^/$cfg /"
done
