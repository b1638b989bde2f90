#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job8.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -k "gather or deepseek" >> $O 2>&1 || exit $?
timeout -k 10 400 python -u scripts/gpu_sweep_smla.py >> $O 2>&1
grep -v "^tests/\|PASSED" $O | tail -30
