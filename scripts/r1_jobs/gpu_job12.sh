#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job12.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py tests/test_gpu_examples.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -k "gdn or flash or attention" >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/gdn/example_gdn.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u bench.py >> $O 2>&1
grep -v "^tests/\|PASSED" $O | tail -22
