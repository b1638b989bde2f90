#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job16.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -x --timeout 120 --timeout-method thread -k "sparse_mla_bwd" >> $O 2>&1 || exit $?
timeout -k 10 400 python -u examples/deepseek_v32/sparse_mla_bwd.py >> $O 2>&1
tail -8 $O
