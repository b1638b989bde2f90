#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job7.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -k "deepseek or persistent" >> $O 2>&1 || exit $?
timeout -k 10 300 python examples/deepseek_v32/inference/generate.py --max-new-tokens 16 >> $O 2>&1 || exit $?
timeout -k 10 200 python examples/gemm/example_gemm_persistent.py >> $O 2>&1 || exit $?
timeout -k 10 200 python examples/blocksparse_gemm/example_blocksparse_gemm.py --m 4096 --n 4096 --k 4096 >> $O 2>&1
grep -v "^tests/\|PASSED" $O
