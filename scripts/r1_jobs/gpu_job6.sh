#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job6.log
: > $O
export PYTHONPATH=$(pwd)
TESTS="tests/test_gpu_examples_misc.py -k deepseek" BENCH=0 PROFILE=0 bash scripts/gpu_round.sh >> $O 2>&1 || exit $?
timeout -k 10 200 python examples/deepseek_v32/sparse_mla_fwd.py >> $O 2>&1 || exit $?
timeout -k 10 200 python examples/deepseek_v32/fp8_lighting_indexer.py >> $O 2>&1 || exit $?
timeout -k 10 200 python examples/deepseek_v32/topk_selector.py >> $O 2>&1 || exit $?
timeout -k 10 300 python examples/deepseek_v32/inference/generate.py --max-new-tokens 16 >> $O 2>&1
cat $O | grep -v "^tests/\|PASSED"
