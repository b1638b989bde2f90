#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job5.log
: > $O
TESTS=tests/test_gpu_examples_misc.py BENCH=0 PROFILE=0 bash scripts/gpu_round.sh >> $O 2>&1 || exit $?
export PYTHONPATH=$(pwd)
timeout -k 10 200 python examples/deepseek_v32/sparse_mla_fwd.py >> $O 2>&1
timeout -k 10 200 python examples/deepseek_v32/fp8_lighting_indexer.py >> $O 2>&1
timeout -k 10 200 python examples/deepseek_v32/topk_selector.py >> $O 2>&1
timeout -k 10 200 python examples/fusedmoe/example_fusedmoe_tilelang.py >> $O 2>&1
cat $O | grep -v "^tests/\|PASSED"
