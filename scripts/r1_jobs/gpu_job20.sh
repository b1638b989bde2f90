#!/bin/bash
# new families: Mamba-2 chunk state, retention, DeepGEMM block-scaled fp8 (tests + reference-shape perf)
cd "$(dirname "$0")/.."
O=gpurun_out/job20.log
: > $O
export PYTHONPATH=$(pwd):$(pwd)/examples/linear_attention:$(pwd)/examples/deepseek_deepgemm
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_examples_linear.py tests/test_deepgemm.py >> $O 2>&1 || exit $?
timeout -k 10 200 python -u examples/linear_attention/example_mamba_chunk_state.py >> $O 2>&1 || exit $?
timeout -k 10 200 python -u examples/linear_attention/example_retention_fwd.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/deepseek_deepgemm/example_deepgemm_fp8_2xAcc.py >> $O 2>&1 || exit $?
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 >> $O 2>&1 || exit $?
grep -E "TFLOPS|passed|failed|metric" $O
