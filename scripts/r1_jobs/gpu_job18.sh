#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job18.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -x --timeout 120 --timeout-method thread -k "varlen" >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/attention_sink/example_gqa_sink_bwd.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/flash_attention/example_mha_fwd_varlen.py >> $O 2>&1
grep -v "^tests/\|PASSED" $O | tail -8
