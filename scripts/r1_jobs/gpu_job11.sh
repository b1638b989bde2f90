#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job11.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -k "gqa_attention_bwd or gdn" >> $O 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gpu_sweep.py fa_fwd '{"block_M":256,"block_N":64,"threads":512}' '{"block_M":256,"block_N":64,"threads":512,"lazy_rescale":true}' '{"block_M":128,"block_N":64,"threads":256,"lazy_rescale":true}' '{"block_M":256,"block_N":64,"threads":512,"lazy_rescale":true,"causal":true}' '{"block_M":256,"block_N":64,"threads":512,"causal":true}' >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/gdn/example_gdn.py >> $O 2>&1
grep -v "^tests/\|PASSED" $O | tail -22
