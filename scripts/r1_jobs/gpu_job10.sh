#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job10.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_examples_misc.py -v -m gpu -x --timeout 120 --timeout-method thread \
  -k "nsa or block_sparse or gdn" >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/deepseek_nsa/example_nsa_fwd.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/blocksparse_attention/example_block_sparse_attn.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/gdn/example_gdn.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/deepseek_v32/sparse_mla_fwd.py --S 4096 --SKV 8192 >> $O 2>&1
grep -v "^tests/\|PASSED" $O | tail -30
