#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job15.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread >> $O 2>&1
rc=$?; echo "pytest rc=$rc" >> $O
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u examples/deepseek_mla/example_mla_decode.py >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/deepseek_mla/example_mla_decode.py --batch 64 --kv_ctx 8192 --num_split 2 >> $O 2>&1 || exit $?
timeout -k 10 300 python -u examples/deepseek_mla/example_mla_decode_paged.py >> $O 2>&1
tail -15 $O
