#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job19.log
: > $O
export PYTHONPATH=$(pwd)
timeout -k 10 300 python -u scripts/gpu_sweep.py fa_fwd_lse '{}' '{"block_M":128}' >> $O 2>&1 || exit $?
timeout -k 10 300 python -u scripts/gpu_sweep.py varlen '{}' >> $O 2>&1
cat $O | grep cfg
