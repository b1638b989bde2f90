#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job2.log
: > $O
timeout -k 10 150 python scripts/gpu_sweep.py sink '{}' '{"causal":false}' >> $O 2>&1 || exit $?
TESTS=tests/test_gpu_examples_misc.py BENCH=0 PROFILE=0 bash scripts/gpu_round.sh >> $O 2>&1 || exit $?
timeout -k 10 150 python scripts/gpu_bench_examples.py mamba fa_bwd >> $O 2>&1
cat $O
