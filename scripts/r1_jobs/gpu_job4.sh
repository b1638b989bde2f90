#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out/job4.log
: > $O
TESTS=tests/test_gpu_examples_misc.py BENCH=0 PROFILE=0 bash scripts/gpu_round.sh >> $O 2>&1 || exit $?
timeout -k 10 200 python scripts/gpu_bench_examples.py fa_bwd mamba sink >> $O 2>&1
timeout -k 10 200 python examples/fusedmoe/example_fusedmoe_tilelang.py >> $O 2>&1
cat $O
