#!/bin/bash
# MoE layer on one MI355X: local / ep / tp (1x1 mesh) + MoE tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_moe.py -q -x > gpurun_out/moe_tests.log 2>&1 || exit 1
for p in local ep tp; do
  timeout -k 10 400 python benchmarks/bench_moe.py --parallel $p --steps 10 --warmup 3 >> gpurun_out/moe_bench.log 2>&1 || exit 2
done
