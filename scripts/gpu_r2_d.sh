#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2d
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_moe.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
TAG=r2d bash scripts/gpu_prof_moe.sh || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log; exit $rc
