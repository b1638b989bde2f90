#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r2c
mkdir -p $OUT
timeout -k 10 400 python -u scripts/sweep_fa.py > $OUT/fa_sweep.log 2>&1; rc=$?; cat $OUT/fa_sweep.log; [ $rc -eq 0 ] || exit $rc
TAG=r2c bash scripts/gpu_prof_moe.sh
