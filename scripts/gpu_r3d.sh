#!/bin/bash
# GEMM A/B, full GPU suite + smoke + bench, memory-bound sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u scripts/proto/gemm_rp_ab.py > gpurun_out/gemm_ab3.log 2>&1; rc=$?
grep -v Warning gpurun_out/gemm_ab3.log | tail -5
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_final.sh || exit 1
timeout -k 10 300 python -u -m tilelang.tools.precision --out gpurun_out/PRECISION.md > gpurun_out/precision.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/membound_sweep.py > gpurun_out/membound.log 2>&1; rc=$?
grep -v Warning gpurun_out/membound.log | tail -40
exit $rc
