#!/bin/bash
# Round-3 first GPU session: GEMM main-loop prototype A/B, then the round-end rehearsal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u scripts/proto/gemm_rp_ab.py > gpurun_out/gemm_rp_ab.log 2>&1; rc=$?
cat gpurun_out/gemm_rp_ab.log | grep -v Warning | tail -20
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_final.sh
