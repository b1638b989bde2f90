#!/bin/bash
# DSL register-prefetched GEMM vs prototype vs hipBLASLt, then the full GPU suite + smoke + bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 400 python -u scripts/proto/gemm_rp_ab.py > gpurun_out/gemm_dsl_prefetch_ab.log 2>&1; rc=$?
grep -v Warning gpurun_out/gemm_dsl_prefetch_ab.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_final.sh
