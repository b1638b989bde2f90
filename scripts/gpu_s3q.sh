#!/bin/bash
set -u
mkdir -p gpurun_out/s3q
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_stage_schedule.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3q/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/s3q/t.log | tail -3
[ $rc -eq 0 ] || exit 1
for i in 1 2 3; do timeout -k 10 300 python bench.py 2>&1 | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['gemm_tflops'], d['attn_tflops'], d['moe_tflops_per_gpu'])"; done
