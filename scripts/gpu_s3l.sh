#!/bin/bash
set -u
mkdir -p gpurun_out/s3l
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 400 python -u -m pytest tests -v -m gpu -k "moe or deepseek" --timeout 120 --timeout-method thread > gpurun_out/s3l/t.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/s3l/t.log | tail -5
[ $rc -eq 0 ] || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py 2>&1 | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['gemm_tflops'], d['attn_tflops'], d['moe_tflops_per_gpu'])"; done
