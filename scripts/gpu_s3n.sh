#!/bin/bash
set -u
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3n
timeout -k 10 600 python -u scripts/moe_gemm_probe.py > gpurun_out/s3n/probe3.log 2>&1; grep -v amdgpu gpurun_out/s3n/probe3.log | tail -12
timeout -k 10 300 python -u -m pytest tests/test_moe.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3n/t.log 2>&1; grep -E "FAILED|passed|failed" gpurun_out/s3n/t.log | tail -3
for i in 1 2; do timeout -k 10 300 python bench.py 2>&1 | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['gemm_tflops'], d['attn_tflops'], d['moe_tflops_per_gpu'])"; done
