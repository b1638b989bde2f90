#!/bin/bash
set -u
mkdir -p gpurun_out/s3q
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 300 python -u -m pytest tests/test_stage_schedule.py tests/test_gpu_kernels.py -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/s3q/t.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/s3q/t.log | tail -3
[ $rc -le 1 ] || exit 1
timeout -k 10 400 python -u scripts/fa_mfma_ab.py --variants m16_n64_s2 m16_sum m32_n64_s2 > gpurun_out/s3q/fa_ab.log 2>&1; grep TF gpurun_out/s3q/fa_ab.log
for i in 1 2 3; do timeout -k 10 300 python bench.py 2>&1 | grep metric | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['gemm_tflops'], d['attn_tflops'], d['moe_tflops_per_gpu'])"; done
