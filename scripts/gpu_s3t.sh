#!/bin/bash
set -u
mkdir -p gpurun_out/s3t
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 500 python -u scripts/fa_mfma_ab.py --variants m16_sum m16_sum_s3 m16_sum_n128 m16_sum_n32 m32_n64_s2 > gpurun_out/s3t/fa_ab.log 2>&1; grep -v amdgpu gpurun_out/s3t/fa_ab.log | tail -7
