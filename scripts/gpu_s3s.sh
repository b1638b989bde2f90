#!/bin/bash
set -u
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3s
timeout -k 10 600 python -u scripts/sweep_gemv_fp4.py > gpurun_out/s3s/sweep.log 2>&1; grep -v amdgpu gpurun_out/s3s/sweep.log
