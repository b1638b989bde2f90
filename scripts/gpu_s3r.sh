#!/bin/bash
set -u
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3r
timeout -k 10 600 python -u scripts/sweep_fp8.py > gpurun_out/s3r/sweep_fp8.log 2>&1; grep -v amdgpu gpurun_out/s3r/sweep_fp8.log
