#!/bin/bash
set -u
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3n
timeout -k 10 600 python -u scripts/moe_gemm_probe.py > gpurun_out/s3n/probe4.log 2>&1; grep -v amdgpu gpurun_out/s3n/probe4.log | tail -12
