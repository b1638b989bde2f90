#!/bin/bash
# MX GEMM inner-loop A/B (TL_MX_PD) + PMC passes of the MX fp8 and per-tensor fp8 kernels
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
mkdir -p gpurun_out/s3y
timeout -k 10 400 python -u scripts/mx_pd_ab.py > gpurun_out/s3y/mx_pd_ab.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/s3y/mx_pd_ab.log | tail -12
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_mx.sh > gpurun_out/s3y/pmc.log 2>&1; rc=$?; tail -50 gpurun_out/s3y/pmc.log; exit $rc
