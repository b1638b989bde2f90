#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 400 python -u scripts/fa_mfma_ab.py --variants m16_n64_s2 m16_sum m32_n64_s2 m32_sum > gpurun_out/fa_sum_ab.log 2>&1 || { grep -v amdgpu.ids gpurun_out/fa_sum_ab.log | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_sum_ab.log
timeout -k 10 300 python -u scripts/fa_mfma_ab.py --causal --variants m16_n64_s2 m16_sum m32_n64_s2 m32_sum > gpurun_out/fa_sum_ab_causal.log 2>&1 || { tail -30 gpurun_out/fa_sum_ab_causal.log; exit 1; }
grep TF gpurun_out/fa_sum_ab_causal.log
