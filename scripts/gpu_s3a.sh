#!/bin/bash
# session 3: FA 16x16 vs 32x32 MFMA A/B (non-causal and causal)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 400 python -u scripts/fa_mfma_ab.py > gpurun_out/fa_mfma_ab.log 2>&1 || { grep -v amdgpu.ids gpurun_out/fa_mfma_ab.log | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_mfma_ab.log
timeout -k 10 300 python -u scripts/fa_mfma_ab.py --causal --variants m16_n64_s2 m32_n64_s2 > gpurun_out/fa_mfma_ab_causal.log 2>&1 || { tail -30 gpurun_out/fa_mfma_ab_causal.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_mfma_ab_causal.log
