#!/bin/bash
# FA forward variant A/B in one process (round-robin, pre-warmed): scripts/fa_variants.py
set -u
OUT=${1:-gpurun_out/fa_ab}
V=${2:-}
mkdir -p $OUT
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 500 python -u scripts/fa_variants.py "$V" > $OUT/fa_ab.log 2>&1; echo "fa rc=$?"; grep -v amdgpu.ids $OUT/fa_ab.log | tail -20
