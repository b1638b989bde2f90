#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
hipcc --offload-arch=gfx950 -O2 -w -I tilelang/include -o /tmp/gemv_fp4_probe csrc/probes/gemv_fp4_probe.hip || exit 1
timeout -k 5 30 /tmp/gemv_fp4_probe > gpurun_out/gemv_fp4_probe.log 2>&1 || { cat gpurun_out/gemv_fp4_probe.log; exit 1; }
cat gpurun_out/gemv_fp4_probe.log
timeout -k 10 300 python -u scripts/proto/fa_pp_ab.py --variants "dsl:" "pp:-DPP=1" "pp_nopin:-DPP=1 -DNOPIN=1" "lock_nopin:-DPP=0 -DNOPIN=1" > gpurun_out/fa_pp_ab2.log 2>&1 || { tail -30 gpurun_out/fa_pp_ab2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/fa_pp_ab2.log
