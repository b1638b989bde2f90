#!/bin/bash
# fp4 cvt probe, FA ping-pong prototype A/B, MoE tail-balanced GPU test.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
hipcc --offload-arch=gfx950 -O2 -w -o /tmp/cvt_fp4_probe csrc/probes/cvt_fp4_probe.hip || exit 1
timeout -k 5 30 /tmp/cvt_fp4_probe > gpurun_out/cvt_fp4_probe.log 2>&1 || { cat gpurun_out/cvt_fp4_probe.log; exit 1; }
grep -E "MISMATCH|mismatches" gpurun_out/cvt_fp4_probe.log | head -12
timeout -k 10 300 python -u scripts/proto/fa_pp_ab.py > gpurun_out/fa_pp_ab.log 2>&1 || { tail -30 gpurun_out/fa_pp_ab.log; exit 1; }
cat gpurun_out/fa_pp_ab.log | grep -v amdgpu.ids
timeout -k 10 200 python -u -m pytest tests/test_moe.py -v -m gpu -k tail_balanced --timeout 120 --timeout-method thread > gpurun_out/moe_t.log 2>&1; tail -2 gpurun_out/moe_t.log
