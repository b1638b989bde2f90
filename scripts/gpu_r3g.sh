#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python -u scripts/debug/probe_fp8_cvt.py > gpurun_out/probe_fp8_cvt.log 2>&1; rc=$?
grep -v Warn gpurun_out/probe_fp8_cvt.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/membound_sweep.py > gpurun_out/membound.log 2>&1; rc=$?
grep -v Warning gpurun_out/membound.log | tail -45
exit $rc
