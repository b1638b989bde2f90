#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 200 python -u scripts/debug/dbg_mla_fp8_s.py > gpurun_out/dbg_mla_s.log 2>&1; rc=$?
grep -v Warn gpurun_out/dbg_mla_s.log | tail -20
exit $rc
