#!/bin/bash
# fp8 MLA debug, precision test, memory-bound sweep with the read-only flush.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u scripts/debug/dbg_mla_fp8.py > gpurun_out/dbg_mla_fp8.log 2>&1; rc=$?
grep -v Warn gpurun_out/dbg_mla_fp8.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_tooling.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/prec_test.log 2>&1; rc=$?
tail -3 gpurun_out/prec_test.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m tilelang.tools.precision --out gpurun_out/PRECISION.md > gpurun_out/precision.log 2>&1 || exit 1
timeout -k 10 400 python -u scripts/membound_sweep.py > gpurun_out/membound.log 2>&1; rc=$?
grep -v Warning gpurun_out/membound.log | tail -40
exit $rc
