#!/bin/bash
# GPU suite, bench, MoE phased/prefetch A/B, bench kernel profile.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 700 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep metric gpurun_out/bench.log
timeout -k 10 300 python -u scripts/prof_moe.py 20 --prefetch-ab > gpurun_out/moe_ab.log 2>&1 || { tail -20 gpurun_out/moe_ab.log; exit 1; }
cat gpurun_out/moe_ab.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python -u bench.py --steps 20 --warmup 5 > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
