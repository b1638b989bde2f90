#!/bin/bash
# fp8 MLA tests, ds_read_tr8 probe, bench kernel profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_gpu_examples.py -m gpu -k "kv_fp8 or group_per_split" -v --timeout 120 --timeout-method thread > gpurun_out/mla8_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|passed|failed" gpurun_out/mla8_tests.log | tail -8
hipcc --offload-arch=gfx950 -O2 -w -o /tmp/tr8_probe csrc/probes/ds_read_tr8.hip && timeout -k 5 30 /tmp/tr8_probe > gpurun_out/tr8_probe.log 2>&1 || exit 1
head -20 gpurun_out/tr8_probe.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench3 -o prof -- python -u bench.py --steps 5 --warmup 3 > gpurun_out/bench_prof.log 2>&1 || { tail -20 gpurun_out/bench_prof.log; exit 1; }
grep metric gpurun_out/bench_prof.log | cut -c1-300
find gpurun_out/prof_bench3 -name "*kernel_stats.csv" | head -3
