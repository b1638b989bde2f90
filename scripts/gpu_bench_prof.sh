#!/bin/bash
# New GEMM/runtime GPU tests, bench, and a kernel-stats profile of the bench (each step time-limited).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "test_gemm or runtime_facade" > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
grep metric gpurun_out/bench.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_bench -name "*kernel_stats.csv" | head -3
