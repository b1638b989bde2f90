#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD:$PYTHONPATH
: > gpurun_out/sk.log
timeout -k 10 300 python -u -m pytest tests/test_moe.py -m gpu -x -v --timeout 120 --timeout-method thread >> gpurun_out/sk.log 2>&1 || { echo FAILED tests; tail -30 gpurun_out/sk.log; exit 1; }
timeout -k 10 300 python scripts/prof_moe.py 20 --sk-ab >> gpurun_out/sk.log 2>&1 || { echo FAILED prof; tail -30 gpurun_out/sk.log; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/sk.log 2>&1 || { echo FAILED bench; tail -30 gpurun_out/sk.log; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_sk -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 >> $GRAFT_REPO_ROOT/gpurun_out/sk.log 2>&1 || { echo FAILED rocprof; tail -30 $GRAFT_REPO_ROOT/gpurun_out/sk.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep -v "PASSED\|^$\|amdgpu.ids" gpurun_out/sk.log | tail -30
find gpurun_out/prof_sk -name "*kernel_stats.csv" | head -3
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_mhainf -o run -- python3 $GRAFT_REPO_ROOT/examples/flash_decoding/example_mha_inference.py >> $GRAFT_REPO_ROOT/gpurun_out/sk.log 2>&1 || { echo FAILED rocprof2; exit 1; }
cd $GRAFT_REPO_ROOT
find gpurun_out/prof_mhainf -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150 | head -8
