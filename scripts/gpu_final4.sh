#!/bin/bash
# Round-end rehearsal after the MX GEMM changes: GPU suite, MX example, smoke(), bench, kernel stats.
set -u
mkdir -p gpurun_out/final4
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/final4/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/final4/pytest_gpu.log | tail -6
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u examples/gemm_fp8/example_tilelang_gemm_mx.py > gpurun_out/final4/mx_example.log 2>&1; rc=$?; echo "mx example rc=$rc"; grep MX gpurun_out/final4/mx_example.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final4/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/final4/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/final4/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; grep metric gpurun_out/final4/bench.log | cut -c1-160
[ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/final4/prof -o bench --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/final4/prof.log 2>&1; echo "rocprof rc=$?"
