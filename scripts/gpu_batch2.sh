set -o pipefail
mkdir -p gpurun_out/benchmarks
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_b2.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/moe_gemm_probe.py '({}, dict(ext_M=32), {}, dict(ext_M=32))' > gpurun_out/moe_ext_probe2.log 2>&1 && \
bash scripts/gpu_bench_tables.sh
