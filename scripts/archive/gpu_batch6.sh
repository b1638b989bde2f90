set -o pipefail
mkdir -p gpurun_out/benchmarks
timeout -k 10 300 python -u -m pytest tests/test_gpu_examples_misc.py -m gpu -x -v --timeout 120 --timeout-method thread -k mamba > gpurun_out/mamba_lean_tests.log 2>&1 && \
timeout -k 10 600 python -u benchmarks/mamba2/benchmark_mamba_chunk_scan.py --out gpurun_out/benchmarks --rows 1024,4096,16384 > gpurun_out/mamba_lean.log 2>&1
