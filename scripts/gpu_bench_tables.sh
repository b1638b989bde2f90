set -o pipefail
mkdir -p gpurun_out/benchmarks
timeout -k 10 600 python -u benchmarks/mamba2/benchmark_mamba_chunk_scan.py --out gpurun_out/benchmarks --rows 1024,4096,16384 > gpurun_out/benchmarks/mamba2_b.log 2>&1 && \
timeout -k 10 500 python -u benchmarks/matmul_fp8/benchmark_matmul.py --out gpurun_out/benchmarks --rows 256,512,1024,4096 > gpurun_out/benchmarks/matmul_fp8_b.log 2>&1
