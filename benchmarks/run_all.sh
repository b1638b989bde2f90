#!/bin/bash
# Reproduce every reference benchmark table on the GPU box (one process per table, each step
# bounded by its own time limit; stops at the first failure).
set -o pipefail
OUT=${1:-gpurun_out/benchmarks}
mkdir -p $OUT
timeout -k 10 900 python -u benchmarks/matmul/benchmark_matmul.py --out $OUT > $OUT/matmul.log 2>&1 && \
timeout -k 10 900 python -u benchmarks/matmul_fp8/benchmark_matmul.py --out $OUT > $OUT/matmul_fp8.log 2>&1 && \
timeout -k 10 900 python -u benchmarks/mamba2/benchmark_mamba_chunk_scan.py --out $OUT > $OUT/mamba2.log 2>&1 && \
timeout -k 10 600 python -u benchmarks/blocksparse_attention/benchmark_block_sparse_fmha.py --out $OUT > $OUT/bsa.log 2>&1 && \
timeout -k 10 900 python -u benchmarks/matmul/benchmark_matmul_intrinsic.py --out $OUT > $OUT/matmul_intrinsic.log 2>&1 && \
timeout -k 10 900 python -u benchmarks/matmul/benchmark_matmul_sp.py --out $OUT > $OUT/matmul_sp.log 2>&1
