set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c1.log 2>&1 && \
timeout -k 10 400 python -u scripts/fa_variants.py '[{"sum_mfma": true, "fold_max": true, "young_prio": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true, "xcd_heads": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true, "xcd_heads": true}]' > gpurun_out/fa_xcd.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_moe.py -m gpu -x -v --timeout 200 --timeout-method thread -k "two_processes" > gpurun_out/moe_mesh_ext_tests.log 2>&1 && \
timeout -k 10 400 python -u scripts/fa_variants.py '[{"sum_mfma": true, "fold_max": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true}, {"sum_mfma": true}, {"sum_mfma": true, "fold_max": true}]' --causal > gpurun_out/fa_causal_v4.log 2>&1 && \
timeout -k 10 400 python -u benchmarks/mamba2/benchmark_mamba_chunk_scan.py --out gpurun_out/benchmarks --rows 4096 > gpurun_out/mamba_xcd.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2.log 2>&1
