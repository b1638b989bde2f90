set -o pipefail
mkdir -p gpurun_out/benchmarks
timeout -k 10 120 ./csrc/probes/mfma_fp6_probe2 > gpurun_out/fp6_probe2.log 2>&1 || exit $?
# a numerics failure (pytest exit 1) does not stop the batch; a timeout / abort / fault does
timeout -k 10 300 python -u -m pytest tests/test_mx_gemm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/mx_fp6_tests.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
bash scripts/gpu_moe_ext.sh && \
timeout -k 10 120 python -u scripts/moe_combine_probe.py > gpurun_out/moe_combine.log 2>&1 && \
bash scripts/gpu_fa_cmd.sh && \
timeout -k 10 300 python -u scripts/fa_bwd_ab.py '[{}, {"tl.gemm_rs_pipe": 4}]' > gpurun_out/fa_bwd_ab.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/bench_b.log 2>&1
