set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_moe.py -x -v --timeout 120 --timeout-method thread -k "tail_balanced_gpu" > gpurun_out/moe_ext_test.log 2>&1 && \
timeout -k 10 400 python -u scripts/moe_gemm_probe.py '({}, dict(ext_M=32), {}, dict(ext_M=32))' > gpurun_out/moe_ext_probe.log 2>&1
