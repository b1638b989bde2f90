set -o pipefail
mkdir -p gpurun_out/benchmarks
timeout -k 10 120 ./csrc/probes/mfma_fp6_probe2 > gpurun_out/fp6_probe2.log 2>&1 && \
bash scripts/gpu_moe_ext.sh && \
bash scripts/gpu_fa_cmd.sh
