set -o pipefail
bash scripts/gpu_suite.sh gpurun_out/suite_r4c || exit $?
timeout -k 10 300 python -u scripts/router_probe.py > gpurun_out/router_probe.log 2>&1
