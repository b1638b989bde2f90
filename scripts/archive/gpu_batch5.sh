set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/fa_variants.py '[{"sum_mfma": true, "fold_max": true, "young_prio": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true, "skip_masked": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true, "skip_masked": true}]' --causal > gpurun_out/fa_causal_skip.log 2>&1 && \
bash scripts/gpu_pmc.sh gpurun_out/pmc_r4c && \
timeout -k 10 400 python -u scripts/sink_ab.py > gpurun_out/sink_fold_ab.log 2>&1
