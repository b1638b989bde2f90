set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/fa_variants.py '[{"sum_mfma": true, "fold_max": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true}, {"sum_mfma": true, "fold_max": true, "pingpong": true}, {"sum_mfma": true, "fold_max": true, "pingpong": true, "young_prio": true}, {"sum_mfma": true, "fold_max": true}]' > gpurun_out/fa_v4.log 2>&1
