#!/bin/bash
# round-5 GPU check: parity / atomic / RCCL world-1 tests, then FA variant A/B (fold vs fma path)
set -u
OUT=${1:-gpurun_out/r5b}
mkdir -p $OUT
export PYTHONPATH=$PWD:${PYTHONPATH:-}
timeout -k 10 600 python -u -m pytest tests/test_language_parity.py tests/test_language_atomic.py tests/test_gpu_rccl.py tests/test_stage_schedule.py -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" $OUT/pytest.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u scripts/fa_variants.py '[{"sum_mfma": true, "fold_max": true, "young_prio": true, "xcd_heads": true}, {"sum_mfma": true, "fold_max": false, "young_prio": true, "xcd_heads": true}, {"sum_mfma": true, "fold_max": true, "xcd_heads": true}, {"sum_mfma": true, "fold_max": false, "xcd_heads": true}, {"sum_mfma": false, "fold_max": false, "xcd_heads": true, "young_prio": true}]' > $OUT/fa_ab.log 2>&1
echo "fa rc=$?"; tail -8 $OUT/fa_ab.log
