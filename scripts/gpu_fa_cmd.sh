set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_intrinsics.py -m gpu -k reduce_k > gpurun_out/rk_tests.log 2>&1 && \
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4pmc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r4a.log 2>&1 && \
timeout -k 10 400 python -u scripts/fa_variants.py '[{"sum_mfma": true}, {"sum_mfma": true, "fold_max": true}, {"sum_mfma": true, "fold_max": true, "young_prio": true}]' --causal > gpurun_out/fa_causal.log 2>&1 && \
cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_LDS --output-format csv -d $R/gpurun_out/r4pmc/p1 -o p -- python3 $R/scripts/prof_bench.py fa 10 > $R/gpurun_out/r4pmc/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM --output-format csv -d $R/gpurun_out/r4pmc/p2 -o p -- python3 $R/scripts/prof_bench.py fa 10 > $R/gpurun_out/r4pmc/p2.log 2>&1 && \
cd $R && python scripts/pmc_summary.py "flashattn" $(find gpurun_out/r4pmc/p1 gpurun_out/r4pmc/p2 -name "*counter_collection.csv") > gpurun_out/r4pmc/fa.md
