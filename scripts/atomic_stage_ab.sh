#!/bin/bash
# A/B of the LDS-staged fragment f32 atomics (TL_ATOMIC_STAGE=0 turns them off process-wide) on the
# kernels that end in tile atomics: NSA bwd dK/dV, the FA bwd single-kernel (atomic dQ) mode and the
# stream-K GEMM example.   bash scripts/atomic_stage_ab.sh [out_dir]
set -o pipefail
OUT=${1:-gpurun_out/atomic_ab}
mkdir -p $OUT
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
FA='import sys; sys.path.insert(0, "examples/flash_attention"); import example_mha_bwd as m; m.BWD_DQ_MODE = "atomic"; m.main()'
SK='import sys; sys.path.insert(0, "examples/gemm_streamk"); import example_tilelang_gemm_streamk as m; m.main(1024, 1024, 8192)'
for st in 0 1; do
  TL_ATOMIC_STAGE=$st timeout -k 10 200 python -u examples/deepseek_nsa/example_nsa_bwd.py > $OUT/nsa_$st.log 2>&1 || exit $?
  TL_ATOMIC_STAGE=$st timeout -k 10 200 python -u -c "$FA" > $OUT/fa_atomic_$st.log 2>&1 || exit $?
  TL_ATOMIC_STAGE=$st timeout -k 10 120 python -u -c "$SK" > $OUT/streamk_$st.log 2>&1 || exit $?
  echo "TL_ATOMIC_STAGE=$st"; grep -h -v amdgpu.ids $OUT/nsa_$st.log $OUT/fa_atomic_$st.log $OUT/streamk_$st.log
done
