#!/bin/bash
# session 3: persistent FA after the clamp, plus kernel-level time split of the backward examples
set -u
mkdir -p gpurun_out/s3d
export TMPDIR=/tmp
export PYTHONPATH=$PWD:${PYTHONPATH:-}
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u scripts/fa_persistent_ab.py > gpurun_out/s3d/fa_persistent_ab3.log 2>&1 || { grep -v amdgpu.ids gpurun_out/s3d/fa_persistent_ab3.log | tail -30; exit 1; }
grep TF gpurun_out/s3d/fa_persistent_ab3.log
prof() {  # name dir script args
  local n=$1 d=$2; shift 2
  cd $R/examples/$d && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s3d/$n -o $n --output-format csv -- python3 "$@" > $R/gpurun_out/s3d/$n.log 2>&1 || { echo "$n FAILED"; tail -20 $R/gpurun_out/s3d/$n.log; cd $R; return 1; }
  cd $R; grep -E "TFLOPS|ms|us" gpurun_out/s3d/$n.log | grep -v amdgpu | tail -3
  python3 - "$(find gpurun_out/s3d/$n -name '*kernel_stats.csv')" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"  {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:70]}")
PY
}
prof fa_bwd flash_attention example_mha_bwd.py || exit 1
prof fa_bwd_causal flash_attention example_mha_bwd.py --causal || exit 1
prof varlen_bwd flash_attention example_mha_bwd_varlen.py || exit 1
prof nsa_bwd deepseek_nsa example_nsa_bwd.py || exit 1
