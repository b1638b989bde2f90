#!/bin/bash
# MoE layer kernel breakdown (rocprofv3 --kernel-trace --stats) on one MI355X.
set -u
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${TAG:-moe}
mkdir -p $OUT
timeout -k 10 500 python scripts/prof_moe.py 20 --check > $OUT/moe.log 2>&1 || { tail -30 $OUT/moe.log; exit 1; }
cat $OUT/moe.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o moe --output-format csv -- python3 $ROOT/scripts/prof_moe.py 10 > $OUT/prof.log 2>&1 || { tail -30 $OUT/prof.log; exit 1; }
cd $ROOT
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{float(r["TotalDurationNs"])/1e3:10.1f} us {int(r["Calls"]):5d} calls {float(r["AverageNs"])/1e3:8.1f} us avg  {r["Name"][:110]}')
PY
