#!/bin/bash
set -u
mkdir -p gpurun_out/s3m
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s3m/prof -o bench --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/s3m/prof.log 2>&1 || { tail -20 $R/gpurun_out/s3m/prof.log; exit 1; }
cd $R
python3 - "$(find gpurun_out/s3m/prof -name '*kernel_trace.csv')" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r['Kernel_Name'][:60]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:8]:
    v2 = v[-40:]
    print(f"{k:60s} n={len(v)} last40: min {min(v2):.1f} med {sorted(v2)[len(v2)//2]:.1f} max {max(v2):.1f} us")
# alternate calls of the tb kernel: even = GEMM1, odd = GEMM2
tb = d.get('moe_expert_gemm_tb_kernel', [])
if tb:
    g1 = tb[-40::2]; g2 = tb[-39::2]
    print("GEMM1 med", sorted(g1)[len(g1)//2], "GEMM2 med", sorted(g2)[len(g2)//2])
PY
