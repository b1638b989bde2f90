import sys, subprocess, json
import os; sys_path = __import__("sys").path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tilelang.ops.dsa import sparse_mla_fwd
import tilelang
cfg = json.loads(sys.argv[1])
f = sparse_mla_fwd.get_tir(1, 4096, 8192, 128, 512, 64, 2048, **cfg)
k = tilelang.compile(f, out_idx=[3,4], target='hip'); open('/tmp/s.hip','w').write(k.get_kernel_source())
out = subprocess.run(['bash','/root/repo/scripts/kres.sh','/tmp/s.hip'],capture_output=True,text=True).stdout
print(cfg, " | ".join(l.split("[")[0].strip() for l in out.splitlines() if any(x in l for x in ("VGPRs","AGPRs","Spill","LDS","Occ"))))
