"""MoE dispatch plan (align_kernel) on the bench layer's shape: the wave-vote form (default on
gfx950) vs the LDS-atomic form -- identical counts / tile tables, every assignment placed once,
vote placement in assignment order; timings.

    python scripts/align_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tilelang.ops import moe as K  # noqa: E402
from tilelang.profiler import do_bench  # noqa: E402

n, E, slot, div = 4096, 8, 288, 2
mr = K.max_padded_rows(n, E, slot)
torch.manual_seed(0)
for name, ids in (("random", torch.randint(0, E, (n, ), device="cuda", dtype=torch.int32)),
                  ("balanced", torch.arange(n, device="cuda", dtype=torch.int32) % E),
                  ("with -1", torch.where(torch.rand(n, device="cuda") < 0.1, -1,
                                          torch.randint(0, E, (n, ), device="cuda")).int())):
  for stable in (False, True):
      outs, ts = {}, {}
      for vote in (False, True):
          k = K.align_kernel(n, E, slot, mr, div, "hip", stable=stable, even=True, vote=vote)
          o = [torch.empty(n, dtype=torch.int32, device="cuda"), torch.empty(mr, dtype=torch.int32, device="cuda"),
               torch.empty(mr // slot, dtype=torch.int32, device="cuda"), torch.empty(E, dtype=torch.int32, device="cuda"),
               torch.empty(mr // slot, dtype=torch.int32, device="cuda")]
          k(ids, *o)
          torch.cuda.synchronize()
          outs[vote] = o
          ts[vote] = do_bench(lambda: k(ids, *o), warmup=20, rep=200)
      a, v = outs[False], outs[True]
      same_tables = all(torch.equal(a[i], v[i]) for i in (2, 3, 4))
      dest, rs = v[0], v[1]
      ok = (dest >= 0) == (ids >= 0)
      placed = dest[dest >= 0].long()
      ok &= True
      perm_ok = bool(ok.all()) and placed.unique().numel() == placed.numel() and \
          torch.equal(rs[placed], (torch.arange(n, device="cuda")[dest >= 0] // div).int())
      # order inside each expert: increasing assignment index <-> increasing padded row
      order_ok = True
      for e in range(E):
          js = torch.nonzero(ids == e).flatten()
          if js.numel() > 1:
              order_ok &= bool((dest[js][1:] > dest[js][:-1]).all())
      print(f"{name} stable={stable}: tables equal {same_tables}, placement ok {perm_ok}, stable {order_ok}, "
            f"atomic {ts[False] * 1e3:.2f} us, vote {ts[True] * 1e3:.2f} us", flush=True)
