"""A/B of the FA forward epilogue (bench config): direct fragment stores vs the O tile through
row-padded LDS (flashattn_pipelined(staged_epilogue=True)); same process, interleaved."""
import sys

import torch

import tilelang
from tilelang.profiler import do_bench

sys.path.insert(0, "examples/flash_attention")
from example_mha_fwd_pipelined import flashattn_pipelined as fa  # noqa: E402
from example_mha_fwd import ref_program  # noqa: E402

B, H, S, D = 1, 64, 4096, 128
q, k, v = (torch.randn(B, S, H, D, device="cuda").to(torch.bfloat16) for _ in range(3))
ref = ref_program(q, k, v, False, 1)
ks = {}
for st in (False, True):
    f = fa.get_tir(B, H, S, D, False, 1, 256, 64, 512, 2, "bfloat16", True, True, False, st)
    ks[st] = tilelang.compile(f, out_idx=[3], target="hip", pass_configs=fa.pass_configs)
    torch.testing.assert_close(ks[st](q, k, v).float(), ref.float(), rtol=2e-2, atol=2e-2)
fl = 4.0 * B * H * S * S * D
cold, warm = {False: [], True: []}, {False: [], True: []}
for _ in range(6):
    for st in (False, True):
        cold[st].append(do_bench(lambda: ks[st](q, k, v), warmup=10, rep=50))
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(20):
            ks[st](q, k, v)
        ev[1].record()
        torch.cuda.synchronize()
        warm[st].append(ev[0].elapsed_time(ev[1]) / 20)
for st in (False, True):
    print(f"{'staged' if st else 'direct'}: cold {fl / min(cold[st]) * 1e-9:.0f} TF, warm {fl / min(warm[st]) * 1e-9:.0f} TF",
          flush=True)
