"""Causal FA backward kernels (examples/flash_attention/example_mha_bwd.py): the causal select on
every tile (``mask_split=False``) vs only on the tiles that cross the diagonal, behind a uniform
branch (``mask_split=True``).  Default causal tiles, same process, round-robin, checked against
fp32 autograd.

    python scripts/fa_bwd_mask_split_ab.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "examples", "flash_attention"))

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
import example_mha_bwd as E  # noqa: E402


def main():
    torch.manual_seed(0)
    for B, H, S, D in ((8, 32, 1024, 64), (2, 32, 4096, 64), (4, 32, 2048, 128)):
        q, k, v, do = (torch.randn(B, S, H, D, device="cuda", dtype=torch.float16) for _ in range(4))
        qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
        E.ref_program(qr, kr, vr, True).float().backward(do.float())
        gq, gk, gv = qr.grad, kr.grad, vr.grad
        o, lse = E.flashattn_fwd(B, H, S, D, True, dtype="float16", **E._tiles(D, D, "fwd", True, S))(q, k, v)
        delta = E.flashattn_bwd_preprocess(B, H, S, D, dtype="float16")(o, do)
        unit = 2.0 * B * H * S * S * D * 0.5
        bw, dqt = E._tiles(D, D, "bwd", True, S), E._tiles(D, D, "dq", True, S)
        dk, dv = torch.empty_like(k), torch.empty_like(v)
        kd = {m: E.flashattn_bwd(B, H, S, D, True, dtype="float16", dq_mode="none", mask_split=m, **bw)
              for m in (False, True)}
        kq = {m: E.flashattn_bwd_dq(B, H, S, D, True, dtype="float16", mask_split=m, **dqt) for m in (False, True)}
        res = {}
        for m in (False, True):
            kd[m](q, k, v, do, lse, delta, dk, dv)
            dq = kq[m](q, k, v, do, lse, delta)
            res[m] = [1e9, 1e9, max((dk.float() - gk).abs().max().item(), (dv.float() - gv).abs().max().item(),
                                    (dq.float() - gq).abs().max().item())]
        for _ in range(3):
            for m in (False, True):
                res[m][0] = min(res[m][0], do_bench(lambda: kd[m](q, k, v, do, lse, delta, dk, dv), warmup=10, rep=50))
                res[m][1] = min(res[m][1], do_bench(lambda: kq[m](q, k, v, do, lse, delta), warmup=10, rep=50))
        print(f"causal b{B} h{H} s{S} d{D}: " + "  ".join(
            f"mask_split={int(m)} dkv {a * 1e3:.1f} us ({4 * unit / a * 1e-9:.0f} TF) dq {b * 1e3:.1f} us "
            f"({3 * unit / b * 1e-9:.0f} TF) err {e:.3f}" for m, (a, b, e) in res.items()), flush=True)


if __name__ == "__main__":
    main()
