"""Does the kernel float -> fp8 conversion agree bit-for-bit with torch (RNE)?"""
import torch

import tilelang
import tilelang.language as T

N = 1 << 20


@T.prim_func
def cvt(A: T.Tensor((N, ), "float32"), B: T.Tensor((N, ), "float8_e4m3fn"), C: T.Tensor((N, ), "float8_e5m2")):
    with T.Kernel(N // 1024, threads=256) as bx:
        for i in T.Parallel(1024):
            B[bx * 1024 + i] = A[bx * 1024 + i]
            C[bx * 1024 + i] = A[bx * 1024 + i]


k = tilelang.compile(cvt, out_idx=[1, 2], target="hip")
g = torch.Generator().manual_seed(0)
for scale in (1.0, 30.0, 400.0, 0.01):
    a = (torch.randn(N, generator=g) * scale).cuda()
    a = a.clamp(-448, 448)
    b, c = k(a)
    for name, out, dt in (("e4m3", b, torch.float8_e4m3fn), ("e5m2", c, torch.float8_e5m2)):
        ref = a.to(dt)
        diff = (out.view(torch.uint8) != ref.view(torch.uint8))
        nd = int(diff.sum())
        msg = f"scale {scale} {name}: {nd} / {N} differ"
        if nd:
            idx = diff.nonzero()[:6, 0]
            msg += "; e.g. " + ", ".join(f"{a[i].item():.6g}->{out[i].float().item():.6g} (torch {ref[i].float().item():.6g})"
                                          for i in idx.tolist())
            # bias: mean signed error of the kernel vs torch relative to |x|
            err_k = (out.float() - a).mean().item()
            err_t = (ref.float() - a).mean().item()
            msg += f"; mean err kernel {err_k:.3e} torch {err_t:.3e}"
        print(msg, flush=True)
