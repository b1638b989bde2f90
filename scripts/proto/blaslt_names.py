"""Runs the vendor GEMMs the quad loop is compared against (fp16 NT 4096^3, 8192^2 x 4096, 8192^3 and
fp8 _scaled_mm 8192^3) a few times each, so a rocprofv3 kernel trace names the hipBLASLt kernels
(their names carry the macro tile, depth-U and schedule options)."""
import torch

for M, N, K in ((4096, 4096, 4096), (8192, 8192, 4096), (8192, 8192, 8192)):
    x = torch.empty(M, K, device="cuda", dtype=torch.float16).uniform_(-1, 1)
    y = torch.empty(N, K, device="cuda", dtype=torch.float16).uniform_(-1, 1)
    for _ in range(3):
        x @ y.T
a = torch.randn(8192, 8192, device="cuda").to(torch.float8_e4m3fn)
b = torch.randn(8192, 8192, device="cuda").to(torch.float8_e4m3fn)
one = torch.ones((), device="cuda")
for _ in range(3):
    torch._scaled_mm(a, b.T, scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
torch.cuda.synchronize()
print("done")
