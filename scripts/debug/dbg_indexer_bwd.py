import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "dsa_sparse_finetune")]
import torch
from indexer_topk_reducesum import indexer_topk_reducesum_interface
from indexer_bwd import indexer_bwd_interface, indexer_bwd
from dsa import ref_indexer_loss
for HI in (16, 32, 64):
    torch.manual_seed(0)
    S, DI, topk = 128, 64, 64
    iq = torch.randn(S, HI, DI).bfloat16(); ik = torch.randn(S, DI).bfloat16(); w = torch.randn(S, HI).bfloat16()
    offsets = torch.tensor([0, 50, S], dtype=torch.int32)
    _, score, idx_abs = indexer_topk_reducesum_interface(iq.cuda(), w.cuda(), ik.cuda(), topk, offsets.cuda(), return_abs=True)
    att = torch.rand(S, topk, device="cuda") * (idx_abs >= 0); att = att / att.sum(-1, keepdim=True)
    dq, dw, dk = indexer_bwd_interface(iq.cuda(), w.cuda(), ik.cuda(), att, score, idx_abs)
    rs = [x.float().requires_grad_(True) for x in (iq, w, ik)]
    ref_indexer_loss(rs[0], rs[1], rs[2], idx_abs.cpu(), att.cpu()).backward()
    for n, a, r in zip(("dq","dw","dk"), (dq, dw, dk), rs):
        e = (a.float().cpu()-r.grad)
        print(HI, n, e.abs().max().item(), r.grad.abs().max().item(), "bad rows", (e.abs().amax(-1) > 0.05).nonzero()[:5].flatten().tolist() if e.dim() > 1 else "")
src = indexer_bwd(128, 32, 64, 64).get_kernel_source()
open(os.path.join(ROOT, "gpurun_out", "indexer_bwd32.hip"), "w").write(src)
