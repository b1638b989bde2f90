"""DeepSeek-V3.2 (DSA) model on tilelang kernels: cache consistency and TP/EP equivalence (CPU, gloo)."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from tilelang.models.deepseek_v32 import ModelArgs, Transformer, generate


def test_incremental_decode_matches_prefill():
    args = ModelArgs.tiny()
    m = Transformer(args, seed=0, device="cpu")
    toks = torch.randint(0, args.vocab_size, (2, 12), generator=torch.Generator().manual_seed(1))
    full = m(toks, 0)
    m2 = Transformer(args, seed=0, device="cpu")
    m2(toks[:, :11], 0)
    step = m2(toks[:, 11:12], 11)
    torch.testing.assert_close(step, full, rtol=3e-2, atol=3e-2)


def test_generate_greedy_is_deterministic():
    args = ModelArgs.tiny()
    m = Transformer(args, seed=0, device="cpu")
    a = generate(m, [[1, 2, 3, 4], [5, 6]], 3)
    m2 = Transformer(args, seed=0, device="cpu")
    assert generate(m2, [[1, 2, 3, 4], [5, 6]], 3) == a
    assert all(len(x) == 3 and all(0 <= t < args.vocab_size for t in x) for x in a)


def _tp_worker(rank, world, port, toks, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m = Transformer(ModelArgs.tiny(), seed=0, device="cpu")
        logits = m(toks, 0)
        if rank == 0:
            torch.save(logits, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_tensor_and_expert_parallel_match_single_rank(tmp_path):
    """world=2: heads / FFN split (TP), routed experts split (EP), vocab-parallel embedding and
    head -- the logits must equal the single-process model's."""
    args = ModelArgs.tiny()
    toks = torch.randint(0, args.vocab_size, (2, 8), generator=torch.Generator().manual_seed(3))
    ref = Transformer(args, seed=0, device="cpu")(toks, 0)
    out = str(tmp_path / "tp2.pt")
    port = 29500 + (os.getpid() % 2000)
    mp.spawn(_tp_worker, args=(2, port, toks, out), nprocs=2, join=True)
    torch.testing.assert_close(torch.load(out, weights_only=True), ref, rtol=3e-2, atol=3e-2)


def test_fp8_checkpoint_format_model():
    """gemm_impl='fp8': every projection is fp8 e4m3 + 128x128 block scales, run as act_quant +
    block-scaled fp8 GEMM (reference model.py ``linear``); logits stay close to the bf16 model
    built from the same weights (fp8 weight/activation rounding only)."""
    from tilelang.models import deepseek_v32 as D
    toks = torch.randint(0, 512, (2, 8), generator=torch.Generator().manual_seed(5))
    ref = Transformer(ModelArgs.tiny(), seed=0, device="cpu")(toks, 0)
    m = Transformer(ModelArgs.tiny(gemm_impl="fp8"), seed=0, device="cpu")
    fp8_layers = [x for x in m.modules() if isinstance(x, D.Linear) and x.scale is not None]
    assert len(fp8_layers) > 10 and all(x.weight.dtype == torch.float8_e4m3fn for x in fp8_layers)
    assert m.head.scale is None  # the output head stays bf16, as the reference's
    out = m(toks, 0)
    rel = (out.float() - ref.float()).norm() / ref.float().norm()
    assert rel < 0.15, rel
    m2 = Transformer(ModelArgs.tiny(gemm_impl="fp8", scale_fmt="ue8m0"), seed=0, device="cpu")
    assert torch.isfinite(m2(toks, 0)).all()
