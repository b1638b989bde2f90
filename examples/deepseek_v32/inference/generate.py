"""DeepSeek-V3.2 generation, one process per MI355X (reference: examples/deepseek_v32/inference/generate.py).

    python examples/deepseek_v32/inference/generate.py --config tiny --max-new-tokens 16
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/deepseek_v32/inference/generate.py \
        --config examples/deepseek_v32/inference/config_671B_v3.2.json --layers 4

Tensor + expert parallel over RCCL (``torch.distributed`` backend "nccl" on ROCm).  With
``--ckpt-path`` every rank loads ``model{rank}-mp{world}.safetensors`` written by convert.py
(reference generate.py:119); without it the weights are random.  ``--layers`` truncates the
61-layer config so a slice of the full-width model fits a quick run.  Prints tokens/s of the
decode phase.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tilelang.models.deepseek_v32 import ModelArgs, Transformer, generate  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="tiny")
    ap.add_argument("--layers", type=int, default=None)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--max-new-tokens", type=int, default=16)
    ap.add_argument("--max-seq-len", type=int, default=512)
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--ckpt-path", default=None, help="directory of convert.py shards")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    over = dict(max_batch_size=a.batch, max_seq_len=a.max_seq_len)
    if a.layers is not None:
        over["n_layers"] = a.layers
    args = ModelArgs.tiny(**over) if a.config == "tiny" else ModelArgs.from_json(a.config, **over)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    torch.manual_seed(0)
    model = Transformer(args, seed=0, device=dev)
    if a.ckpt_path:
        from tilelang.models.deepseek_v32_ckpt import load_model
        load_model(model, os.path.join(a.ckpt_path, f"model{rank}-mp{world}.safetensors"))
    prompts = [torch.randint(0, args.vocab_size, (a.prompt_len, )).tolist() for _ in range(a.batch)]
    generate(model, prompts, 2)  # warm-up: compiles every kernel shape used by prefill + decode
    if dev == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = generate(model, prompts, a.max_new_tokens, a.temperature)
    if dev == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if rank == 0:
        print(f"generated {a.batch}x{a.max_new_tokens} tokens on {world} rank(s) in {dt:.2f}s "
              f"({a.batch * a.max_new_tokens / dt:.1f} tok/s incl. prefill)")
        print(out[0][:16])
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
