"""Convert an HF DeepSeek-V3.2 checkpoint into per-rank shards (reference:
examples/deepseek_v32/inference/convert.py).

    python examples/deepseek_v32/inference/convert.py --hf-ckpt-path /ckpt/DeepSeek-V3.2 \
        --save-path /ckpt/v32-mp8 --n-experts 256 --model-parallel 8

Writes ``model{rank}-mp{mp}.safetensors`` (column-parallel weights split on dim 0, row-parallel on
dim 1, routed experts dealt out whole, fp8 block scales split with their weights) plus the
tokenizer files; ``generate.py --ckpt-path`` loads the rank's shard.  Implementation:
``tilelang.models.deepseek_v32_ckpt.convert``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", ".."))

from tilelang.models.deepseek_v32_ckpt import convert  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hf-ckpt-path", required=True)
    ap.add_argument("--save-path", required=True)
    ap.add_argument("--n-experts", type=int, required=True)
    ap.add_argument("--model-parallel", type=int, required=True)
    a = ap.parse_args()
    for p in convert(a.hf_ckpt_path, a.save_path, a.n_experts, a.model_parallel):
        print(p)


if __name__ == "__main__":
    main()
