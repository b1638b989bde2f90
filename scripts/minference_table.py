"""The reference's MInference table (examples/minference/README.md: B1 H1 D64 fp16, seq 8K-64K, vertical /
slash counts [1000, 200], [1000, 600], [800, 600]; H100 PCIe TileLang 0.105 ... 1.501 ms) on MI355X: the
index conversion (device kernel) and the sparse attention kernel, timed separately and together.

    python scripts/minference_table.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "minference")]

import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402
from example_vertical_slash_sparse_attn import convert_vertical_slash_indexes, vertical_slash_sparse_attention  # noqa: E402,E501

REF = {(8192, 1000, 200): 0.105, (8192, 1000, 600): 0.119, (8192, 800, 600): 0.122, (16384, 1000, 200): 0.167,
       (16384, 1000, 600): 0.258, (16384, 800, 600): 0.255, (32768, 1000, 200): 0.248, (32768, 1000, 600): 0.554,
       (32768, 800, 600): 0.558, (65536, 1000, 200): 0.524, (65536, 1000, 600): 1.501, (65536, 800, 600): 1.489}


def main():
    print("| SEQ_LEN | VS_LIST | convert ms | total ms (convert + attention) | H100 TileLang ms | vs H100 |")
    print("|---|---|---|---|---|---|")
    B, H, D = 1, 1, 64
    for (S, nv, ns), ref in REF.items():
        g = torch.Generator(device="cuda").manual_seed(0)
        q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.float16) for _ in range(3))
        v_idx = torch.randperm(S, device="cuda", generator=g)[:nv].view(1, 1, -1)
        s_idx = torch.randperm(S, device="cuda", generator=g)[:ns].view(1, 1, -1)
        s_idx[..., 0] = 0
        bn = 128 if S <= 32768 else 64
        vertical_slash_sparse_attention(q, k, v, v_idx, s_idx)
        t_conv = do_bench(lambda: convert_vertical_slash_indexes(v_idx, s_idx, S, 128, bn))
        t_all = do_bench(lambda: vertical_slash_sparse_attention(q, k, v, v_idx, s_idx))
        print(f"| {S} | [{nv}, {ns}] | {t_conv:.3f} | {t_all:.3f} | {ref:.3f} | {ref / t_all:.2f}x |", flush=True)


if __name__ == "__main__":
    main()
