"""Block-sparse GQA decode, paged variant (reference: examples/blocksparse_attention/
example_tilelang_sparse_gqa_decode_paged.py).  Kernels: sparse_gqa_decode.py."""
import argparse

import torch

from sparse_gqa_decode import (indices_to_mask, random_selection, ref_program, sparse_gqa_decode_indice,  # noqa: F401
                               sparse_gqa_decode_mask, sparse_gqa_decode_paged)


def run(batch=8, heads=32, heads_kv=8, max_cache_seqlen=8192, dim=128, block_size=32, sparse_ratio=0.8,
        device="cuda", num_split=4, check=True):
    nb = max_cache_seqlen // block_size
    max_sel = max(1, int(nb * (1 - sparse_ratio)))
    g = torch.Generator().manual_seed(0)
    cache_seqlens = torch.randint(max_cache_seqlen // 2, max_cache_seqlen + 1, (batch, ), generator=g).int().to(device)
    q = torch.randn(batch, heads, dim, device=device, dtype=torch.float16)
    k = torch.randn(batch, max_cache_seqlen, heads_kv, dim, device=device, dtype=torch.float16)
    v = torch.randn_like(k)
    idx = random_selection(batch, heads_kv, cache_seqlens.cpu(), block_size, max_sel, device)
    mode = "paged"
    if mode == "varlen_indice":
        kern = sparse_gqa_decode_indice(batch, heads, heads_kv, dim, block_size, max_cache_seqlen, max_sel,
                                        num_split=num_split)
        fn = lambda: kern(q, k, v, idx, cache_seqlens)[-1]  # noqa: E731
    elif mode == "varlen_mask":
        mask = indices_to_mask(idx, nb)
        kern = sparse_gqa_decode_mask(batch, heads, heads_kv, dim, block_size, max_cache_seqlen, num_split=num_split)
        fn = lambda: kern(q, k, v, mask, cache_seqlens)[-1]  # noqa: E731
    else:
        page_size = 64
        max_pages = max_cache_seqlen // page_size
        num_pages = batch * max_pages
        perm = torch.randperm(num_pages, generator=g).int()
        table = perm.view(batch, max_pages).to(device)
        kc = torch.empty(num_pages, page_size, heads_kv, dim, device=device, dtype=torch.float16)
        vc = torch.empty_like(kc)
        kc[table.view(-1).long()] = k.view(batch * max_pages, page_size, heads_kv, dim)
        vc[table.view(-1).long()] = v.view(batch * max_pages, page_size, heads_kv, dim)
        kern = sparse_gqa_decode_paged(batch, heads, heads_kv, dim, block_size, num_pages, page_size, max_pages,
                                       max_sel, num_split=num_split)
        fn = lambda: kern(q, kc, vc, idx, cache_seqlens, table)[-1]  # noqa: E731
    o = fn()
    if check:
        torch.testing.assert_close(o.float(), ref_program(q, k, v, idx, cache_seqlens, block_size), rtol=2e-2,
                                   atol=2e-2)
    return fn


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=8)
    p.add_argument("--heads", type=int, default=32)
    p.add_argument("--heads_kv", type=int, default=8)
    p.add_argument("--max_cache_seqlen", type=int, default=8192)
    p.add_argument("--sparse_ratio", type=float, default=0.8)
    a = p.parse_args()
    fn = run(a.batch, a.heads, a.heads_kv, a.max_cache_seqlen, sparse_ratio=a.sparse_ratio, check=False)
    fn()
    from tilelang.profiler import do_bench
    print(f"sparse GQA decode (paged): {do_bench(fn):.4f} ms")


if __name__ == "__main__":
    main()
