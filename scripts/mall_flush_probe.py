"""Does do_bench's cache flush evict the 256 MiB Infinity Cache (MALL)?  

A streaming copy of a buffer that FITS in the MALL (16-128 MiB) is timed three ways in one
process: no flush (the previous launch left the data MALL-resident), the default read flush
(a max-reduction over 512 MiB) and the reference's write flush.  If the flush evicts, the
flushed copy of a MALL-sized buffer runs at the HBM rate of a 1 GiB buffer (which never fits),
and the unflushed one faster.  Prints one line per size; GB/s counts read + write bytes.

    python scripts/mall_flush_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tilelang.profiler import do_bench  # noqa: E402


def main():
    for mib in (16, 64, 128, 1024):
        n = mib * 1024 * 1024 // 4
        a = torch.randn(n, device="cuda")
        b = torch.empty_like(a)
        fn = lambda: b.copy_(a)  # noqa: E731
        nbytes = 2 * a.numel() * 4
        res = {}
        for mode, kw in (("none", dict(flush_l2=False)), ("read", dict(flush_mode="read")),
                         ("write", dict(flush_mode="write"))):
            ms = do_bench(fn, warmup=20, rep=100, return_mode="median", **kw)
            res[mode] = nbytes / ms / 1e6
        print(f"copy {mib:5d} MiB: no flush {res['none']:7.0f} GB/s | read flush {res['read']:7.0f} GB/s | "
              f"write flush {res['write']:7.0f} GB/s", flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
