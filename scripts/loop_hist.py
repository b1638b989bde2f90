"""Instruction histogram of the innermost loops of a gfx950 .s file: loop_hist.py kernel.s"""
import collections
import re
import sys

lines = open(sys.argv[1]).read().splitlines()
blocks = collections.defaultdict(collections.Counter)
hdr = None
for l in lines:
    m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):(.*)", l)
    if m:
        h = re.search(r"Header=BB(\d+_\d+)", l)
        if m.group(1).startswith(".LBB") and "Loop Header" in l:
            hdr = m.group(1)[4:]
        elif h:
            hdr = h.group(1)
        else:
            hdr = None
        continue
    if hdr is None:
        continue
    t = l.strip().split()
    if t and not t[0].startswith((".", ";")):
        blocks[hdr][t[0]] += 1
for h, c in blocks.items():
    print(f"loop BB{h}: {sum(c.values())} instructions")
    for k, v in c.most_common(int(sys.argv[2]) if len(sys.argv) > 2 else 30):
        print(f"  {k:32s} {v}")
