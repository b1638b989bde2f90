"""VGPR / AGPR / spill / LDS usage of DSL kernels from the compiler's resource remarks (CPU only:
cross-compiles for gfx950).

    python scripts/kernel_resources.py fa '[{"threads": 256}, {"threads": 256, "mfma": "32x32"}]'
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples", "flash_attention")]

import tilelang  # noqa: E402
from tilelang.contrib.hipcc import clang_path  # noqa: E402


def resources(src: str) -> dict:
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "k.hip")
        open(p, "w").write(src)
        inc = os.path.join(ROOT, "tilelang", "include")
        r = subprocess.run([clang_path(), "-x", "hip", "--offload-arch=gfx950", "--offload-device-only",
                            "--no-gpu-bundle-output", "-O3", "-std=c++17", f"-I{inc}", "-c", p, "-o",
                            os.path.join(d, "k.o"), "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
    out = {}
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("sgpr", r"SGPRs: (\d+)"),
                     ("spill_v", r"VGPRs Spill: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                     ("occupancy", r"Occupancy \[waves/SIMD\]: (\d+)")):
        m = re.search(pat, r.stderr)
        out[key] = int(m.group(1)) if m else None
    if r.returncode != 0:
        out["error"] = r.stderr[-800:]
    return out


def main():
    which = sys.argv[1]
    variants = json.loads(sys.argv[2]) if len(sys.argv) > 2 else [{}]
    if which == "fa":
        from example_mha_fwd_pipelined import flashattn_pipelined
        for kw in variants:
            a = dict(block_M=256, block_N=64, threads=512, num_stages=2, q_in_regs=True, sum_mfma=True,
                     fold_max=True)
            pc = dict(flashattn_pipelined.pass_configs)
            pc.update(kw.get("_pc", {}))  # extra pass configs, e.g. {"tl.min_waves_per_eu": 2}
            a.update({k: v for k, v in kw.items() if k != "_pc"})
            f = flashattn_pipelined.get_tir(1, 64, 4096, 128, False, 1, **a)
            src = tilelang.lower(f, target="hip", pass_configs=pc).kernel_source
            print(json.dumps(kw), resources(src), flush=True)


if __name__ == "__main__":
    main()


def isa(src: str) -> str:
    """gfx950 assembly of a generated kernel source (for instruction counts per loop)."""
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "k.hip")
        open(p, "w").write(src)
        inc = os.path.join(ROOT, "tilelang", "include")
        out = os.path.join(d, "k.s")
        subprocess.run([clang_path(), "-x", "hip", "--offload-arch=gfx950", "--offload-device-only",
                        "--no-gpu-bundle-output", "-O3", "-std=c++17", f"-I{inc}", "-S", p, "-o", out], check=True)
        return open(out).read()
