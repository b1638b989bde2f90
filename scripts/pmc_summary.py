"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (mean per dispatch).

    python scripts/pmc_summary.py <regex> file1.csv [file2.csv ...] > summary.md

Only kernels whose name matches <regex> are kept (the CSVs also hold torch's RNG kernels).
Derived columns when the counters are present:
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 256 CUs ... ) is not derivable without
                the clock, so we report MFMA busy per wave-cycle instead:
  mfma/wave   = SQ_VALU_MFMA_BUSY_CYCLES / (4 * SQ_WAVE_CYCLES)  (WAVE_CYCLES counts quad-cycles)
  lds_confl   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES, stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
"""
import collections
import csv
import re
import sys


def main():
    pat = re.compile(sys.argv[1])
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sys.argv[2:]:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not pat.search(name):
                continue
            acc[name[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for name, ctrs in acc.items():
        print(f"### {name}\n")
        print("| counter | mean per dispatch | dispatches |\n|---|---|---|")
        mean = {}
        for c in sorted(ctrs):
            v = ctrs[c]
            mean[c] = sum(v) / len(v)
            print(f"| {c} | {mean[c]:.4g} | {len(v)} |")
        der = []
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "SQ_BUSY_CU_CYCLES" in mean:
            der.append(("MFMA busy / CU busy", mean["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, 4 * mean["SQ_BUSY_CU_CYCLES"])))
        if "SQ_LDS_BANK_CONFLICT" in mean and "SQ_LDS_IDX_ACTIVE" in mean:
            der.append(("LDS bank-conflict cycles / LDS active cycles",
                        mean["SQ_LDS_BANK_CONFLICT"] / max(1.0, mean["SQ_LDS_IDX_ACTIVE"])))
        if "SQ_WAVE_CYCLES" in mean:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in mean:
                    der.append((f"{c} / SQ_WAVE_CYCLES", mean[c] / max(1.0, mean["SQ_WAVE_CYCLES"])))
        if der:
            print("\n| derived | value |\n|---|---|")
            for k, v in der:
                print(f"| {k} | {v:.3f} |")
        print()


if __name__ == "__main__":
    main()
