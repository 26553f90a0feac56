#!/usr/bin/env python3
"""Per-wave SQ figures of the kernels in the PMC passes under OUT (tools/sq_lz.sh).

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md,
"s_memtime tick vs SQ PMC units"); the instruction counts are per wave; WAIT_ANY +
WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES.  VALU issue: a wave64 VALU instruction
takes 2 cycles of its SIMD, so `valu_issue_share` = 2 * VALU per wave * waves per SIMD /
cycles of one wave — the fraction of the SIMD's cycles the kernel's VALU needs at its
occupancy (near 1: issue-bound)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("kolm::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def main():
    out = sys.argv[1]
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            per[short(row.get("Kernel_Name", ""))][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in per.items():
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        w = avg.get("SQ_WAVES", 0.0) or 1.0
        print(f"{k}: dispatches {max(len(v) for v in cs.values())}, waves {w:.0f}")
        for c in sorted(avg):
            if c == "SQ_WAVES":
                continue
            print(f"  {c:24s} total {avg[c]:.4g}  per wave {avg[c] / w:.1f}")
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            cyc = 4 * wc / w  # cycles per wave
            print(f"  cycles per wave {cyc:.0f}")
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c in avg:
                    print(f"  {c[3:]:20s} {avg[c] / wc * 100:.1f} % of wave cycles")
            if "SQ_INSTS_VALU" in avg:
                print(f"  VALU issue cycles per wave (2 per instruction) {2 * avg['SQ_INSTS_VALU'] / w:.0f} "
                      f"= {2 * avg['SQ_INSTS_VALU'] / w / cyc * 100:.1f} % of one wave's cycles")
        if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
            print(f"  LDS bank-conflict share {avg['SQ_LDS_BANK_CONFLICT'] / avg['SQ_LDS_IDX_ACTIVE'] * 100:.1f} %")


if __name__ == "__main__":
    main()
