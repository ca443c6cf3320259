#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSV output per kernel.

    python tools/py/pmc_summary.py gpurun_out/pmc_sq gpurun_out/pmc_tcc ... > profiles/x.md

Sums each counter over a kernel's dispatches (one CSV row per dispatch and
counter), prints one markdown table row per kernel with derived ratios:
L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS), LDS bank conflicts per LDS
instruction, VALU / VMEM instructions per wave.
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("bibfs::(anonymous namespace)::", "").replace("void ", "")
    name = re.sub(r"\(.*", "", name)
    return name[:60]


def main(dirs):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    dur = defaultdict(float)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for row in csv.DictReader(open(f)):
                k = short(row["Kernel_Name"])
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                key = (f, row["Dispatch_Id"])
                disp[k].add(key)
                if key not in seen:
                    seen.add(key)
                    dur[k] += (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3
    counters = sorted({c for k in tot for c in tot[k]})
    print("| kernel | dispatches | " + " | ".join(counters) + " | L2 hit % | LDS conflicts / LDS inst |")
    print("|---" * (len(counters) + 4) + "|")
    for k in sorted(tot, key=lambda k: -len(disp[k])):
        t = tot[k]
        hit = t.get("TCC_HIT_sum", 0.0)
        miss = t.get("TCC_MISS_sum", 0.0)
        l2 = f"{100 * hit / (hit + miss):.1f}" if hit + miss else "-"
        lds = t.get("SQ_INSTS_LDS", 0.0)
        conf = f"{t.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds:.3f}" if lds else "-"
        print(f"| {k} | {len(disp[k])} | " + " | ".join(f"{t.get(c, 0):.4g}" for c in counters) + f" | {l2} | {conf} |")


if __name__ == "__main__":
    main(sys.argv[1:] or ["gpurun_out"])
