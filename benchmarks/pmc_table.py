#!/usr/bin/env python3
"""Markdown table of a rocprofv3 --pmc counter_collection.csv: per kernel,
dispatches and the summed counters, plus LDS bank-conflict cycles per LDS
instruction.

    python benchmarks/pmc_table.py gpurun_out/TAG_pmc_sq/*/NNN_counter_collection.csv [--title T]
"""
import argparse
import collections
import csv
import re


def short(name):
    name = name.split("(")[0] if "(anonymous" not in name else re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--title", default="")
    a = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    names = []
    for r in csv.DictReader(open(a.csv)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
        if r["Counter_Name"] not in names:
            names.append(r["Counter_Name"])
    if a.title:
        print(f"# {a.title}")
    print("| kernel | dispatches | " + " | ".join(names) + " | LDS conflicts / LDS inst |")
    print("|---|---|" + "---|" * len(names) + "---|")
    for k in sorted(vals, key=lambda k: -vals[k].get("SQ_WAVE_CYCLES", 0)):
        v = vals[k]
        lds = v.get("SQ_INSTS_LDS", 0)
        ratio = f"{v.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.3f}" if lds else "-"
        print(f"| {k} | {len(disp[k])} | " + " | ".join(f"{v.get(n, 0):.4g}" for n in names) + f" | {ratio} |")


if __name__ == "__main__":
    main()
