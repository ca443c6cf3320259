#!/usr/bin/env python3
"""Per-query kernel timeline from a rocprofv3 --kernel-trace CSV.

    python tools/py/query_timeline.py <kernel_trace.csv> [--start KERNEL] [--queries N]

Splits the trace at every dispatch of --start (default: the one-shot LDS
search kernel), prints the median query's kernels with start offset, gap
from the previous kernel's end and duration, and a per-kernel median summary.
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def short(n):
    n = n.replace("bibfs::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--start", default="k_lds_bibfs")
    ap.add_argument("--last", type=int, default=30, help="use the last N queries")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.start in r["Kernel_Name"]]
    qs = []
    for j in range(len(starts) - 1):
        qs.append(rows[starts[j]:starts[j + 1]])
    qs = qs[-a.last:]
    spans = [(int(q[-1]["End_Timestamp"]) - int(q[0]["Start_Timestamp"])) / 1e3 for q in qs]
    med = sorted(range(len(qs)), key=lambda i: spans[i])[len(qs) // 2]
    q = qs[med]
    t0 = int(q[0]["Start_Timestamp"])
    prev = None
    print(f"median query: {spans[med]:.1f} us from first to last kernel end ({len(q)} kernels)")
    for r in q:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"  {(s - t0) / 1e3:8.2f} +{gap:6.2f} dur {(e - s) / 1e3:7.2f}  grid {r['Grid_Size_X']:>8}  {short(r['Kernel_Name'])}")
        prev = e
    dur = defaultdict(list)
    for qq in qs:
        per = defaultdict(float)
        for r in qq:
            per[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        for k, v in per.items():
            dur[k].append(v)
    print("per-query kernel time (median over queries that ran it):")
    for k, v in sorted(dur.items(), key=lambda kv: -statistics.median(kv[1])):
        print(f"  {statistics.median(v):8.2f} us  x{len(v):3d}  {k}")


if __name__ == "__main__":
    main()
