#!/usr/bin/env python3
"""Per-query kernel timelines of resident hand-off searches from a rocprofv3
kernel-trace CSV (`rocprofv3 --kernel-trace --output-format csv`): a query's
grid work starts at its k_handoff (auto chain) or its first grid kernel after
a gap; prints offsets / durations and the per-kernel medians.

    python benchmarks/grid_timeline.py gpurun_out/DIR/run_kernel_trace.csv [--queries 3]
"""
import argparse
import csv
import statistics


def short(name):
    for key in ("k_handoff", "k_grid_topdown", "k_grid_hubs", "k_cleanup", "k_grid_bottomup", "k_finish_level",
                "k_publish", "k_lds_server", "k_seed"):
        if key in name:
            return key + ("<auto>" if ", true>" in name else "")
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--queries", type=int, default=4)
    ap.add_argument("--gap-us", type=float, default=15.0, help="idle gap that starts a new group")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    rows = [r for r in rows if r[2] != "k_lds_server" and "rocclr" not in r[2]]
    groups, cur = [], []
    for r in rows:
        if cur and r[0] - max(x[1] for x in cur) > a.gap_us * 1e3:
            groups.append(cur)
            cur = []
        cur.append(r)
    if cur:
        groups.append(cur)
    # keep groups that ran a grid level (a real topdown, not a no-op)
    work = [g for g in groups if any("topdown" in x[2] and x[1] - x[0] > 4000 for x in g)]
    per = {}
    for g in work:
        for st, en, nm, wg in g:
            per.setdefault(nm, []).append((en - st) / 1e3)
    print(f"groups {len(groups)}, with a grid level {len(work)}")
    for nm, v in sorted(per.items(), key=lambda kv: -statistics.median(kv[1]) * len(kv[1])):
        print(f"  {nm:26s} x{len(v):4d} median {statistics.median(v):8.2f} us  mean {statistics.mean(v):8.2f}")
    spans = [(max(x[1] for x in g) - min(x[0] for x in g)) / 1e3 for g in work]
    if spans:
        print(f"  group span median {statistics.median(spans):.2f} us")
    for g in work[1:1 + a.queries]:
        t0 = g[0][0]
        print("--- start(us) dur(us) wgs kernel")
        prev = None
        for st, en, nm, wg in g:
            gap = "" if prev is None else f" gap {(st - prev) / 1e3:6.2f}"
            print(f"  {(st - t0) / 1e3:8.2f} {(en - st) / 1e3:7.2f} {wg:5d} {nm}{gap}")
            prev = en


if __name__ == "__main__":
    main()
