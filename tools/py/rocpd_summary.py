#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd SQLite database
(rocprofv3 --kernel-trace writes <name>_results.db): calls, total / mean /
min / max duration in microseconds, sorted by total time.

    python tools/py/rocpd_summary.py gpurun_out/prof_bench/bench_results.db [--csv out.csv]
"""
import argparse
import csv
import sqlite3
import sys


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    a = ap.parse_args(argv)
    c = sqlite3.connect(a.db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    disp = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    sym = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    cols = [r[1] for r in c.execute(f"pragma table_info({sym})")]
    name_col = "display_name" if "display_name" in cols else ("kernel_name" if "kernel_name" in cols else "name")
    q = (f"select s.{name_col}, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start), "
         f"max(d.end - d.start) from {disp} d join {sym} s on d.kernel_id = s.id group by s.{name_col} "
         f"order by sum(d.end - d.start) desc")
    rows = [(n, k, tot / 1e3, avg / 1e3, mn / 1e3, mx / 1e3) for n, k, tot, avg, mn, mx in c.execute(q)]
    w = csv.writer(open(a.csv, "w", newline="")) if a.csv else None
    hdr = ("kernel", "calls", "total_us", "mean_us", "min_us", "max_us")
    if w:
        w.writerow(hdr)
    print(f"{'calls':>7} {'total_us':>12} {'mean_us':>10} {'min_us':>10} {'max_us':>10}  kernel")
    for r in rows:
        if w:
            w.writerow([r[0], r[1]] + [f"{x:.3f}" for x in r[2:]])
        print(f"{r[1]:>7} {r[2]:>12.1f} {r[3]:>10.2f} {r[4]:>10.2f} {r[5]:>10.2f}  {r[0][:110]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
