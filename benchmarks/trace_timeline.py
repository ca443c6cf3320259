#!/usr/bin/env python3
"""Print per-query kernel timelines from a rocprofv3 run database (rocpd
SQLite, `rocprofv3 --kernel-trace -d DIR -o run`): each query starts at a
kernel whose name contains --start (default: the partitioned engine's k_seed).

    python benchmarks/trace_timeline.py gpurun_out/prof/run_results.db --queries 3,20
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--start", default="k_seed(bibfs::(anonymous namespace)::DView")
    ap.add_argument("--queries", default="3")
    ap.add_argument("--stats", action="store_true", help="per-kernel totals instead")
    a = ap.parse_args()
    cur = sqlite3.connect(a.db).cursor()
    if a.stats:
        for name, cnt, avg, tot in cur.execute(
                "select name, count(*), avg(end-start), sum(end-start) from kernels group by name "
                "order by sum(end-start) desc limit 30"):
            print(f"{cnt:7d} {avg / 1000:9.2f} us {tot / 1e6:9.3f} ms  {name[:90]}")
        return
    rows = cur.execute("select name, start, end, grid_x, workgroup_x, grid_y from kernels order by start").fetchall()
    idx = [i for i, r in enumerate(rows) if a.start in r[0]]
    for q in (int(x) for x in a.queries.split(",")):
        if q >= len(idx):
            continue
        i0 = idx[q]
        i1 = idx[q + 1] if q + 1 < len(idx) else len(rows)
        t0 = rows[i0][1]
        print(f"--- query {q}: start(us) dur(us) grid name")
        for name, st, en, gx, wx, gy in rows[i0:i1]:
            print(f"{(st - t0) / 1000:8.2f} {(en - st) / 1000:7.2f} {gx // max(wx, 1):5d}x{gy} {name[:70]}")


if __name__ == "__main__":
    main()
