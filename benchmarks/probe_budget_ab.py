"""Resident queries on hub graphs at several LDS meet-probe budgets
(HipEngine.lds_probe_edges: frontier edges the probe may read before a
search hands off to grid levels), interleaved in blocks over the same pairs.
One JSON line per graph: mean / median query per budget.

    python benchmarks/probe_budget_ab.py --graphs kron:22:16:1 --budgets 16384,32768,65536
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: F401

from bench import generate, parse_spec, pick_pairs  # noqa: E402
from bidirectional_bfs_amd.ops import HipEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default="kron:22:16:1,kron:20:16:1,kron:25:16:1")
    ap.add_argument("--budgets", default="16384,32768,65536,131072")
    ap.add_argument("--queries", type=int, default=1024)
    ap.add_argument("--blocks", type=int, default=8)
    a = ap.parse_args()
    budgets = [int(x) for x in a.budgets.split(",")]
    for spec in a.graphs.split(","):
        _, n, _, _ = parse_spec(spec)
        eng = generate(HipEngine(0), spec)
        pairs = pick_pairs(eng, n, 64, 12345)
        eng.set_resident(True)
        t = {b: [] for b in budgets}
        per = a.queries // a.blocks
        for b in budgets:  # warm every budget's server build
            eng.lds_probe_edges = b
            for s, d, _ in pairs:
                eng.query(s, d)
        for blk in range(a.blocks):
            for b in budgets:
                eng.lds_probe_edges = b
                eng.query(*pairs[0][:2])  # (a budget change relaunches the server)
                for i in range(per):
                    s, d, h = pairs[(blk * per + i) % len(pairs)]
                    t0 = time.perf_counter()
                    hh, _ = eng.query(s, d)
                    t[b].append(time.perf_counter() - t0)
                    assert hh == h
        eng.set_resident(False)
        out = {"graph": spec, "queries_each": per * a.blocks}
        for b, v in t.items():
            out[f"b{b}_mean_us"] = round(statistics.mean(v) * 1e6, 3)
            out[f"b{b}_median_us"] = round(statistics.median(v) * 1e6, 3)
        print(json.dumps(out), flush=True)
        eng.release()


if __name__ == "__main__":
    main()
