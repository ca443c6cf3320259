#!/usr/bin/env python3
"""Per-pair device search time of the resident server on the bench's 100k
pairs (bench.py pick_pairs), median over repeats, with levels and edges.
Shows which queries dominate the headline mean.

    python benchmarks/pair_latency.py [--graph gnp:100000::6] [--pairs 64] [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="gnp:100000::6")
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--summary", default=None, help="print only one aggregate line, tagged with this label")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)
    import bench
    from bidirectional_bfs_amd.ops import HipEngine

    _, n, _, _ = bench.parse_spec(a.graph)
    eng = bench.generate(HipEngine(0), a.graph)
    eng.set_resident(True)
    pairs = bench.pick_pairs(eng, n, a.pairs, 12345)
    agg = []
    for s, d, h in pairs:
        dev, tot, lds, walk = [], [], [], []
        for _ in range(a.reps):
            r = eng.search(s, d)
            assert r.hops == h
            dev.append(r.search_ms)
            tot.append(r.total_ms)
            lds.append(r.stats["lds_ms"])
            walk.append(r.stats["walk_ms"])
            probe = (r.stats["probe_edges"], r.stats["probe_hit"])
        rec = {"src": s, "dst": d, "hops": h, "search_us": round(statistics.median(dev) * 1e3, 2),
               "query_us": round(statistics.median(tot) * 1e3, 2), "levels": r.levels,
               "edges": r.edges_inspected, "visited": r.visited, "handoff": r.handoff,
               "grid_levels": r.stats["grid_levels"], "lds_us": round(statistics.median(lds) * 1e3, 2),
               "lds_levels": r.stats["lds_levels"], "walk_us": round(statistics.median(walk) * 1e3, 2),
               "probe_edges": probe[0], "probe_hit": probe[1]}
        agg.append(rec)
        if a.summary is None:
            print(json.dumps(rec), flush=True)
    if a.summary is not None:
        print(json.dumps({"label": a.summary, "graph": a.graph, "pairs": len(agg), "reps": a.reps,
                          "search_us_mean": round(statistics.mean(x["search_us"] for x in agg), 2),
                          "query_us_mean": round(statistics.mean(x["query_us"] for x in agg), 2),
                          "handoff_fraction": round(statistics.mean(float(x["handoff"]) for x in agg), 3),
                          "grid_levels_mean": round(statistics.mean(x["grid_levels"] for x in agg), 2),
                          "lds_us_mean": round(statistics.mean(x["lds_us"] for x in agg), 2),
                          "lds_levels_mean": round(statistics.mean(x["lds_levels"] for x in agg), 2),
                          "levels_mean": round(statistics.mean(x["levels"] for x in agg), 2),
                          "handoff_lds_us_mean": round(statistics.mean(
                              [x["lds_us"] for x in agg if x["handoff"]] or [0.0]), 2),
                          "handoff_search_us_mean": round(statistics.mean(
                              [x["search_us"] for x in agg if x["handoff"]] or [0.0]), 2),
                          "handoff_walk_us_mean": round(statistics.mean(
                              [x["walk_us"] for x in agg if x["handoff"]] or [0.0]), 2),
                          "probe_hit_fraction": round(statistics.mean(float(x["probe_hit"]) for x in agg), 3),
                          "probe_edges_mean": round(statistics.mean(x["probe_edges"] for x in agg), 1),
                          "probe_hit_search_us_mean": round(statistics.mean(
                              [x["search_us"] for x in agg if x["probe_hit"]] or [0.0]), 2),
                          "probe_hit_lds_us_mean": round(statistics.mean(
                              [x["lds_us"] for x in agg if x["probe_hit"]] or [0.0]), 2)}),
              flush=True)
    eng.set_resident(False)


if __name__ == "__main__":
    main()
