#!/usr/bin/env python3
"""Hop counts of the resident server (LDS engine, meet probe, hand-offs)
against the grid-only engine (force_grid) on the same graph, many random
pairs back to back -- a GPU-only cross-check for graphs too large for a
host oracle (Kronecker 27: 4.3B directed edges).  One JSON line.

    python benchmarks/crosscheck.py --graph kron:27:16:1 --pairs 400
"""
import argparse
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="kron:27:16:1")
    ap.add_argument("--pairs", type=int, default=400)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--resident", type=int, default=1)
    ap.add_argument("--probe", type=int, default=-1, help="lds_probe_edges (-1: the default)")
    a = ap.parse_args()
    import torch  # noqa: F401
    import bench
    from bidirectional_bfs_amd.ops import HipEngine, make_options

    _, n, _, _ = bench.parse_spec(a.graph)
    eng = bench.generate(HipEngine(0), a.graph)
    rnd = random.Random(a.seed)
    pairs = [(rnd.randrange(n), rnd.randrange(n)) for _ in range(a.pairs)]
    if a.probe >= 0:
        eng.lds_probe_edges = a.probe
    eng.set_resident(bool(a.resident))
    res, info = [], []
    hits = hand = 0
    for s, d in pairs:
        r = eng.search(s, d)
        res.append(r.hops)
        info.append((bool(r.stats["probe_hit"]), bool(r.handoff), r.stats["lds_levels"], r.stats["grid_levels"]))
        hits += bool(r.stats["probe_hit"])
        hand += bool(r.handoff)
        assert r.hops < 0 or (len(r.path) == r.hops + 1 and r.path[0] == s and r.path[-1] == d)
    eng.set_resident(False)
    grid = make_options(force_grid=True)
    wrong = []
    for (s, d), h, inf in zip(pairs, res, info):
        g = eng.search(s, d, grid).hops
        if g != h:
            wrong.append((s, d, h, g) + inf)
    print(json.dumps({"graph": a.graph, "resident": a.resident, "probe": eng.lds_probe_edges, "pairs": len(pairs), "probe_hits": hits, "handoffs": hand,
                      "wrong": len(wrong), "examples": wrong[:5]}), flush=True)
    return 1 if wrong else 0


if __name__ == "__main__":
    sys.exit(main())
