#!/usr/bin/env python3
"""Resident-server stress: many back-to-back queries per graph, every answer's
hop count checked against this repo's CPU engine and every 16th path validated
edge by edge (both state sets, hand-offs, grid levels, cleanups in flight).

    python benchmarks/stress_resident.py [--graphs gnp:3000000::4,kron:20:16:2] [--queries 4000]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", default="gnp:3000000::4,gnp:10000000::1,kron:20:16:2,kron:22:16:1,gnp:100000::6")
    ap.add_argument("--queries", type=int, default=4000)
    ap.add_argument("--pairs", type=int, default=200)
    a = ap.parse_args()
    import torch  # noqa: F401
    import bidirectional_bfs_amd as bb
    from bidirectional_bfs_amd import native
    from bidirectional_bfs_amd.ops import HipEngine

    for spec in a.graphs.split(","):
        g = bb.from_spec(spec)
        cpu = native.SerialBiBfs(g.csr)
        rnd = random.Random(11)
        pairs = [(rnd.randrange(g.n), rnd.randrange(g.n)) for _ in range(a.pairs)]
        truth = [cpu.query(s, d)[0] for s, d in pairs]
        eng = HipEngine(0)
        eng.load(g)
        eng.set_resident(True)
        bad = checked = handed = 0
        t0 = time.perf_counter()
        for i in range(a.queries):
            s, d = pairs[i % len(pairs)]
            h = truth[i % len(pairs)]
            if i % 3 == 0:
                hops, path = eng.query(s, d)
            else:
                r = eng.search(s, d)
                hops, path = r.hops, r.path
                handed += bool(r.handoff)
            if hops != h:
                bad += 1
            elif i % 16 == 0 and h > 0:
                ok, why = native.validate_path(g.csr, s, d, hops, list(path))
                checked += 1
                bad += 0 if ok else 1
        dt = time.perf_counter() - t0
        eng.set_resident(False)
        eng.release()
        print(json.dumps({"graph": spec, "queries": a.queries, "wrong": bad, "paths_validated": checked,
                          "handoffs": handed, "mean_query_us": round(dt / a.queries * 1e6, 2)}), flush=True)
        if bad:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
