#!/usr/bin/env python3
"""Chained auto grid levels on a hub graph, one search at a time with its
outcome (debug aid for the auto chain: run with BIBFS_DEBUG=1).

    python benchmarks/auto_chain_repro.py [--graph kron:20:16:2] [--levels 1,2] [--pairs 8]
"""
import argparse
import faulthandler
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="kron:20:16:2")
    ap.add_argument("--levels", default="1,2")
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--max-degree", type=int, default=1 << 40)
    a = ap.parse_args()
    faulthandler.dump_traceback_later(50, exit=True)
    import torch  # noqa: F401
    import bidirectional_bfs_amd as bb
    from bidirectional_bfs_amd import native
    from bidirectional_bfs_amd.ops import HipEngine

    g = bb.from_spec(a.graph)
    eng = HipEngine(0)
    eng.load(g)
    import random
    rnd = random.Random(9)
    pairs = [(0, g.n - 1)] + [(rnd.randrange(g.n), rnd.randrange(g.n)) for _ in range(a.pairs)]
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    eng.set_resident(True)
    eng.auto_max_degree = a.max_degree
    for lv in [int(x) for x in a.levels.split(",")]:
        eng.auto_levels = lv
        for (s, d), h in zip(pairs, truth):
            t0 = time.perf_counter()
            r = eng.search(s, d)
            dt = time.perf_counter() - t0
            print(f"levels {lv} {s}->{d} hops {r.hops} (truth {h}) handoff {r.handoff} grid {r.stats['grid_levels']} "
                  f"{dt * 1e3:.3f} ms misses {eng.auto_gate_misses}", flush=True)
    eng.set_resident(False)


if __name__ == "__main__":
    main()
