#!/usr/bin/env python3
"""Clean counter workload for the 100k headline (the bench's query pattern):
G(n = 100000, p = 2.2/n) seed 6, the bench's 64 connected pairs rotated.

    --mode oneshot   one k_lds_bibfs dispatch per query (per-dispatch counters
                     = per-query counters)
    --mode resident  the resident server; the timed phase is ONE k_lds_server
                     dispatch serving --queries queries (its mailbox polls
                     between queries are included in its counters)
"""
import argparse
import os
import sys

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bidirectional_bfs_amd.ops import HipEngine  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--mode", choices=["oneshot", "resident"], default="oneshot")
ap.add_argument("--queries", type=int, default=256)
ap.add_argument("--graph", default="gnp:100000::6", help="any bench spec (e.g. gnp:10000000::1 for the LDS server)")
a = ap.parse_args()
eng = bench.generate(HipEngine(0), a.graph)
eng.set_resident(False)
_, n, _, _ = bench.parse_spec(a.graph)
pairs = bench.pick_pairs(eng, n, 64, 12345)
for i in range(128):  # warm: every pair twice
    s, d, _ = pairs[i % len(pairs)]
    eng.search(s, d)
eng.set_resident(a.mode == "resident")
for i in range(a.queries):
    s, d, h = pairs[i % len(pairs)]
    assert eng.search(s, d).hops == h
eng.set_resident(False)
print("pmc workload done", a.graph, a.mode, a.queries, flush=True)
