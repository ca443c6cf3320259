"""Resident LDS-server queries with the device hand-off (a grid level and a
cleanup enqueued behind every query, HipEngine.auto_handoff) on vs off,
interleaved in blocks, same graph and pairs.  One JSON line per graph.

    python benchmarks/auto_handoff_ab.py --graphs kron:22:16:1,gnp:10000000::1
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
    ap.add_argument("--graphs", default="kron:22:16:1,gnp:10000000::1")
    ap.add_argument("--queries", type=int, default=1200)
    ap.add_argument("--blocks", type=int, default=12)
    a = ap.parse_args()
    for spec in a.graphs.split(","):
        _, n, _, _ = parse_spec(spec)
        eng = generate(HipEngine(0), spec)
        pairs = pick_pairs(eng, n, 64, 12345)
        eng.set_resident(True)
        t = {True: [], False: []}
        per = a.queries // a.blocks
        for on in (True, False):
            eng.auto_handoff = on
            for s, d, _ in pairs:
                eng.query(s, d)
        for b in range(a.blocks):
            for on in (True, False):
                eng.auto_handoff = on
                for i in range(per):
                    s, d, h = pairs[(b * per + i) % len(pairs)]
                    t0 = time.perf_counter()
                    hh, _ = eng.query(s, d)
                    t[on].append(time.perf_counter() - t0)
                    assert hh == h
        eng.set_resident(False)
        out = {"graph": spec, "queries_each": per * a.blocks}
        for on, v in t.items():
            k = "auto_on" if on else "auto_off"
            out[k + "_mean_us"] = round(statistics.mean(v) * 1e6, 3)
            out[k + "_median_us"] = round(statistics.median(v) * 1e6, 3)
        print(json.dumps(out), flush=True)
        eng.release()


if __name__ == "__main__":
    main()
