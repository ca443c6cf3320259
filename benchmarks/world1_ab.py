"""World size 1: the partitioned engine's query (DistEngine.query, which hands
the search to its adopted single-GPU engine) against the single-GPU engine's
own query (HipEngine.query), on the same graph and pairs, interleaved in
blocks so drift hits both alike.  Prints one JSON line per graph: per-engine
median / mean query time and the ratio (>= 0.95).

    python benchmarks/world1_ab.py --specs gnp:1000000::2,kron:22:16:1 --steps 200
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: F401  (binds the HIP runtime first)

from bench import generate, pick_pairs  # noqa: E402
from bidirectional_bfs_amd.ops import HipEngine  # noqa: E402
from bidirectional_bfs_amd.parallel import DistEngine  # noqa: E402


def timed(fn, pairs, steps, off):
    ts = []
    for i in range(steps):
        s, d, h = pairs[(off + i) % len(pairs)]
        t0 = time.perf_counter()
        hh, _ = fn(s, d)
        ts.append(time.perf_counter() - t0)
        assert hh == h, (s, d, hh, h)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", default="gnp:1000000::2,kron:22:16:1")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--blocks", type=int, default=4)
    ap.add_argument("--pairs", type=int, default=25)
    a = ap.parse_args()
    for spec in a.specs.split(","):
        n = int(spec.split(":")[1]) if not spec.startswith("kron") else 1 << int(spec.split(":")[1])
        ref = generate(HipEngine(0), spec)
        pairs = pick_pairs(ref, n, a.pairs, 12345)
        ref.set_resident(True)
        de = DistEngine(0, 1, 0, b"", "rccl")  # world size 1, as bench.py's partitioned entries
        de.set_tuning()
        generate(de, spec)
        for f in (ref.query, de.query):  # warm both servers
            timed(f, pairs, 10, 0)
        t_single, t_dist = [], []
        for b in range(a.blocks):
            t_single += timed(ref.query, pairs, a.steps // a.blocks, b)
            t_dist += timed(de.query, pairs, a.steps // a.blocks, b)
        ms = lambda v: round(1e3 * v, 5)  # noqa: E731
        out = {"spec": spec, "steps": len(t_single),
               "single_median_ms": ms(statistics.median(t_single)), "single_mean_ms": ms(statistics.mean(t_single)),
               "dist_median_ms": ms(statistics.median(t_dist)), "dist_mean_ms": ms(statistics.mean(t_dist)),
               "speedup_median": round(statistics.median(t_single) / statistics.median(t_dist), 4),
               "speedup_mean": round(statistics.mean(t_single) / statistics.mean(t_dist), 4)}
        print(json.dumps(out), flush=True)
        ref.set_resident(False)
        ref.release()
        de.release()


if __name__ == "__main__":
    main()
