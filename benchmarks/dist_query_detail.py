#!/usr/bin/env python3
"""Per-query detail of the partitioned engine at world size 1 over RCCL: time,
rounds, host-planned rounds, dense (bottom-up) levels and exchanged bytes for
every query, under several direction policies -- to see which queries make
the mean exceed the median (Kronecker graphs).

    python benchmarks/dist_query_detail.py --spec kron:27 --queries 16 --directions auto,topdown
"""
import argparse
import json
import statistics
import sys
import time

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import bench  # noqa: E402
from bidirectional_bfs_amd.ops import HipEngine, make_options  # noqa: E402
from bidirectional_bfs_amd.parallel import DistEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="kron:27")
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--directions", default="auto,topdown")
    ap.add_argument("--alpha", default="14")
    ap.add_argument("--pair", help="s,d: run only this pair (e.g. under rocprofv3)")
    a = ap.parse_args()
    _, n, _, _ = bench.parse_spec(a.spec)
    ref = bench.generate(HipEngine(0), a.spec)
    pairs = bench.pick_pairs(ref, n, a.queries, 12345)
    if a.pair:
        s0, d0 = (int(x) for x in a.pair.split(","))
        pairs = [(s0, d0, ref.search(s0, d0).hops)] * 4
    ref.release()
    del ref
    eng = DistEngine(0, 1, 0, DistEngine.unique_id())
    bench.generate(eng, a.spec)
    for direction in a.directions.split(","):
        for alpha in [float(x) for x in a.alpha.split(",")]:
            opt = make_options(direction=direction, alpha=alpha)
            for s, d, _ in pairs[:3]:
                eng.search(s, d, opt)
            rows = []
            for s, d, h in pairs:
                t0 = time.perf_counter()
                r = eng.search(s, d, opt)
                ms = (time.perf_counter() - t0) * 1e3
                assert r.found and r.hops == h, (s, d, r.hops, h)
                st = eng.last_stats
                rows.append({"src": s, "dst": d, "hops": h, "ms": round(ms, 4), "rounds": st["rounds"],
                             "host_rounds": st["host_rounds"], "dense_levels": st["dense_levels"],
                             "spec_rounds": st["spec_rounds"], "kb": round(st["exchanged_bytes"] / 1024, 1)})
            ms = [x["ms"] for x in rows]
            print(json.dumps({"spec": a.spec, "direction": direction, "alpha": alpha,
                              "median_ms": round(statistics.median(ms), 4), "mean_ms": round(statistics.mean(ms), 4),
                              "slowest": sorted(rows, key=lambda x: -x["ms"])[:4]}), flush=True)
    eng.release()


if __name__ == "__main__":
    main()
