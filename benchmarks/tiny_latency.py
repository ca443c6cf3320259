#!/usr/bin/env python3
"""End-to-end latency of one shortest-path query through the serving API
(``HipEngine.query``: host call -> resident server -> hops + path as a Python
list), against this repo's -O3 serial CPU engine through the same Python
call shape (``SerialBiBfs.query``), on the bench's graph and pairs.

    python benchmarks/tiny_latency.py [--graph gnp:100000::6] [--pairs 64] [--reps 50]

One JSON line per engine: mean / median host-side query time and the mean
device time (request seen -> answer written, s_memrealtime).  With
BIBFS_NO_TINY=1 the same run measures the general resident server.
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graph", default="gnp:100000::6")
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--per-pair", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime first)

    import bench
    from bidirectional_bfs_amd import native
    from bidirectional_bfs_amd.ops import HipEngine

    kind, n, arg, seed = bench.parse_spec(a.graph)
    eng = bench.generate(HipEngine(0), a.graph)
    eng.set_resident(True)
    pairs = bench.pick_pairs(eng, n, a.pairs, 12345)
    for s, d, h in pairs[:8]:
        eng.query(s, d)
    per = {p: [] for p in range(len(pairs))}
    dev = []
    t_all = []
    for r in range(a.reps):
        for i, (s, d, h) in enumerate(pairs):
            t0 = time.perf_counter()
            hh, path = eng.query(s, d)
            t1 = time.perf_counter()
            assert hh == h and len(path) == h + 1 and path[0] == s and path[-1] == d, (s, d, hh, h)
            t_all.append(t1 - t0)
            per[i].append(t1 - t0)
            dev.append(eng.last_search_ms)
    gpu = {"engine": "tiny" if eng.tiny_engine and not os.environ.get("BIBFS_NO_TINY") else "lds_server",
           "graph": a.graph, "queries": len(t_all),
           "query_us_mean": round(statistics.fmean(t_all) * 1e6, 3),
           "query_us_median": round(statistics.median(t_all) * 1e6, 3),
           "device_us_mean": round(statistics.fmean(dev) * 1e3, 3),
           "tiny_overflows": eng.tiny_overflows}
    print(json.dumps(gpu), flush=True)
    if a.per_pair:
        for i, (s, d, h) in enumerate(pairs):
            print(json.dumps({"src": s, "dst": d, "hops": h,
                              "query_us_median": round(statistics.median(per[i]) * 1e6, 2)}), flush=True)
    eng.set_resident(False)
    eng.release()

    el = native.gen_gnp(n, arg, seed) if kind == "gnp" else native.gen_rmat(n, int(arg), seed, 0.57, 0.19, 0.19)
    cpu = native.SerialBiBfs(native.build_csr(el))
    for s, d, h in pairs[:8]:
        cpu.query(s, d)
    t_all = []
    for r in range(a.reps):
        for s, d, h in pairs:
            t0 = time.perf_counter()
            hh, path = cpu.query(s, d)
            t1 = time.perf_counter()
            assert hh == h and len(path) == h + 1
            t_all.append(t1 - t0)
    print(json.dumps({"engine": "cpu_serial", "graph": a.graph, "queries": len(t_all),
                      "query_us_mean": round(statistics.fmean(t_all) * 1e6, 3),
                      "query_us_median": round(statistics.median(t_all) * 1e6, 3)}), flush=True)


if __name__ == "__main__":
    main()
