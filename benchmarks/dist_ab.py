#!/usr/bin/env python3
"""Partitioned engine at world size 1 over a real RCCL communicator: A/B of the
round-planning modes on the same graphs and connected pairs.

spec_rounds = 0 plans every round on the host (one host wait per round, the
first design); K > 0 enqueues K device-planned rounds per host wait.  Pairs and
their hop counts come from the single-GPU engine; every answer is checked.

    python benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 0,2,4,8 --queries 24

A mode "K:E" also sets the one-rank solo workgroup's edge cap (E = 0: solo off).
"""
import argparse
import json
import statistics
import sys
import time

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import bench  # noqa: E402
from bidirectional_bfs_amd.ops import HipEngine  # noqa: E402
from bidirectional_bfs_amd.parallel import DistEngine, make_tuning  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", default="gnp:1000000::2,kron:22")
    ap.add_argument("--modes", default="0,2,4,8")
    ap.add_argument("--queries", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out")
    ap.add_argument("--slow-ms", type=float, default=0.0, help="also print every query slower than this (stats)")
    a = ap.parse_args()
    out = open(a.out, "a") if a.out else None
    eng = DistEngine(0, 1, 0, DistEngine.unique_id())
    for spec in a.specs.split(","):
        _, n, _, _ = bench.parse_spec(spec)
        ref = bench.generate(HipEngine(0), spec)
        pairs = bench.pick_pairs(ref, n, a.queries, 12345)
        ref.release()
        del ref
        t0 = time.perf_counter()
        bench.generate(eng, spec)
        build_ms = (time.perf_counter() - t0) * 1e3
        for mode in a.modes.split(","):
            k, _, e = mode.partition(":")
            k = int(k)
            solo_e = int(e) if e else None
            if solo_e is None:
                eng.set_tuning(make_tuning(spec_rounds=k))
            else:
                eng.set_tuning(make_tuning(spec_rounds=k, solo=solo_e > 0, solo_edges=max(solo_e, 1)))
            for s, d, _ in pairs[:3]:
                eng.search(s, d)  # warm
            qms, dms, st = [], [], []
            for _ in range(a.reps):
                for s, d, h in pairs:
                    q0 = time.perf_counter()
                    r = eng.search(s, d)
                    qms.append((time.perf_counter() - q0) * 1e3)
                    assert r.found and r.hops == h and len(r.path) == h + 1, (spec, s, d, r.hops, h)
                    dms.append(r.search_ms)
                    st.append(eng.last_stats)
                    if a.slow_ms and qms[-1] > a.slow_ms:
                        x = dict(st[-1])
                        x.pop("trace", None)
                        print(json.dumps({"slow_query": [s, d, h], "ms": round(qms[-1], 4),
                                          "device_ms": round(r.search_ms, 4), "stats": x}), flush=True)
            rec = {
                "spec": spec, "n": n, "spec_rounds": k, "solo_edges": solo_e, "queries": len(qms),
                "build_ms": round(build_ms, 2),
                "median_query_ms": round(statistics.median(qms), 4), "mean_query_ms": round(statistics.mean(qms), 4),
                "median_device_ms": round(statistics.median(dms), 4),
                "mean_rounds": round(statistics.mean(x["rounds"] for x in st), 3),
                "mean_host_syncs": round(statistics.mean(x["host_syncs"] for x in st), 3),
                "mean_host_rounds": round(statistics.mean(x["host_rounds"] for x in st), 3),
                "mean_spec_rounds": round(statistics.mean(x["spec_rounds"] for x in st), 3),
                "mean_solo_rounds": round(statistics.mean(x["solo_rounds"] for x in st), 3),
                "mean_collectives": round(statistics.mean(x["collectives"] for x in st), 3),
                "mean_dense_levels": round(statistics.mean(x["dense_levels"] for x in st), 3),
                "mean_exchanged_kb": round(statistics.mean(x["exchanged_bytes"] for x in st) / 1024, 1),
            }
            line = json.dumps(rec)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()
        eng.release()


if __name__ == "__main__":
    main()
