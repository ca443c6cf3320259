#!/usr/bin/env python3
"""Largest-graph rehearsal on ONE GPU: the same device-generated Kronecker
graph in the single-GPU engine (HipEngine) and in the partitioned engine at
world size 1 (DistEngine over a one-rank RCCL communicator), both resident at
once.  Every answer of both engines is checked edge by edge against the
device CSR (HipEngine.check_path: one row copied per hop) and the two
engines must agree on every hop count.

    python benchmarks/big_rehearsal.py --spec kron:29:16:1 --pairs 8

Prints one JSON line per engine (build time, HBM, per-query times) and a
verdict line.  Needs ~150 GB of HBM at scale 29 (two CSR copies of 17.2 G
directed edges).
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
    ap.add_argument("--spec", default="kron:29:16:1")
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import bench
    from bidirectional_bfs_amd.ops import HipEngine
    from bidirectional_bfs_amd.parallel import DistEngine

    kind, n, arg, seed = bench.parse_spec(a.spec)
    free0, total = torch.cuda.mem_get_info(0)
    t0 = time.perf_counter()
    eng = bench.generate(HipEngine(0), a.spec)
    build_s = time.perf_counter() - t0
    free1, _ = torch.cuda.mem_get_info(0)
    print(json.dumps({"engine": "HipEngine", "spec": a.spec, "n": eng.n, "nnz": eng.nnz,
                      "build_wall_s": round(build_s, 3), "device_build_ms": round(eng.build_ms, 3),
                      "hbm_bytes": free0 - free1, "device_bytes": eng.device_bytes}), flush=True)
    pairs = bench.pick_pairs(eng, n, a.pairs, 12345)
    assert pairs, "no connected pairs"
    single = {}
    for s, d, h in pairs:
        ts = []
        for _ in range(a.reps):
            q0 = time.perf_counter()
            r = eng.search(s, d)
            ts.append((time.perf_counter() - q0) * 1e3)
        assert r.found and r.hops == h and eng.check_path(s, d, h, r.path), ("HipEngine", s, d, h)
        single[(s, d)] = (h, statistics.median(ts), r.search_ms)

    free2, _ = torch.cuda.mem_get_info(0)
    t0 = time.perf_counter()
    de = bench.generate(DistEngine(0, 1, 0, DistEngine.unique_id()), a.spec)
    dbuild_s = time.perf_counter() - t0
    free3, _ = torch.cuda.mem_get_info(0)
    out = {"engine": "DistEngine(world 1)", "spec": a.spec, "build_wall_s": round(dbuild_s, 3),
           "hbm_bytes": free2 - free3, "shard_bytes": de.shard_bytes, "gen_peak_bytes": de.gen_peak_bytes,
           "hbm_total": total, "hbm_free_after_both": free3}
    print(json.dumps(out), flush=True)
    ok = True
    for s, d, h in pairs:
        ts = []
        for _ in range(a.reps):
            q0 = time.perf_counter()
            r = de.search(s, d)
            ts.append((time.perf_counter() - q0) * 1e3)
        good = r.found and r.hops == h and eng.check_path(s, d, h, r.path)
        ok &= good
        hs, ms_single, dev_single = single[(s, d)]
        print(json.dumps({"src": s, "dst": d, "hops": h, "single_gpu_query_ms": round(ms_single, 4),
                          "single_gpu_device_ms": round(dev_single, 4),
                          "partitioned_query_ms": round(statistics.median(ts), 4),
                          "partitioned_device_ms": round(r.search_ms, 4), "agree_and_valid": good}), flush=True)
    print(json.dumps({"spec": a.spec, "pairs": len(pairs), "verified": ok}), flush=True)
    de.release()
    eng.release()
    assert ok


if __name__ == "__main__":
    main()
