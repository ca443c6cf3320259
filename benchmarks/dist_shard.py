#!/usr/bin/env python3
"""CSR-sharded partitioned engine rehearsed on ONE GPU (BASELINE.json config 5:
a scale-27 Kronecker graph sharded over ranks).

P ranks run as threads of this process, each a DistBiBfs over its own 1-D
vertex block (csrc/dist/dist_engine.hip), exchanging through the in-process
local group instead of RCCL.  Every rank generates the graph on the device and
keeps only its block's CSR rows -- the same path `bench.py --mode partitioned`
takes on a multi-GPU node.  The ranks share one GPU, so query times here
include P-fold contention and no xGMI; the point is that sharding, build and
search work at full scale and answer correctly (ranks must agree).

    python benchmarks/dist_shard.py --specs kron:27 --ranks 2,4 --queries 16 --out profiles/x.jsonl
"""
import argparse
import json
import random
import statistics
import sys
import time

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from bidirectional_bfs_amd.models import parse_spec  # noqa: E402
from bidirectional_bfs_amd.parallel import dist_local_generate_run  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", default="kron:22,kron:27")
    ap.add_argument("--ranks", default="2,4")
    ap.add_argument("--queries", type=int, default=48)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out")
    a = ap.parse_args()
    out = open(a.out, "a") if a.out else None
    for spec in a.specs.split(","):
        _, n, _, _ = parse_spec(spec)
        rnd = random.Random(a.seed)
        qs = [(rnd.randrange(n), rnd.randrange(n)) for _ in range(a.queries)]
        for ranks in [int(x) for x in a.ranks.split(",")]:
            t0 = time.perf_counter()
            rs, t = dist_local_generate_run(ranks, spec, qs)
            wall = time.perf_counter() - t0
            found = [(r, ms, st) for r, ms, st in zip(rs, t["query_ms"], t["stats"]) if r.found and r.hops > 0]
            qms = [ms for _, ms, _ in found]
            rec = {
                "spec": spec, "n": n, "ranks": ranks, "queries": len(qs), "found": len(found),
                "build_ms": round(t["build_ms"], 3), "wall_s": round(wall, 3),
                "median_query_ms": round(statistics.median(qms), 4) if qms else None,
                "mean_hops": round(statistics.mean(r.hops for r, _, _ in found), 3) if found else None,
                "mean_rounds": round(statistics.mean(st["rounds"] for _, _, st in found), 3) if found else None,
                "median_round_ms": round(statistics.median(ms / max(1, st["rounds"]) for _, ms, st in found), 4)
                if found else None,
                "mean_exchanged_bytes": round(statistics.mean(st["exchanged_bytes"] for _, _, st in found)) if found else None,
                "dense_levels": sum(st["dense_levels"] for _, _, st in found),
                "local_nnz": t["local_nnz"], "max_shard_fraction": round(max(t["local_nnz"]) / max(1, sum(t["local_nnz"])), 4),
            }
            line = json.dumps(rec)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()


if __name__ == "__main__":
    main()
