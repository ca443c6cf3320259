"""Batched-serving throughput on one MI355X: K random connected queries per
`search_batch` call, swept over graph specs and the HBM-bitmap pass's edge cap.

    python benchmarks/batch_serving.py --spec gnp:10000000::1 --spec kron:22:16:1 \
        --batch 256 --caps 65536,262144,1048576 --out gpurun_out/batch_serving.jsonl

Each line: spec, cap, us/query, queries/s, and how the queries were answered
(LDS pass / HBM-bitmap pass / single-query fallback).  Graphs are generated on
the device (synthetic, seeded); answers are checked hop-for-hop against the
single-query engine for the first batch.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: F401,E402  (binds the HIP runtime first)

from bench import generate, parse_spec  # noqa: E402
from bidirectional_bfs_amd.ops import HipEngine  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", action="append", default=[])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--caps", default="1048576")
    ap.add_argument("--tunings", default="-1:0", help="lds_first:threads pairs, comma-separated")
    ap.add_argument("--seed", type=int, default=11)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    specs = a.spec or ["gnp:10000000::1", "kron:22:16:1"]
    eng = HipEngine(0)
    lines = []
    for spec in specs:
        _, n, _, _ = parse_spec(spec)
        generate(eng, spec)
        rng = random.Random(a.seed)
        pairs = []
        while len(pairs) < a.batch:
            s, d = rng.randrange(n), rng.randrange(n)
            r = eng.search(s, d)
            if r.found and r.hops > 0:
                pairs.append((s, d, r.hops))
        bs = [p[0] for p in pairs]
        bd = [p[1] for p in pairs]
        combos = [(int(c), tuple(int(x) for x in t.split(":"))) for c in a.caps.split(",")
                  for t in a.tunings.split(",")]
        for cap, (lds_first, threads) in combos:
            eng.batch_edge_cap = cap
            eng.set_batch_tuning(lds_first, threads)
            rs = eng.search_batch(list(zip(bs, bd)))
            bad = sum(1 for r, p in zip(rs, pairs) if r.hops != p[2])
            via_hbm = sum(1 for r in rs if r.handoff and r.search_ms == r.total_ms)
            lds = sum(1 for r in rs if not r.handoff)
            eng.search_batch_arrays(bs, bd)
            t0 = time.perf_counter()
            for _ in range(a.reps):
                eng.search_batch_arrays(bs, bd)
            dt = time.perf_counter() - t0
            line = {"spec": spec, "n": n, "m": eng.m, "batch": a.batch, "edge_cap": cap,
                    "lds_first": lds_first, "threads": threads,
                    "us_per_query": dt * 1e6 / (a.reps * a.batch), "queries_per_s": a.reps * a.batch / dt,
                    "lds_pass": lds, "hbm_or_fallback": a.batch - lds, "hbm_pass_est": via_hbm,
                    "mean_hops": sum(p[2] for p in pairs) / len(pairs), "wrong": bad}
            print(json.dumps(line), flush=True)
            lines.append(line)
            assert bad == 0, f"{bad} wrong answers for {spec} cap {cap}"
    if a.out:
        with open(a.out, "a") as f:
            for line in lines:
                f.write(json.dumps(line) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
