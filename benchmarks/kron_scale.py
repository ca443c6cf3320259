#!/usr/bin/env python3
"""Single-GPU Kronecker / R-MAT sweep (BASELINE.json configs 4-5 on one MI355X).

    python benchmarks/kron_scale.py [--scales 20,22,24,26,27] [--queries 16] [--ef 16]

For each scale: generate the Graph500-parameter R-MAT edge list on the GPU
(a = 0.57, b = c = 0.19, scrambled labels), build the CSR on the GPU (64-bit
offsets beyond 2^32 entries), then answer `queries` seeded random
connected pairs with the direction-optimizing engine (LDS engine -> hand-off
to the grid top-down / bottom-up kernels).  One JSON line per scale:
build ms, per-query ms (median, mean), GTEPS(M/t) = M / median query time,
edges actually inspected, grid / bottom-up level counts, HBM held.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bidirectional_bfs_amd.ops import HipEngine, make_options  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--scales", default="20,22,24,26,27")
    ap.add_argument("--ef", type=int, default=16)
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--direction", default="auto", choices=["auto", "topdown", "bottomup"])
    ap.add_argument("--alpha", type=float, default=14.0, help="Beamer top-down -> bottom-up: m_f > m_u / alpha")
    ap.add_argument("--beta", type=float, default=24.0, help="Beamer bottom-up -> top-down: n_f < n / beta")
    ap.add_argument("--force-grid", action="store_true", help="skip the LDS engine: every level on the grid engine")
    ap.add_argument("--resident", action="store_true", help="serve the queries through the resident server")
    a = ap.parse_args()
    eng = HipEngine(a.device)
    opt = make_options(direction=a.direction, alpha=a.alpha, beta=a.beta, force_grid=a.force_grid)
    for scale in [int(x) for x in a.scales.split(",") if x]:
        n, m = 1 << scale, a.ef << scale
        t0 = time.perf_counter()
        eng.generate_rmat(n, m, a.seed)
        build_wall = (time.perf_counter() - t0) * 1e3
        eng.set_resident(a.resident)
        rnd = random.Random(scale)
        pairs, tries = [], 0
        while len(pairs) < a.queries + 2 and tries < 50 * a.queries:
            s, d = rnd.randrange(n), rnd.randrange(n)
            tries += 1
            r = eng.search(s, d, opt)
            if r.found and r.hops > 0:
                pairs.append((s, d))
        times, insp, hops, grid, bu = [], 0, 0, 0, 0
        for s, d in pairs[2:]:  # the first two double as warm-up
            t = time.perf_counter()
            r = eng.search(s, d, opt)
            times.append((time.perf_counter() - t) * 1e3)
            assert r.found and len(r.path) == r.hops + 1
            st = r.stats
            insp += st["edges_inspected"]
            hops += r.hops
            grid += st["grid_levels"]
            bu += st["bottomup_levels"]
        k = max(1, len(times))
        med = statistics.median(times) if times else float("nan")
        print(json.dumps({
            "graph": f"kron:{scale}:{a.ef}:{a.seed}", "n": n, "m": m, "nnz": eng.nnz,
            "device_build_ms": round(eng.build_ms, 3), "build_wall_ms": round(build_wall, 3),
            "queries": len(times), "median_query_ms": round(med, 4), "mean_query_ms": round(sum(times) / k, 4),
            "gteps": round(m / (med * 1e-3) / 1e9, 3), "mean_edges_inspected": insp // k,
            "gteps_inspected": round(insp / k / (med * 1e-3) / 1e9, 3), "mean_hops": hops / k,
            "mean_grid_levels": grid / k, "mean_bottomup_levels": bu / k,
            "device_gb": round(eng.device_bytes / 1e9, 2), "direction": a.direction,
            "alpha": a.alpha, "beta": a.beta, "force_grid": a.force_grid, "resident": a.resident,
        }), flush=True)
        eng.set_resident(False)
        eng.release()
    return 0


if __name__ == "__main__":
    sys.exit(main())
