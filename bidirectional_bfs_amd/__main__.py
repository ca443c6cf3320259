"""python -m bidirectional_bfs_amd <graph.bin|spec> <src> <dst> [--engine serial|hip] [--repeat R] [--json] [--verify]

Python front-end with the reference's positional argv.  ``--engine serial``
is v1, ``hip`` is v3 (single MI355X).  The MPI tiers are the native tools
(``build/bin/second_try``, ``mpi_queue_bibfs``, ``mpi_bibfs``) launched with
mpiexec; see ``bidirectional_bfs_amd.parallel.run_mpi``.
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m bidirectional_bfs_amd")
    ap.add_argument("graph")
    ap.add_argument("src", type=int)
    ap.add_argument("dst", type=int)
    ap.add_argument("--engine", choices=["serial", "hip"], default="hip")
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--verify", action="store_true")
    ap.add_argument("--side", choices=["edges", "frontier", "alternate"], default="edges")
    ap.add_argument("--direction", choices=["auto", "topdown", "bottomup"], default="auto")
    ap.add_argument("--force-grid", action="store_true")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    if a.engine == "hip":
        import torch  # noqa: F401  (one HIP runtime per process: torch's)
    from . import SerialEngine, native
    from .models import from_spec
    from .ops import HipEngine, make_options

    t0 = time.perf_counter()
    g = from_spec(a.graph)
    load_ms = (time.perf_counter() - t0) * 1e3
    if not (0 <= a.src < g.n and 0 <= a.dst < g.n):
        print(f"src/dst must be < N = {g.n}", file=sys.stderr)
        return 1
    opt = make_options(side=a.side, direction=a.direction, force_grid=a.force_grid)
    if a.engine == "serial":
        eng = SerialEngine(g)
        build_ms = 0.0
    else:
        eng = HipEngine(a.device).load(g)
        build_ms = eng.build_ms
        eng.search(a.src, a.dst, opt)  # warm-up
    rs = [eng.search(a.src, a.dst, opt) for _ in range(max(1, a.repeat))]
    r = rs[-1]
    med = statistics.median(x.total_ms for x in rs)
    if a.json:
        print(json.dumps({"engine": a.engine, "graph": a.graph, "n": g.n, "m": g.m, "src": a.src, "dst": a.dst,
                          "found": r.found, "hops": r.hops, "query_ms": med, "load_ms": load_ms,
                          "build_ms": build_ms, "gteps": g.m / (med * 1e-3) / 1e9 if med > 0 else None,
                          "stats": {k: v for k, v in r.stats.items() if k != "trace"}}))
    else:
        if r.found:
            print(f"Shortest path length = {r.hops}")
            print("Path: " + " ".join(map(str, r.path)))
        else:
            print(f"No path found between {a.src} and {a.dst}")
        print(f"[Time] {a.engine} bi-BFS query = {med * 1e-3:.9g} s")
    if a.verify:
        o = native.bfs_oracle(g.csr, a.src, a.dst)
        ok = o.hops == r.hops and (not r.found or native.validate_path(g.csr, a.src, a.dst, r.hops, r.path)[0])
        print(f"Verify: {'OK' if ok else 'MISMATCH'} (oracle hops = {o.hops})")
        return 0 if ok else 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
