#!/usr/bin/env python3
"""Headline benchmark: end-to-end shortest-path queries on the reference graph
shape, reported as GTEPS(M/t) (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--graph gnp:100000::6]
                    [--mode replicated|partitioned] [--extra-graph gnp:10000000::1,kron:22:16:1]
                    [--dist-graphs gnp:1000000::2,kron:22:16:1]

One step = one bidirectional-BFS query per GPU: host call -> search on the
MI355X -> hop count AND the full path back in host memory ("end-to-end ms to
shortest path").  Graph: G(n, p = 2.2/n) exactly like the reference suite
(graphs/make_graphs:8), generated on the device from a fixed seed (synthetic,
there is no dataset); queries are seeded random vertex pairs that are
connected (the first is (0, N-1) like benchmark_test.sh:43), fixed before
timing and rotated over every step, so no result is reused.

Modes (N > 1 is launched by torch.distributed.run, one rank per GPU):
  replicated  (default, weak scaling) every GPU holds the whole graph and
              answers its own queries -- production query serving;
  partitioned (strong scaling) the graph is 1-D partitioned over the GPUs and
              every query is one collective search over RCCL (v4 capability).

value = whole-job GTEPS = M * (queries answered by all GPUs) / max-rank wall
time; vs_baseline divides by the best published 100k number in BASELINE.md
(v1 serial: 0.116 ms -> 0.952 GTEPS(M/t)).

Secondary configs (BASELINE.json), reported under detail and never folded
into `value`: `extra` = the same serving loop on 10M-vertex G(n,p) and on a
scale-22 Kronecker (R-MAT, Graph500 parameters; the direction-optimizing grid
engine); with N > 1 GPUs, `partitioned` = the 1-D partitioned RCCL engine
(one collective search over all GPUs, strong scaling) on 1M G(n,p) (the v4
config) and on Kronecker scale 22.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import threading
import time

import torch  # first: the HIP runtime torch ships is the one our extension then binds to
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_100K_GTEPS = 110000 / (0.115546e-3) / 1e9  # v1 @ 100k, M ~ 1.1 (N - 1)
BASELINE_100K_MS = 0.115546


def parse_spec(spec: str):
    """gnp:N[:p[:seed]], rmat:N:M[:seed] or kron:SCALE[:EF[:seed]] -> (kind, n, arg, seed)."""
    f = spec.split(":")
    if f[0] == "gnp":
        n = int(f[1])
        return "gnp", n, (float(f[2]) if len(f) > 2 and f[2] else 2.2000000001 / n), (int(f[3]) if len(f) > 3 else 1)
    if f[0] == "rmat":
        return "rmat", int(f[1]), int(f[2]), (int(f[3]) if len(f) > 3 else 1)
    if f[0] == "kron":
        scale, ef = int(f[1]), (int(f[2]) if len(f) > 2 else 16)
        return "rmat", 1 << scale, ef << scale, (int(f[3]) if len(f) > 3 else 1)
    raise ValueError(f"bench graph spec must be gnp:/rmat:/kron:, got {spec!r}")


def generate(eng, spec: str):
    kind, n, arg, seed = parse_spec(spec)
    if kind == "gnp":
        eng.generate_gnp(n, arg, seed)
    else:
        eng.generate_rmat(n, arg, seed)
    return eng


def pick_pairs(eng, n: int, count: int, seed: int):
    """Seeded connected (src, dst) pairs; (0, N-1) first (benchmark_test.sh:43)."""
    rng = random.Random(seed)
    pairs, tries = [], 0
    cand = [(0, n - 1)]
    while len(pairs) < count and tries < 50 * count:
        s, d = cand.pop() if cand else (rng.randrange(n), rng.randrange(n))
        tries += 1
        r = eng.search(s, d)
        if r.found and r.hops > 0:
            pairs.append((s, d))
    return pairs


def report(a, world: int, head: dict, extra: dict, partitioned: dict) -> dict:
    """The one JSON line rank 0 prints (driver contract)."""
    return {
        "metric": "GTEPS(M/t), end-to-end bi-BFS shortest-path query (G(n,2.2/n), path returned to host)",
        "value": round(head["gteps"], 4),
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(head["ms_per_step"], 6),
        "higher_is_better": True,
        "scaling": "strong" if a.mode == "partitioned" else "weak",
        "vs_baseline": round(head["gteps"] / BASELINE_100K_GTEPS, 3) if head["n"] == 100000 else None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "model": f"G(n={head['n']}, p=2.2/n) seed={head['seed']}, M={head['m']}",
            "global_batch": world if a.mode == "replicated" else 1,
            "seq_len": head["n"],
            "parallelism": (f"dp{world}" if a.mode == "replicated" else f"vertex-partition{world}"),
        },
        "detail": {
            "query_ms": round(head["ms_per_step"], 6),
            "device_ms_per_query": round(head["device_ms_per_query"], 6),
            "baseline_best_100k_ms": BASELINE_100K_MS,
            "gteps_inspected": head["gteps_inspected"],
            "mean_hops": head["mean_hops"],
            "graph_build_ms": round(head["build_ms"], 3),
            "resident_server": a.mode == "replicated" and not a.no_resident,
            "batched_serving": head["batched"],
            "extra": extra,
            "partitioned": partitioned,
        },
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--graph", default="gnp:100000::6")
    ap.add_argument("--mode", choices=["replicated", "partitioned"], default="replicated")
    ap.add_argument("--extra-graph", default="gnp:10000000::1,kron:22:16:1",
                    help="comma-separated secondary configs reported under 'extra' (empty to skip)")
    ap.add_argument("--dist-graphs", default="gnp:1000000::2,kron:22:16:1",
                    help="N > 1 only: configs run through the partitioned RCCL engine (empty to skip)")
    ap.add_argument("--dist-steps", type=int, default=20)
    ap.add_argument("--secondary-timeout", type=float, default=240.0,
                    help="seconds allowed for the extra + partitioned configs together; past it the "
                         "headline line is printed with the unfinished configs marked and every rank exits")
    ap.add_argument("--extra-steps", type=int, default=50)
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--no-resident", action="store_true",
                    help="launch one kernel per query instead of the resident query server")
    ap.add_argument("--batch", type=int, default=256,
                    help="also measure batched serving: K queries per launch, one CU each (0 = skip)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for the bench's own barriers/reductions (nccl = RCCL; "
                         "gloo lets several ranks share one GPU for rehearsals)")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev  # one rank per GPU; with gloo, extra ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            dist.init_process_group(backend="gloo")

    from bidirectional_bfs_amd.ops import HipEngine
    from bidirectional_bfs_amd.parallel import DistEngine

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def run_config(spec: str, steps: int, warmup: int, mode: str = a.mode):
        _, n, _, seed = parse_spec(spec)
        t0 = time.perf_counter()
        if mode == "partitioned" and world > 1:
            eng = generate(DistEngine.from_torch_distributed(local), spec)
            m = eng.m
        else:
            eng = generate(HipEngine(local), spec)
            eng.set_resident(not a.no_resident)
            m = eng.m
        build_s = time.perf_counter() - t0
        pairs = pick_pairs(eng, n, a.pairs if mode != "partitioned" else min(a.pairs, steps + warmup), 12345)
        assert pairs, f"no connected pairs found in {spec}"

        def query(i):
            if mode == "partitioned" and world > 1:
                s, d = pairs[i % len(pairs)]
            else:
                s, d = pairs[(i * world + rank) % len(pairs)]
            r = eng.search(s, d)
            path = r.path  # the path is part of every answer (materialised on the host)
            assert r.found and len(path) == r.hops + 1
            return r

        resident = hasattr(eng, "set_resident") and not a.no_resident

        def park():
            # A device-wide synchronize waits for every kernel, the resident
            # server included: stop it first (it relaunches on the next query).
            if resident:
                eng.set_resident(False)

        for i in range(warmup):
            query(i)
        park()
        barrier()
        if resident:
            eng.set_resident(True)  # lazily relaunched by the first timed query (launch cost is timed)
        done = [None] * steps
        t0 = time.perf_counter()
        for i in range(steps):
            done[i] = query(warmup + i)  # answer checked in query(); statistics read after the clock
        park()  # server shutdown is inside the timed region
        barrier()
        dt = max_over_ranks(time.perf_counter() - t0)
        hops = sum(r.hops for r in done)
        insp = sum(r.edges_inspected for r in done)
        dev_ms = sum(r.search_ms for r in done)
        queries = steps * (1 if mode == "partitioned" else world)
        batched = None
        if a.batch > 0 and mode == "replicated" and hasattr(eng, "search_batch"):
            # throughput serving: K distinct queries per launch (pairs cycled), steady state
            park()
            bp = [pairs[(i * world + rank) % len(pairs)] for i in range(a.batch)]
            bs = [s for s, _ in bp]
            bd = [d for _, d in bp]
            for _ in range(3):
                eng.search_batch_arrays(bs, bd)
            barrier()
            reps = max(3, steps // 40)
            tb = time.perf_counter()
            for _ in range(reps):
                bh, boff, _paths = eng.search_batch_arrays(bs, bd)
                assert (bh >= 0).all() and (boff[1:] - boff[:-1] == bh + 1).all()
            barrier()
            bdt = max_over_ranks(time.perf_counter() - tb)
            bq = reps * a.batch * world
            batched = {"batch": a.batch, "launches": reps, "ms_per_batch": bdt * 1e3 / reps,
                       "us_per_query": bdt * 1e6 / (reps * a.batch), "queries_per_s": bq / bdt,
                       "gteps": m * bq / bdt / 1e9}
        out = {
            "n": n, "m": m, "seed": seed, "wall_s": dt, "ms_per_step": dt * 1e3 / steps,
            "gteps": m * queries / dt / 1e9,
            "gteps_inspected": insp * (1 if mode == "partitioned" else world) / dt / 1e9,
            "mean_hops": hops / steps, "device_ms_per_query": dev_ms / steps,
            "build_ms": build_s * 1e3, "end_to_end_first_query_ms": build_s * 1e3 + dt * 1e3 / steps,
            "queries": queries, "batched": batched,
        }
        if mode == "partitioned" and world > 1:
            out["engine"] = f"DistBiBfs/{eng.backend} x{world}"
            out["last_query_stats"] = eng.last_stats
        if hasattr(eng, "release"):
            eng.release()  # free HBM before the next config
        return out

    head = run_config(a.graph, a.steps, a.warmup)
    extra = {}
    partitioned = {}
    printed = threading.Lock()

    def emit():
        if rank == 0 and printed.acquire(blocking=False):
            print(json.dumps(report(a, world, head, extra, partitioned)), flush=True)

    def watchdog():
        # A secondary config that hangs (e.g. a collective that never completes
        # on some rank) must not take the headline measurement with it.
        for d in (extra, partitioned):
            for k, v in list(d.items()):
                if v is None:
                    d[k] = {"error": f"watchdog: unfinished after {a.secondary_timeout:.0f} s"}
        emit()
        sys.stdout.flush()
        os._exit(0)

    dog = threading.Timer(a.secondary_timeout, watchdog)
    dog.daemon = True
    dog.start()
    for spec in filter(None, a.extra_graph.split(",")):
        extra[spec] = None
        try:
            extra[spec] = run_config(spec, a.extra_steps, min(a.warmup, 10), "replicated")
        except Exception as exc:  # report, never hide, a failing secondary config
            extra[spec] = {"error": repr(exc)}
    if world > 1 and a.mode == "replicated" and a.dist_backend == "nccl":
        for spec in filter(None, a.dist_graphs.split(",")):
            partitioned[spec] = None
            try:
                partitioned[spec] = run_config(spec, a.dist_steps, 3, "partitioned")
            except Exception as exc:
                partitioned[spec] = {"error": repr(exc)}

    emit()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    dog.cancel()  # after the teardown: a hung final barrier is covered too
    return 0


if __name__ == "__main__":
    sys.exit(main())
