#!/usr/bin/env python3
"""Headline benchmark: end-to-end shortest-path queries on the reference graph
shape, reported as GTEPS(M/t) (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--graph gnp:100000::6]
                    [--mode replicated|partitioned] [--extra-graph gnp:10000000::1,kron:22:16:1]
                    [--dist-graphs gnp:1000000::2,kron:22:16:1,kron:auto]

One step = one bidirectional-BFS query per GPU: host call -> search on the
MI355X -> hop count AND the full path back in host memory ("end-to-end ms to
shortest path").  Graph: G(n, p = 2.2/n) exactly like the reference suite
(graphs/make_graphs:8), generated on the device from a fixed seed (synthetic,
there is no dataset); queries are seeded random vertex pairs that are
connected (the first is (0, N-1) like benchmark_test.sh:43), fixed before
timing and rotated over every step, so no result is reused.

Launch: N > 1 runs one rank per GPU.  Under torch.distributed.run (the
driver's launcher) the ranks come from the environment; `python bench.py
--gpus N` without a launcher starts torch.distributed.run itself as a child
process BEFORE anything touches the GPU, forwards rank 0's line and exits with
the child's status.

Two scaling curves, both measured at every N:
  headline    (`value`, weak scaling, mode "replicated") every GPU holds the
              whole graph and answers its own queries -- production query
              serving; value = aggregate GTEPS over all GPUs;
  partitioned (`detail.partitioned`, strong scaling, the v4 capability) the
              graph is 1-D partitioned over the N GPUs (device-generated CSR
              shards) and every query is ONE collective search over RCCL;
              configs: 1M G(n,p) (BASELINE config 3), Kronecker 22 (config 4)
              and Kronecker 27, 2.15B edges (config 5).  Each is checked
              against the single-GPU engine's hop counts (`verified`).
`--mode partitioned` makes the partitioned engine the headline instead.

vs_baseline divides by the best published 100k number in BASELINE.md (v1
serial: 0.116 ms -> 0.952 GTEPS(M/t)); `cpu_serial_ms` is this repo's own -O3
serial engine on the same graph and pairs, for an explicit CPU comparison.
"""
from __future__ import annotations

import argparse
import json
import os
import random
import socket
import subprocess
import statistics
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

BASELINE_100K_GTEPS = 110000 / (0.115546e-3) / 1e9  # v1 @ 100k, M ~ 1.1 (N - 1)
BASELINE_100K_MS = 0.115546


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--graph", default="gnp:100000::6")
    ap.add_argument("--mode", choices=["replicated", "partitioned"], default="replicated")
    ap.add_argument("--extra-graph", default="gnp:10000000::1,kron:22:16:1",
                    help="comma-separated secondary configs reported under 'extra' (empty to skip)")
    ap.add_argument("--dist-graphs", default="gnp:1000000::2,kron:22:16:1,kron:auto",
                    help="configs run through the partitioned RCCL engine at every N (empty to skip); "
                         "kron:auto = Kronecker 27 (2.15B edges, ~17 GB of CSR) on one GPU, and for N >= 2 "
                         "Kronecker 30 with the edge factor that makes the CSR ~1.35x ONE GPU's HBM (a graph "
                         "no single MI355X can hold: edge factor 44, ~390 GB, on 288 GB parts), verified "
                         "without any single-GPU copy")
    ap.add_argument("--dist-steps", type=int, default=20)
    ap.add_argument("--secondary-timeout", type=float, default=420.0,
                    help="seconds allowed for the extra + partitioned configs together; past it the "
                         "headline line is printed with the unfinished configs marked")
    ap.add_argument("--strict", action="store_true",
                    help="exit non-zero when a secondary (extra / partitioned) config fails or times out; "
                         "by default such a failure is reported in detail.secondary_errors only.  A partitioned "
                         "config that returns WRONG answers (verified false) always exits 5")
    ap.add_argument("--extra-steps", type=int, default=50)
    ap.add_argument("--pairs", type=int, default=64)
    ap.add_argument("--no-resident", action="store_true",
                    help="launch one kernel per query instead of the resident query server")
    ap.add_argument("--batch", type=int, default=256,
                    help="also measure batched serving: K queries per launch, one CU each (0 = skip)")
    ap.add_argument("--no-cpu-ref", action="store_true", help="skip the CPU serial comparison")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"],
                    help="process-group backend for the bench's own barriers/reductions (nccl = RCCL; "
                         "gloo lets several ranks share one GPU for rehearsals; auto = gloo exactly when "
                         "the ranks on a node outnumber its GPUs)")
    ap.add_argument("--dist-comm", default="auto", choices=["auto", "rccl", "ipc"],
                    help="collective transport of the partitioned engine: rccl (one rank per GPU), ipc "
                         "(HIP-IPC staging buffers; ranks may share a GPU), auto = ipc when ranks share a GPU")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# self-launch (no GPU is touched in this process)
# ---------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_cmd(nproc: int, argv) -> list:
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)


def spawn_ranks(nproc: int, argv, cmd=None) -> int:
    """Run the N-rank job as a child process group, forward rank 0's JSON line.

    Returns the child's exit status, or 1 when it exited 0 without a line."""
    cmd = cmd or launcher_cmd(nproc, argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for ln in proc.stdout.splitlines():
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        elif s:
            print(s, file=sys.stderr)
    if line is not None:
        print(line, flush=True)
    if proc.returncode != 0:
        return proc.returncode
    return 0 if line is not None else 1


# ---------------------------------------------------------------------------
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


HBM_DEFAULT = 288 * 10**9  # MI355X HBM3E per GPU (used when the device does not say)


def csr_bytes(spec: str) -> int:
    """Device bytes of the whole graph's CSR (u64 row offsets, u32 columns, both directions)."""
    kind, n, arg, _ = parse_spec(spec)
    m = int(arg) if kind == "rmat" else int(arg * n * (n - 1) / 2)
    return 8 * (n + 1) + 4 * 2 * m


def world_scaled(spec: str, world: int, hbm_bytes: int = HBM_DEFAULT) -> str:
    """kron:auto -> Kronecker 27 (2.15B edges, ~17 GB CSR) on one GPU, where the
    single-GPU engine is the reference; for N >= 2 a graph NO single GPU can
    hold: Kronecker 30 with the edge factor that makes the CSR ~1.35x one
    GPU's HBM (edge factor 44, ~390 GB on 288 GB parts), capped so a rank's
    shard stays within ~70% of its HBM."""
    if spec != "kron:auto":
        return spec
    if world <= 1:
        return "kron:27:16:1"
    unit = 8 * (1 << 30)  # CSR bytes per unit of edge factor at scale 30 (4 B x 2 directions x 2^30)
    ef = int((1.35 * hbm_bytes - 8 * (1 << 30)) // unit)
    ef = min(ef, int((0.7 * hbm_bytes * world - 8 * (1 << 30)) // unit))
    return f"kron:30:{max(16, ef)}:1"


def generate(eng, spec: str):
    kind, n, arg, seed = parse_spec(spec)
    if kind == "gnp":
        eng.generate_gnp(n, arg, seed)
    else:
        eng.generate_rmat(n, arg, seed)
    return eng


def pick_pairs(eng, n: int, count: int, seed: int):
    """Seeded connected (src, dst) pairs; (0, N-1) first (benchmark_test.sh:43).
    Returns [(src, dst, hops)]."""
    rng = random.Random(seed)
    pairs, tries = [], 0
    cand = [(0, n - 1)]
    while len(pairs) < count and tries < 50 * count:
        s, d = cand.pop() if cand else (rng.randrange(n), rng.randrange(n))
        tries += 1
        r = eng.search(s, d)
        if r.found and r.hops > 0:
            pairs.append((s, d, int(r.hops)))
    return pairs


PARTITIONED_HEADLINE = "gnp:1000000::2"  # BASELINE config 3: 1M-vertex G(n, 2.2/n), vertex-partitioned


def partitioned_top(partitioned: dict) -> dict:
    """Top-level fields beside the replicated headline: the partitioned
    engine's BASELINE config-3 numbers (one query = one collective search over
    every rank), so a scaling curve over N shows the v4 capability and not only
    N independent servers.  None where that config did not run or failed."""
    p = partitioned.get(PARTITIONED_HEADLINE)
    ok = isinstance(p, dict) and "error" not in p and p.get("ms_per_query") is not None
    return {
        "partitioned_config": PARTITIONED_HEADLINE,
        "partitioned_ms_per_query": p["ms_per_query"] if ok else None,
        "partitioned_speedup_vs_single_gpu": p.get("speedup_vs_single_gpu") if ok else None,
        "partitioned_speedup_vs_single_gpu_median": p.get("speedup_vs_single_gpu_median") if ok else None,
        "partitioned_gteps": round(p["gteps"], 4) if ok and p.get("gteps") is not None else None,
        "partitioned_collectives_per_round": p.get("collectives_per_round") if ok else None,
        "partitioned_verified": p.get("verified") if ok else None,
    }


def report(a, world: int, head: dict, extra: dict, partitioned: dict, rccl_ranks=None,
           comm_init_ms=None) -> dict:
    """The one JSON line rank 0 prints (driver contract)."""
    part = a.mode == "partitioned"
    return {
        "metric": "GTEPS(M/t), end-to-end bi-BFS shortest-path query (G(n,2.2/n), path returned to host)",
        "value": round(head["gteps"], 4),
        "unit": "GTEPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(head["ms_per_step"], 6),
        "higher_is_better": True,
        "scaling": "strong" if part else "weak",
        "vs_baseline": round(head["gteps"] / BASELINE_100K_GTEPS, 3) if head["n"] == 100000 else None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "model": f"G(n={head['n']}, p=2.2/n) seed={head['seed']}, M={head['m']}",
            "global_batch": 1 if part else world,
            "seq_len": head["n"],
            "parallelism": (f"vertex-partition{world}" if part else f"dp{world}"),
        },
        **partitioned_top(partitioned),
        "detail": {
            "query_ms": round(head["ms_per_step"], 6),
            "device_ms_per_query": round(head["device_ms_per_query"], 6),
            "cpu_serial_ms": head.get("cpu_serial_ms"),
            "cpu_serial_query_ms": head.get("cpu_serial_query_ms"),
            "baseline_best_100k_ms": BASELINE_100K_MS,
            "gteps_inspected": head["gteps_inspected"],
            "mean_hops": head["mean_hops"],
            "graph_build_ms": round(head["build_ms"], 3),
            "server_launch_ms": head.get("server_launch_ms"),
            "tiny_server": head.get("tiny_server"),
            "tiny_overflows": head.get("tiny_overflows"),
            "resident_server": (not part) and not a.no_resident,
            "batched_serving": head["batched"],
            "rccl_ranks": rccl_ranks,
            "weak_scaling": "headline: replicated graph, every GPU answers its own queries (no inter-GPU traffic)",
            "strong_scaling": "partitioned: one query = one collective search over all GPUs (RCCL over xGMI)",
            "extra": extra,
            "partitioned": partitioned,
            # the partitioned engine's communicator, made once for every config
            "partitioned_comm_init_ms": round(comm_init_ms, 3) if comm_init_ms is not None else None,
            # secondary configs that failed, were unverified or hit the watchdog
            "secondary_errors": sorted(
                k for d in (extra, partitioned) for k, v in d.items()
                if v is None or "error" in v or v.get("verified") is False),
        },
    }


def exit_status(partitioned: dict, failed: bool, strict: bool) -> int:
    """Wrong answers are never a soft failure: a partitioned config that ran
    and returned a wrong hop count or path fails the run (5).  Timeouts and
    setup errors of secondary configs fail it only with --strict (4)."""
    wrong = sorted(k for k, v in partitioned.items() if isinstance(v, dict) and v.get("verified") is False)
    if wrong:
        print(f"bench.py: partitioned config(s) {wrong} returned wrong answers", file=sys.stderr)
        return 5
    if failed:
        print("bench.py: a secondary config failed (detail.secondary_errors)", file=sys.stderr)
    return 4 if (failed and strict) else 0


def cpu_serial_ms(spec: str, pairs, reps: int = 20, oracle_pairs: int = 0):
    """This repo's -O3 serial engine (v1 parity) on the same graph and pairs:
    (median engine-internal search ms, mean of it, mean end-to-end query ms
    through the same Python call + path access as the GPU loop, pairs whose
    GPU hop count a unidirectional host BFS (bfs_oracle) re-derived).  Every
    pair's hop count is also held to the serial engine's."""
    from bidirectional_bfs_amd import native

    kind, n, arg, seed = parse_spec(spec)
    el = native.gen_gnp(n, arg, seed) if kind == "gnp" else native.gen_rmat(n, int(arg), seed, 0.57, 0.19, 0.19)
    csr = native.build_csr(el)
    del el
    oracle_ok = 0
    for s, d, h in pairs[:oracle_pairs]:
        assert native.bfs_oracle(csr, s, d).hops == h, (spec, s, d, h)
        oracle_ok += 1
    eng = native.SerialBiBfs(csr)
    ts = []
    q = reps * len(pairs)
    for i in range(q):
        s, d, h = pairs[i % len(pairs)]
        r = eng.search(s, d)
        assert r.found and r.hops == h and len(r.path) == h + 1, (s, d, r.hops, h)
        ts.append(r.search_ms)
    ts_first = ts[:len(pairs)]
    # end to end through the same serving call shape as the GPU loop: (hops, path list)
    t0 = time.perf_counter()
    for i in range(q):
        s, d, h = pairs[i % len(pairs)]
        hh, path = eng.query(s, d)
        assert hh == h and len(path) == h + 1 and path[0] == s and path[-1] == d
    e2e = (time.perf_counter() - t0) * 1e3 / q
    ts.sort()
    # every pass above after the first finds the pairs' neighbourhoods in the
    # CPU caches; the first search of each pair (ts_first) is the cold number
    first = sorted(ts_first)
    return ts[len(ts) // 2], sum(ts) / len(ts), e2e, oracle_ok, sum(first) / len(first)


def cpu_fields(med: float, mean: float, e2e: float, oracle_ok: int, first: float, gpu_ms: float) -> dict:
    """The CPU comparison of one replicated config (same graph, same pairs).
    cpu_serial_query_ms repeats the pairs (warm CPU caches after the first
    pass, as the GPU loop's pairs were searched before its timing too);
    cpu_serial_first_pass_ms is the mean search of each pair's first run."""
    return {"cpu_serial_ms": round(med, 6), "cpu_serial_mean_ms": round(mean, 6),
            "cpu_serial_query_ms": round(e2e, 6), "cpu_serial_first_pass_ms": round(first, 6),
            "speedup_vs_cpu_serial_query": round(e2e / gpu_ms, 3) if gpu_ms else None,
            "cpu_oracle_checked_pairs": oracle_ok}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return spawn_ranks(a.gpus, argv)  # before any GPU call in this process
    world = int(env_world or "1")
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        return 2

    import torch  # first: the HIP runtime torch ships is the one our extension then binds to
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = max(1, torch.cuda.device_count())
    # several ranks on one GPU (a gloo / IPC rehearsal): decided alike on every
    # rank from the launcher's ranks-per-node, never from this rank's index
    shared_gpu = int(os.environ.get("LOCAL_WORLD_SIZE", world)) > ndev
    # (no GPU_MAX_HW_QUEUES=1 here, unlike the partitioned-only launchers: a
    # rank's resident single-GPU server is a persistent kernel, and with one
    # queue the hand-off levels queued behind it waited for its idle exit --
    # 10M queries 0.09 -> 172 ms in the 2-rank rehearsal,
    # profiles/r6_bench_2rank_1gpu_ipc_hwq1_end.json)
    if a.dist_backend == "auto":
        a.dist_backend = "gloo" if shared_gpu else "nccl"
    local = local % ndev
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group(backend="nccl", device_id=dev)
        else:
            # gloo prints its connection report on fd 1: keep it off the JSON
            # line's stream (the rendezvous and first collective, on stderr)
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                dist.init_process_group(backend="gloo")
                dist.barrier()
            finally:
                os.dup2(saved, 1)
                os.close(saved)

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

    def all_ranks_ok(ok: bool) -> bool:
        if world == 1:
            return ok
        t = torch.tensor([0.0 if ok else 1.0], dtype=torch.float64, device=dev if a.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item()) == 0.0

    def run_replicated(spec: str, steps: int, warmup: int, cpu_ref: bool = False):
        _, n, _, seed = parse_spec(spec)
        t0 = time.perf_counter()
        eng = generate(HipEngine(local), spec)
        eng.set_resident(not a.no_resident)
        m = eng.m
        build_s = time.perf_counter() - t0
        pairs = pick_pairs(eng, n, a.pairs, 12345)
        assert pairs, f"no connected pairs found in {spec}"

        def query(i):
            # the serving API: (hops, path) with the path as a host-side list
            s, d, h = pairs[(i * world + rank) % len(pairs)]
            hh, path = eng.query(s, d)
            assert hh == h and len(path) == h + 1 and path[0] == s and path[-1] == d
            return hh

        resident = not a.no_resident

        def park():
            # A device-wide synchronize waits for every kernel, the resident
            # server included: stop it first (it relaunches on the next query).
            if resident:
                eng.set_resident(False)

        # Setup, untimed: the device is synchronized with the server down, then
        # the resident server is launched and answers one query (its launch is
        # reported as server_launch_ms, like graph_build_ms).
        park()
        barrier()
        ts = time.perf_counter()
        if resident:
            eng.set_resident(True)
        query(0)
        launch_ms = (time.perf_counter() - ts) * 1e3
        for i in range(warmup):
            query(i)

        def stream_barrier():
            # The resident server never completes, so a device-wide synchronize
            # would wait for its idle exit: every rank instead syncs the engine's
            # own streams (nothing else is queued) and meets the others.  Every
            # timed query's answer -- hop count and path -- is in host memory
            # before the next starts.
            if world > 1:
                dist.barrier()
            eng.synchronize()

        stream_barrier()
        ov0 = eng.tiny_overflows
        t0 = time.perf_counter()
        for i in range(steps):
            query(warmup + i)  # answer checked in query()
        # closing bracket: this rank's streams synchronized, its clock read,
        # then the barrier -- the max over ranks is the slowest rank's K steps
        # from the common start, without the closing barrier's own latency
        # (~50-500 us with gloo / RCCL: several steps of a ~15 us query)
        eng.synchronize()
        dt_local = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        dt = max_over_ranks(dt_local)
        # queries of the timed loop the tiny server handed to the general engine
        timed_overflows = int(max_over_ranks(float(eng.tiny_overflows - ov0)))
        # statistics, untimed: the same queries again, reading the per-query
        # device time and edges inspected the timed loop did not touch
        hops = insp = 0
        dev_ms = 0.0
        for i in range(steps):
            hops += query(warmup + i)
            dev_ms += eng.last_search_ms
            insp += eng.last_edges_inspected
        # direction-optimizing evidence (BASELINE config 4), untimed: how many
        # levels ran on the grid / bottom-up, and how many searches left LDS
        nd = min(steps, 64)
        gl = bu = ho = 0
        for i in range(nd):
            s_, d_, _ = pairs[((warmup + i) * world + rank) % len(pairs)]
            st = eng.search(s_, d_).stats
            gl += st["grid_levels"]
            bu += st["bottomup_levels"]
            ho += 1 if st["handoff"] else 0
        park()
        barrier()  # device-wide synchronize with the server down
        queries = steps * world
        batched = None
        if a.batch > 0:
            # throughput serving: K distinct queries per launch (pairs cycled), steady state
            park()
            bp = [pairs[(i * world + rank) % len(pairs)] for i in range(a.batch)]
            bs = [s for s, _, _ in bp]
            bd = [d for _, d, _ in bp]
            bh_ref = [h for _, _, h in bp]
            for _ in range(3):
                eng.search_batch_arrays(bs, bd)
            barrier()
            reps = max(3, steps // 40)
            tb = time.perf_counter()
            fallbacks = 0
            for _ in range(reps):
                bh, boff, _paths = eng.search_batch_arrays(bs, bd)
                fallbacks += eng.last_batch_fallbacks
                assert (bh >= 0).all() and (boff[1:] - boff[:-1] == bh + 1).all()
            barrier()
            bdt = max_over_ranks(time.perf_counter() - tb)
            assert list(bh) == bh_ref
            bq = reps * a.batch * world
            batched = {"batch": a.batch, "launches": reps, "ms_per_batch": bdt * 1e3 / reps,
                       "us_per_query": bdt * 1e6 / (reps * a.batch), "queries_per_s": bq / bdt,
                       "gteps": m * bq / bdt / 1e9,
                       # queries re-run one by one (level above the batch edge cap / long path)
                       "fallback_queries_per_batch": fallbacks / reps}
        out = {
            "n": n, "m": m, "seed": seed, "wall_s": dt, "ms_per_step": dt * 1e3 / steps,
            "gteps": m * queries / dt / 1e9,
            "gteps_inspected": insp * world / dt / 1e9,
            "mean_hops": hops / steps, "device_ms_per_query": dev_ms / steps,
            "build_ms": build_s * 1e3, "server_launch_ms": round(launch_ms, 4),
            "tiny_server": bool(eng.tiny_engine and resident),
            "tiny_overflows": timed_overflows,  # timed-loop queries re-run on the general engine (max over ranks)
            "end_to_end_first_query_ms": build_s * 1e3 + launch_ms,
            "queries": queries, "batched": batched,
            "grid_levels_per_query": gl / nd, "bottomup_levels_per_query": bu / nd,
            "handoff_fraction": ho / nd,
        }
        eng.release()  # free HBM before the next config
        if cpu_ref and not a.no_cpu_ref:
            # headline: 20 passes over the pairs; extras (10M, Kronecker): 3,
            # plus a unidirectional host BFS of their first 4 pairs
            big = n > 1000000 or m > 10000000
            out.update(cpu_fields(*cpu_serial_ms(spec, pairs, reps=3 if big else 20, oracle_pairs=4 if big else 0),
                                  out["ms_per_step"]))
        return out

    comm = a.dist_comm if a.dist_comm != "auto" else ("ipc" if shared_gpu else "rccl")
    dstate = {}

    def dist_engine():
        """ONE partitioned engine (one communicator) for every config: its
        bootstrap -- the first RCCL communicator of the process pays ~3.5 s of
        library / kernel loading -- is reported once (partitioned_comm_init_ms),
        not inside the first config; release() frees a config's graph.  At
        world size 1 the engine's collectives are copies to itself (an
        in-process group of one: no RCCL bootstrap, no unique id needed)."""
        if "eng" not in dstate:
            barrier()
            t0 = time.perf_counter()
            if world == 1:
                uid = DistEngine.unique_id(comm) if os.environ.get("BIBFS_WORLD1_COMM") == comm else b""
                dstate["eng"] = DistEngine(0, 1, local, uid, comm)
            else:
                dstate["eng"] = DistEngine.from_torch_distributed(local, backend=comm)
            dstate["init_ms"] = max_over_ranks((time.perf_counter() - t0) * 1e3)
        return dstate["eng"]

    def run_partitioned(spec: str, steps: int, warmup: int):
        """Strong scaling: the graph sharded over all ranks, one collective search per query.
        Where the graph fits one GPU, pairs, hop counts and the speedup come
        from the single-GPU engine on the same graph; a graph that does not
        (kron:auto at N >= 2) is verified without any single-GPU copy: pairs
        picked by the partitioned engine, every checked path validated edge by
        edge by the owners of its vertices, and hop counts cross-checked by a
        unidirectional partitioned BFS."""
        _, n, _, seed = parse_spec(spec)
        hbm_total = torch.cuda.mem_get_info(dev)[1]
        fits = csr_bytes(spec) <= 0.6 * hbm_total
        single_ms, single_med_ms, single_reason, pairs = None, None, None, None
        npairs = min(a.pairs, steps + warmup)
        if fits:
            ref = generate(HipEngine(local), spec)
            pairs = pick_pairs(ref, n, npairs, 12345)
            assert pairs, f"no connected pairs found in {spec}"
            # the single-GPU engine on the same graph and pairs (resident serving),
            # so every partitioned entry states its speedup over one GPU
            ref.set_resident(True)
            # warm: every pair once (the engine under test gets the same pass
            # below -- its CSR is a fresh allocation, cold in L2 / MALL)
            for i in range(max(warmup, len(pairs))):
                ref.query(*pairs[i % len(pairs)][:2])
            ts = time.perf_counter()
            sq = []
            for i in range(steps):
                s_, d_, h_ = pairs[(warmup + i) % len(pairs)]
                q0 = time.perf_counter()
                assert ref.query(s_, d_)[0] == h_
                sq.append(time.perf_counter() - q0)
            single_ms = max_over_ranks((time.perf_counter() - ts) * 1e3 / steps)
            single_med_ms = max_over_ranks(statistics.median(sq) * 1e3)
            ref.set_resident(False)
            ref.release()
            del ref
        else:
            single_reason = (f"the graph's CSR ({csr_bytes(spec) / 1e9:.0f} GB) does not fit one GPU's HBM "
                             f"({hbm_total / 1e9:.0f} GB): there is no single-GPU run to compare with")
        torch.cuda.synchronize()
        barrier()
        eng = dist_engine()  # (communicator made once, reported apart from every graph build)
        eng.set_tuning()
        t0 = time.perf_counter()
        generate(eng, spec)
        build_ms = max_over_ranks((time.perf_counter() - t0) * 1e3)
        free_b, total_b = torch.cuda.mem_get_info(dev)
        hbm_used = total_b - free_b
        m = eng.m
        if pairs is None:  # picked by the partitioned engine itself (collective searches)
            pairs = pick_pairs(eng, n, npairs, 12345)
            assert pairs, f"no connected pairs found in {spec}"
        wrong = []

        def query(i):
            # statistics passes: the full SearchResult (stats read after it)
            s, d, h = pairs[i % len(pairs)]
            r = eng.search(s, d)
            if not (r.found and r.hops == h and len(r.path) == h + 1 and r.path[0] == s and r.path[-1] == d):
                wrong.append((s, d, h, r.hops))
            return r

        def lean(i):
            # timed loops: the serving call, (hops, path) -- the same shape as the
            # single-GPU reference loop above; stats are read outside the timing
            s, d, h = pairs[i % len(pairs)]
            hh, path = eng.query(s, d)
            if not (hh == h and len(path) == h + 1 and path[0] == s and path[-1] == d):
                wrong.append((s, d, h, hh))

        for i in range(max(warmup, len(pairs))):  # every pair once, as the single-GPU loop
            lean(i)
        # the engine's own barrier (RCCL allreduce + its streams drained); no
        # device-wide synchronize: at world size 1 the single-GPU engine's
        # resident server stays up across it, as in the headline loop
        eng.barrier()
        if world > 1:
            dist.barrier()
        qt = []
        t0 = time.perf_counter()
        for i in range(steps):
            q0 = time.perf_counter()
            lean(warmup + i)
            qt.append(time.perf_counter() - q0)
        # (the loop's end, as for the single-GPU loop above: every query is a
        # collective search, so the ranks leave it together; the barrier after
        # it -- an allreduce and the engine's streams drained -- is not a query)
        t_end = time.perf_counter()
        eng.barrier()
        dt = max_over_ranks(t_end - t0)
        # the same queries again, untimed, for the per-query statistics
        done = []
        for i in range(steps):
            done.append((query(warmup + i), eng.last_stats))
        ok = all_ranks_ok(not wrong)
        st = [s for _, s in done]
        rounds = sum(s["rounds"] for s in st) / steps
        out = {
            "engine": f"DistBiBfs/{eng.backend}", "ranks": world, "rccl_ranks": eng.world,
            "n": n, "m": m, "seed": seed, "build_ms": round(build_ms, 3),
            "local_nnz_max": int(max_over_ranks(float(eng.local_nnz))),
            "csr_bytes_total": csr_bytes(spec), "hbm_bytes_per_gpu": int(hbm_total), "fits_one_gpu": fits,
            # per-rank HBM, measured: the CSR shard; the most the rank held at
            # once during the build (shard + generator temporaries, counted per
            # allocation -- build only, before the search state exists) and the
            # device's free-memory drop over it (hipMemGetInfo low-water mark);
            # what it holds for search (shard + search state)
            "shard_bytes_max": int(max_over_ranks(float(eng.shard_bytes))),
            "gen_peak_bytes_max": int(max_over_ranks(float(eng.gen_peak_bytes))),
            "gen_hbm_peak_bytes_max": int(max_over_ranks(float(eng.gen_hbm_peak_bytes))),
            "resident_bytes_max": int(max_over_ranks(float(eng.resident_bytes))),
            "hbm_used_bytes_max": int(max_over_ranks(float(hbm_used))),
            "queries": steps, "ms_per_query": round(dt * 1e3 / steps, 5),
            "median_query_ms_rank0": round(sorted(qt)[len(qt) // 2] * 1e3, 5),
            "max_query_ms_rank0": round(max(qt) * 1e3, 5),
            "single_gpu_ms": round(single_ms, 5) if single_ms is not None else None,
            "speedup_vs_single_gpu": round(single_ms / (dt * 1e3 / steps), 4) if single_ms is not None else None,
            # the same ratio on medians (max over ranks of each rank's median):
            # one multi-millisecond outlier in 20 timed queries moves the means
            "single_gpu_median_ms": round(single_med_ms, 5) if single_med_ms is not None else None,
            "speedup_vs_single_gpu_median": (round(single_med_ms / max_over_ranks(statistics.median(qt) * 1e3), 4)
                                             if single_med_ms is not None else None),
            "single_gpu_reason": single_reason,
            "gteps": m * steps / dt / 1e9,
            "device_ms_per_query": round(sum(r.search_ms for r, _ in done) / steps, 5),
            "mean_hops": sum(r.hops for r, _ in done) / steps,
            "mean_rounds": rounds,
            "ms_per_round": round(dt * 1e3 / steps / rounds, 5) if rounds else None,
            "host_syncs_per_query": sum(s["host_syncs"] for s in st) / steps,
            "exchanged_bytes_per_query": sum(s["exchanged_bytes"] for s in st) / steps,
            "collectives_per_query": sum(s["collectives"] for s in st) / steps,
            "collectives_per_round": sum(s["collectives"] for s in st) / max(1, sum(s["rounds"] for s in st)),
            "speculative_rounds_per_query": sum(s["spec_rounds"] for s in st) / steps,
            "dense_levels_per_query": sum(s["dense_levels"] for s in st) / steps,
            # pipelined searches that stalled and finished with exact plans
            "pipe_drains_per_query": sum(s.get("pipe_drains", 0) for s in st) / steps,
            "verified": ok, "checked_queries": steps + warmup,
            "world1_engine": ("single-GPU engine over the rank's own device CSR (DistTuning.world1_single)"
                              if world == 1 and st and st[0].get("single_engine") else None),
        }
        if world == 1:
            # the partitioned rounds at world size 1 (solo workgroup + speculative
            # rounds), side by side with the default single-engine path
            eng.set_tuning(world1_single=False)
            for i in range(3):
                lean(i)
            eng.barrier()
            t1 = time.perf_counter()
            for i in range(steps):
                lean(warmup + i)
            eng.barrier()
            out["rounds_engine_ms_per_query"] = round((time.perf_counter() - t1) * 1e3 / steps, 5)
            eng.set_tuning()
        # distributed verification (untimed, no graph copy anywhere): each
        # checked path edge looked up by the owner of its first vertex, and the
        # hop counts re-derived by a unidirectional partitioned BFS
        nchk = min(len(pairs), 8)
        bad_paths, bad_hops = 0, 0
        for i in range(nchk):
            s_, d_, h_ = pairs[i]
            r = eng.search(s_, d_)
            if not eng.validate_path(s_, d_, r.hops, list(r.path)):
                bad_paths += 1
            if i < 3 and eng.search_unidirectional(s_, d_).hops != h_:
                bad_hops += 1
        dist_ok = all_ranks_ok(bad_paths == 0 and bad_hops == 0)
        out["verification"] = {
            "pairs_from": "single-GPU engine" if fits else "partitioned engine",
            "hops_vs_single_gpu": fits,
            # hop counts held to an independent engine: every timed pair when the
            # single-GPU engine picked them, else only the unidirectional BFS pairs
            # (the timed loop's check is then self-consistency: ADVICE r4)
            "hops_cross_checked": (steps + warmup) if fits else min(nchk, 3),
            "paths_checked_distributed": nchk, "bad_paths": bad_paths,
            "unidirectional_bfs_checked": min(nchk, 3), "bad_hops": bad_hops}
        out["verified"] = ok and dist_ok
        # per-round split (untimed): device stamps at the entry and exit of
        # every speculative round's kernels -> kernel time vs the gaps the
        # candidate exchange and the status allgather leave
        out.update(round_split(eng, query, warmup, min(steps, 8)))
        if world > 1:
            # the same timed loop with exact plans (DistTuning.pipeline off: a
            # status allgather per round beside the candidate exchange), side by
            # side with the default pipelined rounds (one collective per round)
            eng.set_tuning(pipeline=False)
            for i in range(2):
                lean(i)
            eng.barrier()
            barrier()
            t1 = time.perf_counter()
            for i in range(steps):
                lean(warmup + i)
            eng.barrier()
            dte = max_over_ranks(time.perf_counter() - t1)
            ex = {"ms_per_query": round(dte * 1e3 / steps, 5),
                  "pipelined_speedup": round(dte / dt, 4)}
            ex.update(round_split(eng, query, warmup, min(steps, 8), pipeline=False))
            out["pipeline_off"] = ex
            eng.set_tuning()
            out["verified"] = all_ranks_ok(not wrong) and dist_ok
        else:
            out["pipeline_off"] = None  # one rank: nothing is exchanged, every plan is exact
        if wrong:
            out["mismatch"] = wrong[:4]
        out["comm"] = eng.backend
        eng.release()
        return out, eng.world

    def round_split(eng, query, first: int, count: int, pipeline: bool = True) -> dict:
        eng.set_tuning(stamps=True, pipeline=pipeline)
        acc = {"stamped_rounds": 0, "expand_us": 0.0, "claim_us": 0.0, "exchange_us": 0.0, "status_us": 0.0}
        for i in range(count):
            query(first + i)
            st = eng.last_stats
            for k in acc:
                acc[k] += st[k]
        eng.set_tuning(pipeline=pipeline)
        nr = acc["stamped_rounds"]
        if not nr:
            return {"stamped_rounds_per_query": 0.0}
        per = {k: round(max_over_ranks(acc[k] / nr), 3) for k in ("expand_us", "claim_us", "exchange_us", "status_us")}
        return {"stamped_rounds_per_query": nr / count,
                "kernel_us_per_round": round(per["expand_us"] + per["claim_us"], 3),
                "exchange_us_per_round": per["exchange_us"],
                "status_us_per_round": per["status_us"],
                "expand_us_per_round": per["expand_us"], "claim_us_per_round": per["claim_us"]}

    if a.mode == "partitioned":
        ph, rccl_ranks = run_partitioned(a.graph, a.steps, a.warmup)
        head = {"n": ph["n"], "m": ph["m"], "seed": ph["seed"], "gteps": ph["gteps"],
                "ms_per_step": ph["ms_per_query"], "device_ms_per_query": ph["device_ms_per_query"],
                "gteps_inspected": None, "mean_hops": ph["mean_hops"], "build_ms": ph["build_ms"],
                "batched": None, "partitioned": ph}
    else:
        head = run_replicated(a.graph, a.steps, a.warmup, cpu_ref=True)
        rccl_ranks = None
    extra = {}
    partitioned = {}
    printed = threading.Lock()
    state = {"rccl_ranks": rccl_ranks}

    def emit():
        if rank == 0 and printed.acquire(blocking=False):
            print(json.dumps(report(a, world, head, extra, partitioned, state["rccl_ranks"],
                                    state.get("comm_init_ms"))), flush=True)

    def watchdog():
        # A secondary config that hangs (e.g. a collective that never completes
        # on some rank) must not take the headline measurement with it; the
        # run still fails (non-zero exit) so the hang is not mistaken for success.
        for d in (extra, partitioned):
            for k, v in list(d.items()):
                if v is None:
                    d[k] = {"error": f"watchdog: unfinished after {a.secondary_timeout:.0f} s"}
        emit()
        sys.stdout.flush()
        sys.stderr.write("bench.py: secondary configs unfinished at the watchdog deadline\n")
        rc = exit_status(partitioned, True, a.strict)
        os._exit(3 if rc == 4 else rc)

    dog = threading.Timer(a.secondary_timeout, watchdog)
    dog.daemon = True
    dog.start()
    failed = False
    for spec in filter(None, a.extra_graph.split(",")):
        extra[spec] = None
        try:
            extra[spec] = run_replicated(spec, a.extra_steps, min(a.warmup, 10), cpu_ref=True)
        except Exception as exc:  # report, never hide, a failing secondary config
            extra[spec] = {"error": repr(exc)}
            failed = True
    if a.mode == "replicated" and (world == 1 or comm == "ipc" or (a.dist_backend == "nccl" and not shared_gpu)):
        for spec in filter(None, a.dist_graphs.split(",")):
            # (ranks sharing one GPU -- an IPC rehearsal -- share its HBM: no
            # "bigger than one GPU" graph there)
            spec = world_scaled(spec, 1 if shared_gpu else world, torch.cuda.mem_get_info(dev)[1])
            partitioned[spec] = None
            try:
                partitioned[spec], state["rccl_ranks"] = run_partitioned(spec, a.dist_steps, 3)
                if not partitioned[spec]["verified"]:
                    failed = True
            except Exception as exc:
                partitioned[spec] = {"error": repr(exc)}
                failed = True
    state["comm_init_ms"] = dstate.get("init_ms")

    emit()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    dog.cancel()  # after the teardown: a hung final barrier is covered too
    return exit_status(partitioned, failed, a.strict)


if __name__ == "__main__":
    sys.exit(main())
