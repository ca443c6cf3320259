#!/usr/bin/env python3
"""Partitioned-engine stress on the in-process local group (P ranks on one
GPU, each generating its own shard): many queries per (graph, P), hop counts
against this repo's CPU engine on the same generated graph, every found path
validated collectively by the owners of its vertices (verify).

    python benchmarks/stress_dist_local.py [--specs gnp:1000000::2,kron:20:16:1] [--ranks 2,3,4,8] [--queries 256]

--procs: the ranks are separate processes over the IPC transport
(parallel.dist_proc_matrix), every option set of --option-sets per group.
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", default="gnp:1000000::2,kron:20:16:1,rmat:262144:4194304:4")
    ap.add_argument("--ranks", default="2,3,4,8")
    ap.add_argument("--queries", type=int, default=256)
    ap.add_argument("--pipeline", type=int, default=1)
    ap.add_argument("--procs", action="store_true", help="ranks as processes over the IPC transport")
    a = ap.parse_args()
    import torch  # noqa: F401
    import bidirectional_bfs_amd as bb
    from bidirectional_bfs_amd import native
    from bidirectional_bfs_amd.models import parse_spec
    from bidirectional_bfs_amd.parallel import dist_local_generate_run, dist_proc_matrix, make_tuning

    rc = 0
    for spec in a.specs.split(","):
        g = bb.from_spec(spec)  # the same seeded generator the ranks run on the device
        cpu = native.SerialBiBfs(g.csr)
        _, n, _, _ = parse_spec(spec)
        rnd = random.Random(3)
        qs = [(rnd.randrange(n), rnd.randrange(n)) for _ in range(a.queries)]
        truth = [cpu.query(s, d)[0] for s, d in qs]
        for P in [int(x) for x in a.ranks.split(",")]:
            t0 = time.perf_counter()
            if a.procs:
                got, _ = dist_proc_matrix(P, spec, qs, [({}, {"pipeline": bool(a.pipeline)})], verify=8)
                rs, _, run = got[0]
                t = {"path_valid": run["path_valid"], "uni_hops": run["uni_hops"]}
            else:
                rs, t = dist_local_generate_run(P, spec, qs, tuning=make_tuning(pipeline=bool(a.pipeline)), verify=8)
            dt = time.perf_counter() - t0
            wrong = sum(1 for r, h in zip(rs, truth) if (r.hops if r.found else -1) != h)
            bad_paths = sum(1 for ok in t.get("path_valid", []) if ok == 0)  # 1 valid, -1 no path
            uni = [(u, h) for u, h in zip(t.get("uni_hops", []), truth) if u != -2]  # -2: not re-run
            uni_bad = sum(1 for u, h in uni if u != h)
            rec = {"spec": spec, "ranks": P, "transport": "ipc-processes" if a.procs else "local-threads",
                   "pipeline": bool(a.pipeline), "queries": len(qs), "wrong_hops": wrong, "bad_paths": bad_paths,
                   "uni_checked": len(uni), "uni_wrong": uni_bad, "wall_s": round(dt, 2)}
            print(json.dumps(rec), flush=True)
            if wrong or bad_paths or uni_bad:
                rc = 1
    return rc


if __name__ == "__main__":
    sys.exit(main())
