"""Cost of the multi-process IPC transport (csrc/dist/ipc_comm.hip) per
collective and per query, by HIP runtime: Python workers that import torch
first (torch's bundled HIP runtime) or not (/opt/rocm's), and mpi_bibfs
(/opt/rocm's).  BIBFS_IPC_STATS=1 makes every rank print its mean host time
per collective (stream wait = own stream reaching the collective; rendezvous
= waiting for the peers).  One JSON line per setup.

    python benchmarks/ipc_transport.py [--spec gnp:1000000::2] [--ranks 2,4] [--queries 16]
"""
import argparse
import json
import os
import random
import re
import statistics
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bidirectional_bfs_amd.models import parse_spec  # noqa: E402
from bidirectional_bfs_amd.parallel import MPIEXEC, dist_proc_launch  # noqa: E402

STAT = re.compile(r"\[ipc rank (\d+)\] (\d+) collectives: ([\d.]+) us mean stream wait, ([\d.]+) us mean rendezvous, "
                  r"([\d.]+) us mean host time")


def stats_of(text):
    rows = [tuple(float(x) for x in m.groups()) for m in STAT.finditer(text)]
    if not rows:
        return {}
    return {"collectives": int(rows[0][1]),
            "stream_wait_us": round(statistics.mean(r[2] for r in rows), 2),
            "rendezvous_us": round(statistics.mean(r[3] for r in rows), 2),
            "host_us_per_collective": round(statistics.mean(r[4] for r in rows), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="gnp:1000000::2")
    ap.add_argument("--ranks", default="2,4")
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--torch", default="0,1", help="BIBFS_PROC_TORCH values: 0 no torch, 1 imported, 2 + device context")
    a = ap.parse_args()
    _, n, _, _ = parse_spec(a.spec)
    rnd = random.Random(3)
    qs = [(0, n - 1)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(a.queries - 1)]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for P in [int(x) for x in a.ranks.split(",")]:
        for torch_first in a.torch.split(","):
            env = {"BIBFS_PROC_TORCH": torch_first, "BIBFS_IPC_STATS": "1"}
            rcs, outs, el = dist_proc_launch(P, a.spec, qs, [({}, {}), ({}, {})], env=env, timeout=300)
            run = outs[0]["runs"][-1] if "runs" in outs[0] else {}
            ms = run.get("query_ms", [])
            rec = {"setup": {"0": "python workers, /opt/rocm runtime", "1": "python workers, torch runtime",
                             "2": "python workers, torch runtime + torch device context"}[torch_first],
                   "ranks": P, "spec": a.spec, "rcs": rcs,
                   "median_query_ms": round(statistics.median(ms), 4) if ms else None,
                   "mean_rounds": round(statistics.mean(st.get("rounds", 0) for st in run.get("last_stats", [{}])), 2)
                   if run.get("last_stats") else None}
            rec.update(stats_of("".join(o.get("log", "") for o in outs)))
            errs = [o.get("error") for o in outs if o.get("error")]
            if errs:
                rec["errors"] = errs[:2]
            print(json.dumps(rec), flush=True)
        cmd = [MPIEXEC, "-n", str(P), os.path.join(root, "build", "bin", "mpi_bibfs"), a.spec, "0", str(n - 1),
               "--comm", "ipc", "--repeat", "20", "--json"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, BIBFS_IPC_STATS="1"))
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        rec = {"setup": "mpi_bibfs, /opt/rocm runtime", "ranks": P, "spec": a.spec, "rc": r.returncode}
        if line:
            d = json.loads(line[-1])
            rec["median_query_ms"] = d.get("query_ms")
        rec.update(stats_of(r.stderr))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
