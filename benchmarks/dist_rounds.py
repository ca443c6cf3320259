#!/usr/bin/env python3
"""Where a partitioned round's time goes: kernel vs exchange, per round.

P ranks run as threads of this process on ONE GPU (the in-process local
group, csrc/dist/comm.hip), each generating its own CSR shard, with
DistTuning.stamps on: every speculative round records s_memrealtime at the
entry and the last-workgroup exit of its expansion launch(es) and of its
claim launch (csrc/dist/dist_engine.hip, RoundStamp).  Per round:

  expand_us    k_spec_expand (+ k_td_hubs) on this rank
  claim_us     k_spec_claim
  exchange_us  expansion end -> claim start: the owner-addressed candidate
               exchange (here device-to-device copies between the ranks'
               streams; RCCL send/recv on a node) plus the launch gap
  status_us    claim end -> next expansion start: the status allgather plus
               the launch gap (pipelined rounds, the default with P > 1: the
               launch gap alone -- the status travels with the next exchange)

Rank 0's numbers, median over queries of the per-round means.  The ranks
share the GPU's CUs, so kernel times are an upper bound for one rank per
GPU; the exchange column is the local group's copies, not xGMI.

    python benchmarks/dist_rounds.py --specs gnp:1000000::2,kron:22 --ranks 1,2,4 --pipeline 1,0

--procs runs the ranks as separate PROCESSES over the HIP-IPC transport
(csrc/dist/ipc_comm.hip, parallel.dist_proc_matrix) instead of threads of one
process: every collective is then a host rendezvous between processes plus a
pull kernel, the cost a round pays between processes on one GPU.
"""
import argparse
import json
import random
import statistics
import sys

import torch  # noqa: F401  (binds the HIP runtime first)

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from bidirectional_bfs_amd.models import parse_spec  # noqa: E402
from bidirectional_bfs_amd.parallel import dist_local_generate_run, dist_proc_matrix, make_tuning  # noqa: E402


def per_round(stats, key):
    vals = [st[key] / st["stamped_rounds"] for st in stats if st["stamped_rounds"]]
    return round(statistics.median(vals), 3) if vals else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--specs", default="gnp:1000000::2,kron:22")
    ap.add_argument("--ranks", default="1,2,4")
    ap.add_argument("--pipeline", default="1,0", help="DistTuning.pipeline values to run (P > 1)")
    ap.add_argument("--queries", type=int, default=24)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--solo", type=int, default=1, help="P = 1: 0 runs the multi-workgroup rounds (stampable)")
    ap.add_argument("--procs", action="store_true", help="ranks as processes over the IPC transport")
    ap.add_argument("--dev-sync", default="1", help="DistTuning.dev_sync values to run (IPC processes)")
    a = ap.parse_args()
    for spec in a.specs.split(","):
        _, n, _, _ = parse_spec(spec)
        rnd = random.Random(a.seed)
        qs = [(rnd.randrange(n), rnd.randrange(n)) for _ in range(a.queries)]
        for ranks in [int(x) for x in a.ranks.split(",")]:
            for pv, dv in [(int(x), int(y)) for x in a.pipeline.split(",") for y in a.dev_sync.split(",")]:
                if not pv and ranks == 1:
                    continue
                if a.procs:
                    tk = {"stamps": True, "pipeline": bool(pv), "solo": bool(a.solo), "dev_sync": bool(dv)}
                    got, _ = dist_proc_matrix(ranks, spec, qs, [({}, tk)])
                    rs, st0, run = got[0]
                    t = {"query_ms": run["query_ms"], "stats": st0}
                else:
                    tun = make_tuning(stamps=True, pipeline=bool(pv), solo=bool(a.solo), dev_sync=bool(dv))
                    rs, t = dist_local_generate_run(ranks, spec, qs, tuning=tun)
                keep = [(r, ms, st) for r, ms, st in zip(rs, t["query_ms"], t["stats"]) if r.found and r.hops > 0]
                sts = [st for _, _, st in keep]
                rec = {
                    "spec": spec, "ranks": ranks, "pipeline": bool(pv) and ranks > 1, "queries": len(keep),
                    "transport": "ipc-processes" if a.procs else "local-threads", "dev_sync": bool(dv),
                    "dev_sync_rounds_per_query": (round(statistics.mean(st["dev_sync_rounds"] for st in sts), 2)
                                                  if sts else None),
                    "median_query_ms": round(statistics.median(ms for _, ms, _ in keep), 4) if keep else None,
                    "mean_rounds": round(statistics.mean(st["rounds"] for st in sts), 2) if sts else None,
                    "mean_stamped_rounds": round(statistics.mean(st["stamped_rounds"] for st in sts), 2) if sts else None,
                    # collectives of the whole search (seed gather, rounds, path gather) per
                    # accounted round, and per enqueued round (pipelined: +1 round at the end)
                    "collectives_per_round": (round(sum(st["collectives"] for st in sts) /
                                                    max(1, sum(st["rounds"] for st in sts)), 3) if sts else None),
                    "collectives_per_query": round(statistics.mean(st["collectives"] for st in sts), 2) if sts else None,
                    "spec_rounds_per_query": round(statistics.mean(st["spec_rounds"] for st in sts), 2) if sts else None,
                    "pipe_drains": sum(st["pipe_drains"] for st in sts),
                    "expand_us_per_round": per_round(sts, "expand_us"),
                    "claim_us_per_round": per_round(sts, "claim_us"),
                    "exchange_us_per_round": per_round(sts, "exchange_us"),
                    "status_us_per_round": per_round(sts, "status_us"),
                    "small_expand_rounds": sum(st["small_expand_rounds"] for st in sts),
                    "small_claim_rounds": sum(st["small_claim_rounds"] for st in sts),
                    "host_rounds": sum(st["host_rounds"] for st in sts),
                    "solo_rounds": sum(st["solo_rounds"] for st in sts),
                    "walk_insert_us_per_query": round(statistics.mean(st.get("walk_insert_us", 0.0) for st in sts), 2) if sts else None,
                    "walk_chain_us_per_query": round(statistics.mean(st.get("walk_chain_us", 0.0) for st in sts), 2) if sts else None,
                }
                for k, nk in (("sx_plan_us", "small_expand_rounds"), ("sx_staging_us", "small_expand_rounds"),
                              ("sx_stage_us", "small_expand_rounds"),
                              ("sx_edges_us", "small_expand_rounds"), ("sx_end_us", "small_expand_rounds"),
                              ("sc_claims_us", "small_claim_rounds"), ("sc_end_us", "small_claim_rounds")):
                    tot, cnt = sum(st[k] for st in sts), sum(st[nk] for st in sts)
                    rec[k + "_per_small_round"] = round(tot / cnt, 3) if cnt else None
                if rec["expand_us_per_round"] is not None:
                    rec["kernel_us_per_round"] = round(rec["expand_us_per_round"] + (rec["claim_us_per_round"] or 0), 3)
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
