"""Round-by-round specification of the partitioned engine (single process).

Which sides a round expands is a function of the reduced frontier sizes only
(csrc/dist/dist_engine.hip, plan_round): both sides in lockstep while their
frontier degree sums are both <= 2^16 or within 2x, otherwise the side with
the smaller degree sum (or smaller frontier, or strict alternation).  What a
round discovers is a function of the BFS level sets only -- independent of
the partition, the exchange path (candidates, count sync, overflow to
bottom-up) and the direction.  So every engine that implements the protocol
must produce exactly this trace:

    [(side, depth, frontier, frontier_edges, discovered, sides_in_round), ...], hops

The native engine reports it with SearchOptions.trace (stats.trace) and the
gloo model (tests/dist_protocol_model.py) in ``result.trace``.

Pipelined rounds (DistTuning.pipeline, more than one rank): a round's plan is
made before the previous round's claims are reduced, so round r's sides come
from the frontier sizes round r - 1 started with (round 0: none -- both
roots in lockstep, or side 0 when the policy picks one side); the
meet and an exhausted side are still found in the round that has them, so
the trace and the hop count follow the same level sets (``pipelined=True``).
"""
import numpy as np

LOCKSTEP_EDGES = 1 << 16  # dist_engine.hip kLockstepEdges
LOCKSTEP_MAX_EDGES = 1 << 20  # dist_engine.hip kLockstepMaxEdges


def round_trace(csr, src: int, dst: int, side: str = "edges", lockstep: bool = True, pipelined: bool = False):
    row_off = np.asarray(csr.row_off, dtype=np.int64)
    col = np.asarray(csr.col, dtype=np.int64)
    deg = np.diff(row_off)
    src, dst = int(src), int(dst)
    if src == dst:
        return [], 0
    n = len(deg)
    dist = [np.full(n, -1, np.int64), np.full(n, -1, np.int64)]
    dist[0][src] = 0
    dist[1][dst] = 0
    front = [np.array([src], np.int64), np.array([dst], np.int64)]
    cnt, fed, depth, turn = [1, 1], [int(deg[src]), int(deg[dst])], [0, 0], 0
    trace = []
    seen = []  # frontier sizes each round started with
    while True:
        seen.append((list(cnt), list(fed)))
        if pipelined:  # round 0 sees nothing yet (the seed's reduction rides its exchange)
            pc, pf = seen[-2] if len(seen) >= 2 else ([0, 0], [0, 0])
        else:
            pc, pf = cnt, fed
        flo, fhi = min(pf), max(pf)
        if lockstep and side != "alternate" and (fhi <= LOCKSTEP_EDGES or (fhi <= 2 * flo and fhi <= LOCKSTEP_MAX_EDGES)):
            sides = [0, 1]
        elif side == "alternate":
            sides, turn = [turn], turn ^ 1
        elif side == "frontier":
            sides = [0 if pc[0] <= pc[1] else 1]
        else:
            sides = [0 if pf[0] <= pf[1] else 1]
        new = {}
        for s in sides:
            f = front[s]
            nb = np.concatenate([col[row_off[u]:row_off[u + 1]] for u in f]) if f.size else np.zeros(0, np.int64)
            nb = np.unique(nb)
            new[s] = nb[dist[s][nb] < 0]
        for s in sides:
            dist[s][new[s]] = depth[s] + 1
        best = None
        for s in sides:
            hit = new[s][dist[1 - s][new[s]] >= 0]
            if hit.size:
                k = int((depth[s] + 1 + dist[1 - s][hit]).min())
                best = k if best is None else min(best, k)
        for s in sides:
            trace.append((s, depth[s], cnt[s], fed[s], int(new[s].size), len(sides)))
            depth[s] += 1
            front[s] = new[s]
        if best is not None:
            return trace, best
        dead = False
        for s in sides:
            cnt[s], fed[s] = int(new[s].size), int(deg[new[s]].sum())
            dead = dead or cnt[s] == 0
        if dead:
            return trace, -1
