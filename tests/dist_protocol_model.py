"""Reference MODEL of the native partitioned engine's round protocol (test-only).

``csrc/dist/dist_engine.hip`` (``DistBiBfs``) is the only multi-GPU engine of
the framework.  This file re-states its round semantics with plain numpy and
``torch.distributed`` collectives so the protocol can be exercised by CPU
processes over ``gloo`` (``tests/test_dist_protocol.py``); it is not a
product path and is never run on GPUs.  Both this model and the native engine
are checked round by round against ``tests/dist_round_spec.py``.

Protocol (reference capability: v4/mpi_bas.cpp:79-132 and the v2 draft's
frontier exchange, v2/main-v2.cpp:59-83):

* 1-D block partition, blocks rounded to 64 vertices: rank r owns
  ``[r * chunk, min(n, (r + 1) * chunk))`` -- its CSR rows and the owned
  slices of both visited sets, parents and frontier queues.
* Per round the replicated policy expands both sides in lockstep while their
  frontiers are comparable, else one side (smaller frontier-edge sum by
  default), each with a direction (Beamer alpha/beta, as the single-GPU engine).
* Top-down: owned frontier vertices claim owned neighbours locally and emit
  ``(v, u)`` candidates for remote owners; ``all_reduce(MAX)`` of the
  candidate count sizes one padded ``all_gather``; owners claim from it
  (lowest parent id wins, so every backend gives the same tree).  A count
  above the capacity switches the level to bottom-up.
* Bottom-up: ``all_gather`` of the owned frontier bitmap slices; every
  unvisited owned vertex scans its row for a frontier neighbour.
* One ``all_reduce(SUM)`` of (new vertices, their degree sum) per side and
  one ``all_reduce(MIN)`` of the meet key (length << 32 | vertex, lengths
  exact from per-vertex depths) end the round; the first round with a meet
  stops the search and its minimum key is the distance.
* The path is walked with one ``all_reduce(MIN)`` per step: the owner of the
  current vertex contributes its parent, every other rank contributes ~0.
* Pipelined rounds (``pipelined=True``; the native ``DistTuning::pipeline``):
  a round's reduction reaches the planner one round late (natively it rides
  the next round's candidate exchange), so round r is planned from the
  rounds up to r - 2 and a meet or an exhausted side found in round r stops
  the search when round r + 1 has already run; the answer is still round r's
  minimum key and the path is unchanged (round r + 1 claims only vertices
  neither chain goes through).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

NONE = np.uint32(0xFFFFFFFF)
NO_KEY = 1 << 62          # meet key (length << 32 | vertex) when no meet
LOCKSTEP_EDGES = 1 << 16  # both frontiers this small (edges): lockstep round (native: kLockstepEdges)
LOCKSTEP_MAX_EDGES = 1 << 20  # balanced frontiers above this: single-side rounds (native: kLockstepMaxEdges)


@dataclass
class DistSearchResult:
    found: bool
    hops: int
    path: List[int]
    meet: int
    levels: int = 0
    sparse_levels: int = 0
    dense_levels: int = 0
    edges_inspected: int = 0
    trace: list = field(default_factory=list)


class TorchDistBiBfs:
    """Collective engine: construct and call ``search`` on every rank of the group."""

    def __init__(self, edges: np.ndarray, n: int, group=None, device=None, candidate_cap: int = 1 << 16,
                 alpha: float = 14.0, beta: float = 24.0):
        import torch
        import torch.distributed as dist

        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.P = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cpu")
        self.n = int(n)
        self.chunk = ((self.n + self.P - 1) // self.P + 63) // 64 * 64
        self.lo = min(self.n, self.rank * self.chunk)
        self.hi = min(self.n, self.lo + self.chunk)
        self.cap = int(candidate_cap)
        self.alpha, self.beta = float(alpha), float(beta)
        e = np.asarray(edges, dtype=np.uint32).reshape(-1, 2)
        e = e[e[:, 0] != e[:, 1]]
        both = np.concatenate([e, e[:, ::-1]], axis=0)
        self.m_input = int(e.shape[0])
        own = (both[:, 0] >= self.lo) & (both[:, 0] < self.hi)
        rows = both[own]
        order = np.argsort(rows[:, 0], kind="stable")
        rows = rows[order]
        cnt = np.bincount(rows[:, 0] - self.lo, minlength=self.hi - self.lo) if self.hi > self.lo else np.zeros(0, np.int64)
        self.row_off = np.zeros(self.hi - self.lo + 1, dtype=np.int64)
        np.cumsum(cnt, out=self.row_off[1:])
        self.col = rows[:, 1].astype(np.int64)
        # global degree of owned vertices (frontier-edge sums for the policy)
        self.deg = np.diff(self.row_off)

    # ---------------------------------------------------------------- collectives
    def _allreduce(self, arr, op):
        t = self.torch.as_tensor(np.asarray(arr, dtype=np.int64), device=self.device)
        self.dist.all_reduce(t, op=op, group=self.group)
        return t.cpu().numpy()

    def _allgather(self, arr: np.ndarray) -> np.ndarray:
        t = self.torch.as_tensor(np.ascontiguousarray(arr, dtype=np.int64), device=self.device)
        out = [self.torch.empty_like(t) for _ in range(self.P)]
        self.dist.all_gather(out, t, group=self.group)
        return np.stack([o.cpu().numpy() for o in out])

    def owner(self, v):
        return np.asarray(v, dtype=np.int64) // self.chunk

    # ---------------------------------------------------------------- search
    def _mode(self, s, direction, dirn, cnt, fed, ved, nnz_total):
        if direction == "topdown":
            return 1
        if direction == "bottomup":
            return 2
        m_u = nnz_total - ved[s]
        if dirn[s] == 1 and fed[s] > m_u / self.alpha:
            dirn[s] = 2
        elif dirn[s] == 2 and cnt[s] < self.n / self.beta:
            dirn[s] = 1
        return dirn[s]

    def _level(self, s, mode, dnew, front, vis, parent, dep, res) -> np.ndarray:
        """One level of side s (same phases as the native engine); returns the
        owned vertices it claimed (sorted global ids)."""
        ROp = self.dist.ReduceOp
        new_local: List[int] = []

        def claim(lv, u):
            vis[s][lv] = True
            parent[s][lv] = int(u)
            dep[s][lv] = dnew
            new_local.append(int(lv + self.lo))

        if mode == 1:
            # local claims + remote candidates
            cand_v, cand_u = [], []
            for u in front[s]:
                lu = u - self.lo
                for v in self.col[self.row_off[lu]:self.row_off[lu + 1]]:
                    if self.lo <= v < self.hi:
                        if not vis[s][v - self.lo]:
                            claim(v - self.lo, u)
                    else:
                        cand_v.append(int(v))
                        cand_u.append(int(u))
            maxc = int(self._allreduce([len(cand_v)], ROp.MAX)[0])
            if maxc > self.cap:
                mode = 2  # finish the level bottom-up; local claims stay valid
                res.dense_levels += 1
            else:
                res.sparse_levels += 1
                if maxc > 0:
                    blk = np.full(1 + 2 * maxc, -1, dtype=np.int64)
                    blk[0] = len(cand_v)
                    blk[1:1 + len(cand_v)] = cand_v
                    blk[1 + maxc:1 + maxc + len(cand_u)] = cand_u
                    allb = self._allgather(blk)
                    got_v = np.concatenate([b[1:1 + b[0]] for b in allb])
                    got_u = np.concatenate([b[1 + maxc:1 + maxc + b[0]] for b in allb])
                    mine = (got_v >= self.lo) & (got_v < self.hi)
                    got_v, got_u = got_v[mine], got_u[mine]
                    order = np.lexsort((got_u, got_v))  # per vertex: lowest parent first
                    for v, u in zip(got_v[order], got_u[order]):
                        if not vis[s][int(v) - self.lo]:
                            claim(int(v) - self.lo, u)
        else:
            res.dense_levels += 1
        if mode == 2:
            fbits = np.zeros(self.chunk, dtype=np.int64)
            fbits[front[s] - self.lo] = 1
            gb = self._allgather(fbits).reshape(-1)  # global frontier membership, index = vertex id
            for lv in np.nonzero(~vis[s])[0]:
                nb = self.col[self.row_off[lv]:self.row_off[lv + 1]]
                hit = nb[gb[nb] == 1] if nb.size else nb
                if hit.size:
                    claim(lv, hit.min())
        return np.array(sorted(new_local), dtype=np.int64)

    def search(self, src: int, dst: int, side: str = "edges", direction: str = "auto",
               want_path: bool = True, lockstep: bool = True, pipelined: bool = False) -> DistSearchResult:
        ROp = self.dist.ReduceOp
        src, dst = int(src), int(dst)
        if src == dst:
            return DistSearchResult(True, 0, [src], src)
        L = self.hi - self.lo
        vis = [np.zeros(L, dtype=bool), np.zeros(L, dtype=bool)]
        parent = [np.full(L, -1, dtype=np.int64), np.full(L, -1, dtype=np.int64)]
        dep = [np.full(L, -1, dtype=np.int64), np.full(L, -1, dtype=np.int64)]
        front: List[np.ndarray] = [np.zeros(0, np.int64), np.zeros(0, np.int64)]  # owned global ids
        root = (src, dst)
        root_deg = [0, 0]
        for s in (0, 1):
            if self.lo <= root[s] < self.hi:
                li = root[s] - self.lo
                vis[s][li] = True
                dep[s][li] = 0
                front[s] = np.array([root[s]], np.int64)
                root_deg[s] = int(self.deg[li])
        rd = self._allreduce(root_deg, ROp.SUM)
        cnt, fed = [1, 1], [int(rd[0]), int(rd[1])]
        ved = list(fed)
        depth, dirn, turn = [0, 0], [1, 1], 0
        res = DistSearchResult(False, -1, [], int(NONE))
        nnz_total = 2 * int(self._allreduce([self.m_input if self.rank == 0 else 0], ROp.SUM)[0])
        key = NO_KEY
        # executed rounds whose reductions the planner has not seen yet:
        # (sides, sums, key, trace rows); accounted one round late when pipelined
        pending = []
        act_cnt, act_fed = list(cnt), list(fed)  # the true frontier sizes (trace records)
        if pipelined:  # the seed's reduction rides round 0's exchange: round 0 is planned blind
            pending.append(([0, 1], [cnt[0], fed[0], cnt[1], fed[1]], NO_KEY, []))
            cnt, fed = [0, 0], [0, 0]
            ved = [0, 0]
        stop = False
        while True:
            while len(pending) > (1 if pipelined else 0):
                psides, psums, pkey, rows = pending.pop(0)
                res.trace += rows
                if pkey != NO_KEY:
                    key = pkey
                    stop = True
                    break
                dead = False
                for s in psides:
                    cnt[s], fed[s] = int(psums[2 * s]), int(psums[2 * s + 1])
                    ved[s] += fed[s]
                    dead = dead or cnt[s] == 0  # that side's component is exhausted
                if dead:
                    stop = True
                    break
            if stop:
                break
            # rounds: both sides in lockstep while their frontiers are comparable
            flo, fhi = min(fed), max(fed)
            if lockstep and side != "alternate" and (fhi <= LOCKSTEP_EDGES or
                                                      (fhi <= 2 * flo and fhi <= LOCKSTEP_MAX_EDGES)):
                sides = [0, 1]
            elif side == "alternate":
                sides, turn = [turn], turn ^ 1
            elif side == "frontier":
                sides = [0 if cnt[0] <= cnt[1] else 1]
            else:
                sides = [0 if fed[0] <= fed[1] else 1]
            new = {}
            for s in sides:
                mode = self._mode(s, direction, dirn, cnt, fed, ved, nnz_total)
                res.edges_inspected += fed[s]
                new[s] = self._level(s, mode, depth[s] + 1, front, vis, parent, dep, res)
                res.levels += 1
            # meet: a vertex claimed this round that the other side holds closes
            # a path of exactly depth_s + depth_o; the round's minimum is the distance
            best = NO_KEY
            for s in sides:
                arr = new[s]
                if arr.size:
                    li = arr - self.lo
                    hit = vis[s ^ 1][li]
                    if hit.any():
                        keys = (depth[s] + 1 + dep[s ^ 1][li[hit]]) * (1 << 32) + arr[hit]
                        best = min(best, int(keys.min()))
            contrib = []
            for s in (0, 1):
                arr = new.get(s)
                contrib += [0, 0] if arr is None else [arr.size, int(self.deg[arr - self.lo].sum()) if arr.size else 0]
            sums = self._allreduce(contrib, ROp.SUM)
            gkey = int(self._allreduce([best], ROp.MIN)[0])
            rows = []
            for s in sides:
                rows.append((s, depth[s], act_cnt[s], act_fed[s], int(sums[2 * s]), len(sides)))
                depth[s] += 1
                front[s] = new[s]
                act_cnt[s], act_fed[s] = int(sums[2 * s]), int(sums[2 * s + 1])
            pending.append((sides, sums, gkey, rows))
        if key == NO_KEY:
            return res
        meet, hops = key & 0xFFFFFFFF, key >> 32
        res.found, res.meet, res.hops = True, meet, hops
        if want_path:
            own = self.lo <= meet < self.hi
            big = int(NONE)
            md = self._allreduce([int(dep[0][meet - self.lo]) if own else big,
                                  int(dep[1][meet - self.lo]) if own else big], ROp.MIN)
            dd = [int(md[0]), int(md[1])]
            assert dd[0] + dd[1] == hops, (dd, hops)
            chains = [[meet], [meet]]
            cur = [meet, meet]
            for i in range(max(dd)):
                contrib = []
                for q in (0, 1):
                    c = big
                    if i < dd[q] and self.lo <= cur[q] < self.hi:
                        c = int(parent[q][cur[q] - self.lo])
                    elif i >= dd[q]:
                        c = cur[q] if self.rank == 0 else big
                    contrib.append(c)
                red = self._allreduce(contrib, ROp.MIN)
                for q in (0, 1):
                    if i < dd[q]:
                        cur[q] = int(red[q])
                        chains[q].append(cur[q])
            res.path = chains[0][::-1] + chains[1][1:]
        return res
