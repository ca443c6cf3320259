"""Partitioned bidirectional BFS over ``torch.distributed`` collectives.

This is the same per-level protocol as the RCCL engine
(``csrc/dist/dist_engine.hip``, ``DistBiBfs``) written against
``torch.distributed`` so that it runs on ANY backend: ``gloo`` on CPU
processes (how the protocol is tested without GPUs, ``tests/test_dist_protocol.py``)
or ``nccl`` (= RCCL) with device tensors.  It is the portable multi-process
path; the native engine is the fast one.

Protocol (reference capability: v4/mpi_bas.cpp:79-132 and the v2 draft's
frontier exchange, v2/main-v2.cpp:59-83):

* 1-D block partition, blocks rounded to 64 vertices: rank r owns
  ``[r * chunk, min(n, (r + 1) * chunk))`` -- its CSR rows and the owned
  slices of both visited sets, parents and frontier queues.
* Per level the replicated policy picks a side (smaller frontier-edge sum by
  default) and a direction (Beamer alpha/beta, as the single-GPU engine).
* Top-down: owned frontier vertices claim owned neighbours locally and emit
  ``(v, u)`` candidates for remote owners; ``all_reduce(MAX)`` of the
  candidate count sizes one padded ``all_gather``; owners claim from it
  (lowest parent id wins, so every backend gives the same tree).  A count
  above the capacity switches the level to bottom-up.
* Bottom-up: ``all_gather`` of the owned frontier bitmap slices; every
  unvisited owned vertex scans its row for a frontier neighbour.
* One ``all_reduce(SUM)`` of (new vertices, their degree sum) and one
  ``all_reduce(MIN)`` of the local meet candidate end the level; the first
  level with a meet stops the search (hops = depth_S + depth_T, the
  first-meet argument of SURVEY.md §2.2).
* The path is walked with one ``all_reduce(MIN)`` per step: the owner of the
  current vertex contributes its parent, every other rank contributes ~0.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

NONE = np.uint32(0xFFFFFFFF)


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
    def search(self, src: int, dst: int, side: str = "edges", direction: str = "auto",
               want_path: bool = True) -> DistSearchResult:
        ROp = self.dist.ReduceOp
        src, dst = int(src), int(dst)
        if src == dst:
            return DistSearchResult(True, 0, [src], src)
        L = self.hi - self.lo
        vis = [np.zeros(L, dtype=bool), np.zeros(L, dtype=bool)]
        parent = [np.full(L, -1, dtype=np.int64), np.full(L, -1, dtype=np.int64)]
        front: List[np.ndarray] = [np.zeros(0, np.int64), np.zeros(0, np.int64)]  # owned global ids
        root = (src, dst)
        root_deg = [0, 0]
        for s in (0, 1):
            if self.lo <= root[s] < self.hi:
                li = root[s] - self.lo
                vis[s][li] = True
                front[s] = np.array([root[s]], np.int64)
                root_deg[s] = int(self.deg[li])
        rd = self._allreduce(root_deg, ROp.SUM)
        cnt, fed = [1, 1], [int(rd[0]), int(rd[1])]
        ved = list(fed)
        depth, dirn, turn = [0, 0], [1, 1], 0
        res = DistSearchResult(False, -1, [], int(NONE))
        nnz_total = 2 * int(self._allreduce([self.m_input if self.rank == 0 else 0], ROp.SUM)[0])
        meet = -1
        while True:
            if side == "alternate":
                s, turn = turn, turn ^ 1
            elif side == "frontier":
                s = 0 if cnt[0] <= cnt[1] else 1
            else:
                s = 0 if fed[0] <= fed[1] else 1
            o = s ^ 1
            if direction == "topdown":
                mode = 1
            elif direction == "bottomup":
                mode = 2
            else:
                m_u = nnz_total - ved[s]
                if dirn[s] == 1 and fed[s] > m_u / self.alpha:
                    dirn[s] = 2
                elif dirn[s] == 2 and cnt[s] < self.n / self.beta:
                    dirn[s] = 1
                mode = dirn[s]
            res.edges_inspected += fed[s]
            new_local: List[int] = []
            if mode == 1:
                # local claims + remote candidates
                cand_v, cand_u = [], []
                for u in front[s]:
                    lu = u - self.lo
                    nb = self.col[self.row_off[lu]:self.row_off[lu + 1]]
                    for v in nb:
                        if self.lo <= v < self.hi:
                            lv = v - self.lo
                            if not vis[s][lv]:
                                vis[s][lv] = True
                                parent[s][lv] = u
                                new_local.append(int(v))
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
                            lv = int(v) - self.lo
                            if not vis[s][lv]:
                                vis[s][lv] = True
                                parent[s][lv] = int(u)
                                new_local.append(int(v))
            if mode == 2:
                words = self.chunk
                fbits = np.zeros(words, dtype=np.int64)
                fbits[front[s] - self.lo] = 1
                gb = self._allgather(fbits).reshape(-1)  # global frontier membership, index = vertex id
                for lv in np.nonzero(~vis[s])[0]:
                    nb = self.col[self.row_off[lv]:self.row_off[lv + 1]]
                    hit = nb[gb[nb] == 1] if nb.size else nb
                    if hit.size:
                        vis[s][lv] = True
                        parent[s][lv] = int(hit.min())
                        new_local.append(int(lv + self.lo))
            new_local_arr = np.array(sorted(new_local), dtype=np.int64)
            lm = NONE
            if new_local_arr.size:
                hits = new_local_arr[vis[o][new_local_arr - self.lo]]
                if hits.size:
                    lm = np.uint32(hits.min())
            sums = self._allreduce([new_local_arr.size, int(self.deg[new_local_arr - self.lo].sum()) if new_local_arr.size else 0],
                                   ROp.SUM)
            gmeet = int(self._allreduce([int(lm)], ROp.MIN)[0])
            res.levels += 1
            res.trace.append((s, depth[s], cnt[s], fed[s], int(sums[0]), mode))
            depth[s] += 1
            front[s] = new_local_arr
            if gmeet != int(NONE):
                meet = gmeet
                break
            if int(sums[0]) == 0:
                break
            cnt[s], fed[s] = int(sums[0]), int(sums[1])
            ved[s] += fed[s]
        if meet < 0:
            return res
        res.found, res.meet, res.hops = True, meet, depth[0] + depth[1]
        if want_path:
            chains = [[meet], [meet]]
            cur = [meet, meet]
            for i in range(max(depth)):
                contrib = []
                for q in (0, 1):
                    c = int(NONE)
                    if i < depth[q] and cur[q] != root[q] and self.lo <= cur[q] < self.hi:
                        c = int(parent[q][cur[q] - self.lo])
                    elif i >= depth[q] or cur[q] == root[q]:
                        c = cur[q] if self.rank == 0 else int(NONE)
                    contrib.append(c)
                red = self._allreduce(contrib, ROp.MIN)
                for q in (0, 1):
                    if i < depth[q]:
                        cur[q] = int(red[q])
                        chains[q].append(cur[q])
            res.path = chains[0][::-1] + chains[1][1:]
        return res
