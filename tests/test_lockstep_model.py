"""CPU model of the GPU LDS engine's schedule (csrc/hip/engine_kernels.hip):
lockstep rounds (both sides expand concurrently, claims interleaved in an
arbitrary order), single-side rounds, depth-parity hash keys and the
minimum-candidate meet rule.  Checks the rule itself against BFS distances on
random graphs, independently of the kernel code."""
import random

import numpy as np
import pytest

from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.models import Graph

SMALL = 256


def model_search(csr, s, t, rnd, lockstep=True):
    if s == t:
        return 0
    row, col = csr.row_off, csr.col
    H = [{s: 0}, {t: 0}]  # vertex -> depth parity
    front = [[s], [t]]
    depth = [0, 0]

    def edges(q):
        return sum(int(row[u + 1] - row[u]) for u in front[q])

    while True:
        e0, e1 = edges(0), edges(1)
        lock = lockstep and e0 <= SMALL and e1 <= SMALL
        sides = [0, 1] if lock else [0 if e0 <= e1 else 1]
        # every (side, parent, neighbour) claim attempt of this round, interleaved arbitrarily
        ops = [(q, u, int(v)) for q in sides for u in front[q] for v in col[row[u]:row[u + 1]]]
        rnd.shuffle(ops)
        new = {q: [] for q in sides}
        best = None
        for q, u, v in ops:
            if v in H[q]:
                continue
            a1 = depth[q] + 1
            H[q][v] = a1 & 1
            new[q].append(v)
            o = 1 - q
            if v in H[o]:
                b = depth[o]
                dob = b if H[o][v] == (b & 1) else b + 1
                cand = a1 + dob
                best = cand if best is None else min(best, cand)
        for q in sides:
            depth[q] += 1
            front[q] = new[q]
        if best is not None:
            return best
        if any(not front[q] for q in sides):
            return -1


@pytest.mark.parametrize("seed", range(40))
def test_lockstep_rule_random(seed):
    rnd = random.Random(seed)
    n = rnd.randint(20, 400)
    m = rnd.randint(n // 2, 3 * n)
    e = np.array([[rnd.randrange(n), rnd.randrange(n)] for _ in range(m)], dtype=np.uint32)
    g = Graph.from_edges(n, e)
    for _ in range(10):
        s, t = rnd.randrange(n), rnd.randrange(n)
        expect = native.bfs_oracle(g.csr, s, t).hops
        for lock in (True, False):
            assert model_search(g.csr, s, t, rnd, lock) == expect


def test_lockstep_rule_reference_shape():
    rnd = random.Random(5)
    g = Graph(native.gen_gnp(100000, native.reference_p(100000), 6))
    for _ in range(20):
        s, t = rnd.randrange(g.n), rnd.randrange(g.n)
        assert model_search(g.csr, s, t, rnd) == native.bfs_oracle(g.csr, s, t).hops
