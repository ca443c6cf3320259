"""Serial engine (v1 capability) against independent oracles, incl. the
reference's bugs that must NOT be reproduced."""
import random

import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

from bidirectional_bfs_amd import SerialEngine, native
from bidirectional_bfs_amd.models import Graph, gnp, rmat
from bidirectional_bfs_amd.ops import make_options
from bidirectional_bfs_amd.utils.oracle import check_result, scipy_hops


def run_all_policies(g, s, d):
    out = []
    for side in ("edges", "frontier", "alternate"):
        r = SerialEngine(g).search(s, d, make_options(side=side))
        out.append(r)
    return out


@settings(max_examples=60, deadline=None)
@given(
    n=st.integers(2, 60),
    m=st.integers(0, 120),
    seed=st.integers(0, 10**6),
)
def test_random_graphs_vs_scipy(n, m, seed):
    rng = np.random.default_rng(seed)
    e = rng.integers(0, n, size=(m, 2), dtype=np.uint32)  # duplicates + self loops included
    g = Graph.from_edges(n, e)
    for _ in range(4):
        s, d = int(rng.integers(n)), int(rng.integers(n))
        expect = scipy_hops(n, e[e[:, 0] != e[:, 1]], s, d)
        for r in run_all_policies(g, s, d):
            check_result(g.csr, s, d, r.hops, r.path, expect)


def test_src_equals_dst_is_zero():
    g = gnp(10000, seed=1)
    r = SerialEngine(g).search(5, 5)
    assert r.found and r.hops == 0 and list(r.path) == [5]  # reference v1 printed 2


def test_unreachable_and_isolated():
    g = Graph.from_edges(6, [[0, 1], [1, 2], [3, 4]])
    r = SerialEngine(g).search(0, 4)
    assert not r.found and r.hops == -1 and list(r.path) == []
    r = SerialEngine(g).search(5, 0)  # isolated source
    assert not r.found


def test_path_and_star():
    n = 2000
    path = Graph.from_edges(n, [[i, i + 1] for i in range(n - 1)])
    r = SerialEngine(path).search(0, n - 1)
    assert r.hops == n - 1 and list(r.path) == list(range(n))
    star = Graph.from_edges(n, [[0, i] for i in range(1, n)])
    r = SerialEngine(star).search(7, 1999)
    check_result(star.csr, 7, 1999, r.hops, r.path, 2)


@pytest.mark.parametrize("spec", [("gnp", 100000, 6, 0, 99999, 17), ("gnp", 1000, 1, 0, 999, 9)])
def test_reference_shape(spec):
    _, n, seed, s, d, hops = spec
    g = gnp(n, seed=seed)
    r = SerialEngine(g).search(s, d)
    check_result(g.csr, s, d, r.hops, r.path, hops)


def test_rmat_many_pairs():
    g = rmat(5000, 40000, 3)
    rnd = random.Random(1)
    for _ in range(50):
        s, d = rnd.randrange(5000), rnd.randrange(5000)
        r = SerialEngine(g).search(s, d)
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)


def test_trace_levels_consistent():
    g = gnp(100000, seed=6)
    r = SerialEngine(g).search(0, 99999, make_options(trace=True))
    tr = r.stats["trace"]
    assert len(tr) == r.stats["levels"] and sum(t["edges"] for t in tr) == r.stats["edges_inspected"]
    depth = {0: 0, 1: 0}
    for t in tr:
        assert t["depth"] == depth[t["side"]]
        depth[t["side"]] += 1
    assert depth[0] + depth[1] == r.hops
