"""The native partitioned engine (csrc/dist/dist_engine.hip) with P > 1 ranks on
ONE GPU: P threads, each a DistBiBfs over its own vertex block, exchanging
through the in-process local group instead of RCCL.
Covers lockstep rounds (exchange overlapped with the opposite expand),
single-side rounds, forced top-down / bottom-up, unreachable pairs and
src == dst, against the CPU oracle."""
import random

import numpy as np
import pytest

import bidirectional_bfs_amd as bb
from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.models import Graph
from bidirectional_bfs_amd.parallel import dist_local_run
from bidirectional_bfs_amd.utils.oracle import check_result

pytestmark = pytest.mark.gpu


def _pairs(n, k, seed):
    rnd = random.Random(seed)
    return [(0, n - 1), (5, 5)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(k)]


@pytest.mark.parametrize("ranks", [2, 3, 4])
@pytest.mark.parametrize("spec", ["gnp:20000::6", "rmat:16384:262144:3"])
def test_local_group_matches_oracle(ranks, spec):
    import torch  # noqa: F401  (binds the HIP runtime first)

    g = bb.from_spec(spec)
    qs = _pairs(g.n, 10, ranks)
    expect = [native.bfs_oracle(g.csr, s, d).hops for s, d in qs]
    for kw in ({}, {"lockstep": False}, {"direction": "topdown"}, {"direction": "bottomup"},
               {"side": "alternate"}, {"side": "frontier", "lockstep": False}):
        rs = dist_local_run(ranks, g, qs, **kw)
        for (s, d), r, e in zip(qs, rs, expect):
            check_result(g.csr, s, d, r.hops, r.path, e)


def test_local_group_disconnected_and_tiny():
    import torch  # noqa: F401

    g = Graph.from_edges(200, [[0, 1], [1, 2], [2, 3], [150, 151], [151, 199]])
    qs = [(0, 3), (3, 0), (0, 199), (150, 199), (7, 8), (199, 150)]
    rs = dist_local_run(4, g, qs)
    for (s, d), r in zip(qs, rs):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)


def test_local_group_long_path():
    import torch  # noqa: F401

    n = 3000
    g = Graph.from_edges(n, np.stack([np.arange(n - 1), np.arange(1, n)], 1).astype(np.uint32))
    rs = dist_local_run(3, g, [(0, n - 1), (17, 2900)])
    assert rs[0].hops == n - 1 and list(rs[0].path) == list(range(n))
    assert rs[1].hops == 2900 - 17


@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("spec", ["kron:14:16:3", "gnp:50000::6"])
def test_local_group_device_generated_shards(ranks, spec):
    """Each rank generates the graph on the device and keeps only its CSR
    shard (the multi-GPU bench path); answers match the host oracle and the
    shards partition the directed edge set."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import dist_local_generate_run

    g = bb.from_spec(spec)  # host generator: same edge list as the device one
    qs = _pairs(g.n, 8, 11)
    rs, t = dist_local_generate_run(ranks, spec, qs)
    for (s, d), r in zip(qs, rs):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
    assert len(t["query_ms"]) == len(qs) and t["build_ms"] > 0
    assert len(t["local_nnz"]) == ranks and sum(t["local_nnz"]) == g.csr.nnz
