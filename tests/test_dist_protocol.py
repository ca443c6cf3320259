"""The partitioned engine's round protocol on CPU processes over gloo: the
test-only model (tests/dist_protocol_model.py) against the serial oracle AND
round by round against the protocol spec (tests/dist_round_spec.py) that the
native engine's GPU tests assert too: top-down candidate exchange, overflow
to bottom-up, Beamer switching, unreachable pairs, path reconstruction."""
import os
import socket
import sys

import numpy as np
import pytest

import bidirectional_bfs_amd as bb
from bidirectional_bfs_amd import native


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, specs, queue):
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from dist_protocol_model import TorchDistBiBfs

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = []
        for spec, cap, pairs, kw in specs:
            g = bb.from_spec(spec)
            eng = TorchDistBiBfs(g.edge_array(), g.n, candidate_cap=cap)
            for s, d in pairs:
                r = eng.search(s, d, **kw)
                out.append((spec, s, d, r.found, r.hops, list(r.path), r.sparse_levels, r.dense_levels,
                            [tuple(int(x) for x in t) for t in r.trace], kw))
        if rank == 0:
            queue.put(out)
    finally:
        dist.destroy_process_group()


def _run(world, specs):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, specs, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    return q.get()


def _pairs(n, k, seed):
    rng = np.random.default_rng(seed)
    return [(0, n - 1)] + [tuple(int(x) for x in rng.integers(0, n, 2)) for _ in range(k)]


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_protocol_matches_oracle(world):
    specs = [
        ("gnp:3000::3", 1 << 16, _pairs(3000, 8, 1), {}),
        ("gnp:3000::3", 4, _pairs(3000, 4, 2), {}),               # tiny capacity: overflow -> bottom-up
        ("rmat:4096:40000:2", 1 << 16, _pairs(4096, 6, 3), {}),   # hubs: Beamer switches to bottom-up
        ("gnp:3000::3", 1 << 16, _pairs(3000, 3, 4), {"direction": "bottomup"}),
        ("gnp:3000::3", 1 << 16, _pairs(3000, 3, 5), {"side": "alternate"}),
        ("gnp:3000::3", 1 << 16, _pairs(3000, 4, 6), {"lockstep": False}),
        ("rmat:4096:40000:2", 4, _pairs(4096, 3, 7), {"lockstep": False}),
        # pipelined rounds (DistTuning.pipeline): lagged plans, one extra round
        ("gnp:3000::3", 1 << 16, _pairs(3000, 8, 8), {"pipelined": True}),
        ("rmat:4096:40000:2", 1 << 16, _pairs(4096, 6, 9), {"pipelined": True}),
        ("gnp:3000::3", 1 << 16, _pairs(3000, 4, 10), {"pipelined": True, "lockstep": False}),
    ]
    out = _run(world, specs)
    graphs = {}
    dense = 0
    from dist_round_spec import round_trace

    for spec, s, d, found, hops, path, sparse_l, dense_l, trace, kw in out:
        g = graphs.setdefault(spec, bb.from_spec(spec))
        o = native.bfs_oracle(g.csr, s, d)
        assert found == o.found and hops == o.hops, (spec, s, d, hops, o.hops)
        want, whops = round_trace(g.csr, s, d, side=kw.get("side", "edges"), lockstep=kw.get("lockstep", True),
                                  pipelined=kw.get("pipelined", False))
        assert trace == want and (whops if whops >= 0 else -1) == (hops if found else -1), (spec, s, d, kw)
        if found:
            ok, why = native.validate_path(g.csr, s, d, hops, path)
            assert ok, (spec, s, d, why)
        dense += dense_l
    assert dense > 0  # the bottom-up exchange was exercised


def test_round_spec_hops_match_oracle():
    """The protocol spec itself: its hop count is the BFS distance, every
    policy, including unreachable pairs and src == dst."""
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from dist_round_spec import round_trace

    for spec in ("gnp:3000::3", "rmat:4096:40000:2"):
        g = bb.from_spec(spec)
        for s, d in _pairs(g.n, 12, 9) + [(5, 5)]:
            o = native.bfs_oracle(g.csr, s, d)
            for kw in ({}, {"lockstep": False}, {"side": "alternate"}, {"side": "frontier", "lockstep": False},
                       {"pipelined": True}, {"pipelined": True, "lockstep": False}):
                trace, hops = round_trace(g.csr, s, d, **kw)
                assert hops == (o.hops if o.found else -1), (spec, s, d, kw)
                if s != d:
                    assert trace and trace[0][1] == 0  # first expansion starts at depth 0
