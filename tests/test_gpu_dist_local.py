"""The native partitioned engine (csrc/dist/dist_engine.hip) with P > 1 ranks on
ONE GPU: P threads, each a DistBiBfs over its own vertex block, exchanging
through the in-process local group instead of RCCL.
Covers lockstep rounds, pipelined rounds (one collective per round),
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


# ---- device-planned speculative rounds, exchange branches, failure paths ----

def _check_all(g, qs, rs):
    for (s, d), r in zip(qs, rs):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)


@pytest.mark.parametrize("spec_rounds", [0, 1, 4, 8])
def test_speculative_rounds_match_oracle_and_cut_host_syncs(spec_rounds):
    """spec_rounds = 0 plans every round on the host (one wait per round); K > 0
    enqueues K device-planned rounds per wait."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    g = bb.from_spec("gnp:100000::6")
    qs = _pairs(g.n, 12, 21)
    rs, st = dist_local_run(2, g, qs, tuning=make_tuning(spec_rounds=spec_rounds), return_stats=True)
    _check_all(g, qs, rs)
    for (s, d), r, x in zip(qs, rs, st):
        if s == d or not r.found:
            continue
        if spec_rounds == 0:
            assert x["spec_rounds"] == 0 and x["host_rounds"] == x["rounds"]
        else:
            # one wait per batch of K rounds, + the path walk and the final cleanup wait
            batches = -(-x["rounds"] // spec_rounds) + 1
            assert x["host_syncs"] <= batches + 2 + x["host_rounds"], x
            assert x["path_collectives"] == 1, x  # ONE allgather for the whole path


@pytest.mark.parametrize("ranks", [1, 2, 4])
def test_tiny_capacities_force_count_sync_and_overflow(ranks):
    """A 4-pair candidate block and no host-bound sizing: big sparse levels stall
    the speculative batch, the host sizes the exchange with a count allreduce,
    and counts above the block finish the level bottom-up."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    # (exact plans: a pipelined search sees a level's size two rounds late and
    # often meets before its drain reaches the host-planned round)
    tune = make_tuning(cap=4, nosync_bytes=0, spec_cap_max=1024, spec_stall_edges=1024, world1_single=False,
                       pipeline=False)
    seen = {"host_rounds": 0, "count_syncs": 0, "overflow_levels": 0}
    for spec in ("kron:14:16:3", "gnp:20000::6"):
        g = bb.from_spec(spec)
        qs = _pairs(g.n, 10, 5)
        for kw in ({}, {"lockstep": False}, {"direction": "topdown"}):
            rs, st = dist_local_run(ranks, g, qs, tuning=tune, return_stats=True, **kw)
            _check_all(g, qs, rs)
            for k in seen:
                seen[k] += sum(x[k] for x in st)
    assert seen["host_rounds"] > 0 and seen["count_syncs"] > 0, seen
    if ranks > 1:  # one rank owns every vertex: nothing is ever offered, nothing overflows
        assert seen["overflow_levels"] > 0, seen


def test_path_walk_fallback_per_hop():
    """Visited sets above walk_max: the path is rebuilt hop by hop (one
    allreduce per hop) instead of from one gathered parent table."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    g = bb.from_spec("gnp:20000::6")
    qs = _pairs(g.n, 8, 9)
    rs, st = dist_local_run(3, g, qs, tuning=make_tuning(walk_max=1), return_stats=True)
    _check_all(g, qs, rs)
    assert any(x["path_collectives"] > 1 for x, r in zip(st, rs) if r.found and r.hops > 1)


@pytest.mark.parametrize("mode", [1, 2])
def test_failing_rank_aborts_every_rank(mode):
    """Rank 1 throws (mode 1) or hangs past the watchdog (mode 2) mid-search:
    the group is torn down and the run reports the failure instead of hanging."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    g = bb.from_spec("gnp:20000::6")
    qs = _pairs(g.n, 3, 2)
    with pytest.raises(RuntimeError) as ei:
        dist_local_run(3, g, qs, tuning=make_tuning(timeout_s=1.0), fault=(1, 2, mode))
    msg = str(ei.value)
    assert "injected fault" in msg or "timed out" in msg or "aborted" in msg, msg


@pytest.mark.parametrize("ranks", [1, 2, 3])
@pytest.mark.parametrize("spec_rounds", [0, 4])
def test_native_rounds_follow_protocol_spec(ranks, spec_rounds):
    """Round by round, the native engine expands the sides the protocol spec
    says and discovers what the BFS levels say (tests/dist_round_spec.py --
    the same spec the CPU model is held to in tests/test_dist_protocol.py),
    whether rounds are planned on the device or on the host, and through
    tiny exchange blocks (count syncs, overflow to bottom-up).  Exact plans
    follow the exact spec; pipelined plans (P > 1, the default) the spec's
    lagged side choice -- unless the search drained to exact plans, where
    the hop count is still checked."""
    import torch  # noqa: F401
    from dist_round_spec import round_trace

    from bidirectional_bfs_amd.parallel import make_tuning

    for spec in ("gnp:20000::6", "rmat:16384:262144:3"):
        g = bb.from_spec(spec)
        qs = _pairs(g.n, 6, 13)
        for kw in ({}, {"lockstep": False}, {"side": "alternate"}, {"side": "frontier", "lockstep": False},
                   {"direction": "bottomup"}):
            # (world1_single off: one rank runs the partitioned rounds too)
            for tune in (make_tuning(spec_rounds=spec_rounds, world1_single=False, pipeline=False),
                         make_tuning(spec_rounds=spec_rounds, cap=4, nosync_bytes=0, spec_stall_edges=64,
                                     world1_single=False, pipeline=False),
                         make_tuning(spec_rounds=spec_rounds, owner_cap=2, world1_single=False, pipeline=False),
                         make_tuning(spec_rounds=spec_rounds, world1_single=False),
                         make_tuning(spec_rounds=spec_rounds, owner_cap=64, world1_single=False)):
                rs, st = dist_local_run(ranks, g, qs, tuning=tune, trace=True, return_stats=True, **kw)
                for (s, d), r, x in zip(qs, rs, st):
                    # (pipelining needs a one-round lookahead and a graph without hubs)
                    piped = bool(x["pipelined"])
                    if spec.startswith("gnp") and tune.pipeline and ranks > 1 and spec_rounds == 1 and s != d:
                        assert piped, (spec, s, d, kw)
                    want, hops = round_trace(g.csr, s, d, side=kw.get("side", "edges"),
                                             lockstep=kw.get("lockstep", True), pipelined=piped)
                    if piped and (x["pipe_drains"] or x["host_rounds"]):
                        assert r.hops == hops, (spec, s, d, kw, r.hops, hops)  # pipelined, then exact plans
                        continue
                    got = [(t["side"], t["depth"], t["frontier"], t["edges"], t["discovered"]) for t in r.stats["trace"]]
                    exp = [w[:5] for w in want]
                    # a single-side level stops at its first meet (every meet of such a
                    # level has the same length): the meeting round may discover less
                    if got and exp and len(got) == len(exp) and got[-1][4] < exp[-1][4]:
                        assert got[-1][:4] == exp[-1][:4] and 0 < got[-1][4], (spec, s, d, kw, got[-1], exp[-1])
                        got, exp = got[:-1], exp[:-1]
                    assert got == exp, (spec, s, d, kw)
                    assert r.hops == hops, (spec, s, d, r.hops, hops)


def test_out_of_range_query_keeps_group_serving():
    """A bad query raises on every rank before any collective and does not
    abort the communicator: the next valid query still gets the oracle's answer."""
    import torch  # noqa: F401

    g = bb.from_spec("gnp:20000::6")
    qs = [(0, g.n - 1), (g.n + 5, 3), (3, g.n), (17, 4242), (0, g.n - 1)]
    rs = dist_local_run(3, g, qs)
    assert rs[1].hops == -2 and rs[2].hops == -2
    for i in (0, 3, 4):
        s, d = qs[i]
        check_result(g.csr, s, d, rs[i].hops, rs[i].path, native.bfs_oracle(g.csr, s, d).hops)


@pytest.mark.parametrize("spec", ["gnp:40000::3", "kron:15:16:2"])
def test_generated_shards_hold_only_their_rows(spec):
    """Every rank generates its shard straight from the generator: its peak
    allocation is its own rows (+ one cursor array), never the edge list."""
    import torch  # noqa: F401

    from bidirectional_bfs_amd.parallel import dist_local_generate_run

    g = bb.from_spec(spec)
    qs = _pairs(g.n, 6, 4)
    rs, t = dist_local_generate_run(3, spec, qs)
    for (s, d), r in zip(qs, rs):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
    edge_list_bytes = 8 * g.m
    for nnz, shard, peak in zip(t["local_nnz"], t["shard_bytes"], t["gen_peak_bytes"]):
        rows = (g.n + 2) // 3 + 64
        assert shard <= nnz * 4 + (rows + 1) * 8
        assert peak <= shard + (rows + 1) * 8
        assert peak < edge_list_bytes  # the old path held the whole edge list on every rank
    assert sum(t["local_nnz"]) == g.csr.nnz


# ---- one rank: the solo workgroup (k_spec_solo), its hand-off and the terminal walk ----

@pytest.mark.parametrize("spec", ["gnp:20000::6", "kron:14:16:3", "rmat:16384:262144:3"])
def test_world1_solo_matches_oracle_and_hands_off(spec):
    """One rank: the solo workgroup runs the small rounds, hands big frontiers
    (Kronecker hubs) and bottom-up plans to the multi-workgroup / host rounds,
    and the round that ends the search walks the path into pinned memory.
    Every option combination against the oracle, solo on and off."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    g = bb.from_spec(spec)
    qs = _pairs(g.n, 12, 21)
    expect = [native.bfs_oracle(g.csr, s, d).hops for s, d in qs]
    for solo in (True, False):
        for kw in ({}, {"lockstep": False}, {"direction": "bottomup"}, {"side": "alternate"},
                   {"want_path": False}):
            rs, st = dist_local_run(1, g, qs, tuning=make_tuning(solo=solo, world1_single=False), return_stats=True,
                                    **kw)
            for (s, d), r, e in zip(qs, rs, expect):
                if kw.get("want_path") is False:
                    assert r.hops == e, (s, d, r.hops, e)
                else:
                    check_result(g.csr, s, d, r.hops, r.path, e)
            if solo and not kw:
                assert any(x["solo_rounds"] > 0 for x in st), st[:3]
            if not solo:
                assert all(x["solo_rounds"] == 0 for x in st)


def test_world1_solo_long_path_and_disconnected():
    """A 5000-hop path (one vertex per frontier: every round in the one
    launch) and unreachable pairs (a side exhausted inside the solo loop)."""
    import torch  # noqa: F401

    n = 5000
    line = np.stack([np.arange(n - 1), np.arange(1, n)], 1).astype(np.uint32)
    g = Graph.from_edges(n + 3, np.concatenate([line, np.array([[n, n + 1]], np.uint32)]))
    from bidirectional_bfs_amd.parallel import make_tuning

    rs, st = dist_local_run(1, g, [(0, n - 1), (17, 2900), (0, n + 1), (n + 2, 3)], return_stats=True,
                            tuning=make_tuning(world1_single=False))
    assert rs[0].hops == n - 1 and list(rs[0].path) == list(range(n))
    assert rs[1].hops == 2900 - 17 and list(rs[1].path) == list(range(17, 2901))
    assert not rs[2].found and not rs[3].found
    assert st[0]["solo_rounds"] >= (n - 1) // 2 and st[0]["host_rounds"] == 0


def test_world1_back_to_back_queries_keep_state_clean():
    """No host wait for the state reset between searches (k_cleanup trails in
    the stream): many back-to-back queries, alternating roots, stay exact."""
    import torch  # noqa: F401

    g = bb.from_spec("gnp:30000::4")
    rnd = random.Random(5)
    qs = [(rnd.randrange(g.n), rnd.randrange(g.n)) for _ in range(60)]
    from bidirectional_bfs_amd.parallel import make_tuning

    for single in (False, True):
        rs, st = dist_local_run(1, g, qs, tuning=make_tuning(world1_single=single), return_stats=True)
        for (s, d), r in zip(qs, rs):
            check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
        # world1_single: the rank's CSR is served by the single-GPU engine (no rounds)
        assert all(x["single_engine"] == (1 if single else 0) for x in st if x["levels"])


@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_owner_blocks_overflow_into_continuation_rounds(ranks):
    """Owner-addressed exchange with 2-pair blocks: candidates that do not fit
    their owner's block are re-offered by continuation rounds (same level, no
    expansion) until every one is claimed; answers stay exact and meets found
    before the level completes wait for it (the level's minimum)."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    cont = 0
    for spec in ("gnp:20000::6", "kron:14:16:3"):
        g = bb.from_spec(spec)
        qs = _pairs(g.n, 10, 17)
        for kw in ({}, {"lockstep": False}, {"side": "alternate"}, {"direction": "topdown"}):
            rs, st = dist_local_run(ranks, g, qs, tuning=make_tuning(owner_cap=2), return_stats=True, **kw)
            _check_all(g, qs, rs)
            cont += sum(x["cont_rounds"] for x in st)
    assert cont > 0


def test_owner_addressed_exchange_moves_only_addressed_bytes():
    """Default sizing: the bytes a rank receives per query are the blocks
    addressed to it (plus the per-round status), far below P full candidate
    blocks per round."""
    import torch  # noqa: F401

    g = bb.from_spec("gnp:100000::6")
    qs = _pairs(g.n, 8, 3)
    for ranks in (2, 4):
        rs, st = dist_local_run(ranks, g, qs, return_stats=True)
        _check_all(g, qs, rs)
        for x, r in zip(st, rs):
            if r.found and r.hops > 2:
                # a 256-pair block per owner and side at most once per round, in the worst case
                assert x["exchanged_bytes"] <= x["rounds"] * (ranks - 1) * 2 * (2 + 2 * 4096) * 4 + 65536, x


@pytest.mark.parametrize("ranks", [2, 3, 4])
def test_pipeline_on_and_off_match_oracle_and_count_collectives(ranks):
    """DistTuning.pipeline: with it (the default) a speculative round is ONE
    collective -- the candidate exchange carries the previous round's
    reduction -- and without it two (exchange + status allgather); answers
    match the oracle either way.  Hub graphs run exact plans (the engine's
    choice); bottom-up drains the pipeline (the first stall) and finishes
    with exact plans."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    for spec in ("gnp:20000::6", "gnp:200000::3", "rmat:16384:262144:3"):
        g = bb.from_spec(spec)
        qs = _pairs(g.n, 10, 29)
        for kw in ({}, {"lockstep": False}, {"direction": "bottomup"}):
            per = {}
            for pipe in (True, False):
                rs, st = dist_local_run(ranks, g, qs, tuning=make_tuning(pipeline=pipe), return_stats=True, **kw)
                _check_all(g, qs, rs)
                sr = sum(x["spec_rounds"] for x in st)
                per[pipe] = (sum(x["collectives"] for x in st), sr, sum(x["pipe_drains"] + x["host_rounds"] for x in st))
            if spec.startswith("gnp") and not kw:
                coll, sr, drained = per[True]
                assert drained == 0, (spec, per)
                # one collective per enqueued round, plus the seed's gather and the path's
                assert coll <= sr + 2 * len(qs), (spec, per)
                assert per[False][0] >= 2 * per[False][1], (spec, per)


def test_pipeline_drains_on_spills_to_continuation_rounds():
    """2-pair owner blocks spill in the first pipelined round: the next plan
    stalls, the host drains the pipeline (the pending round accounted
    exactly) and continuation rounds complete the level -- hop counts and
    paths still exact."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    g = bb.from_spec("gnp:50000::8")
    qs = _pairs(g.n, 12, 77)
    rs, st = dist_local_run(3, g, qs, tuning=make_tuning(owner_cap=2), return_stats=True)
    _check_all(g, qs, rs)
    assert sum(x["pipe_drains"] for x in st) > 0
    assert sum(x["cont_rounds"] for x in st) > 0


@pytest.mark.parametrize("ranks", [2, 4])
def test_round_stamps_split_kernel_and_exchange(ranks):
    """DistTuning.stamps: the speculative rounds of a P > 1 search are stamped
    (expansion / claim kernels, and the gaps the exchanges leave between
    them); answers unchanged, pipelined rounds and exact plans."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import make_tuning

    g = bb.from_spec("gnp:200000::5")
    qs = _pairs(g.n, 8, 41)
    for pipe in (False, True):
        rs, st = dist_local_run(ranks, g, qs, tuning=make_tuning(stamps=True, pipeline=pipe), return_stats=True)
        _check_all(g, qs, rs)
        stamped = [x for r, x in zip(rs, st) if r.found and r.hops > 2]
        assert stamped and all(x["stamped_rounds"] > 0 for x in stamped)
        for x in stamped:
            assert x["stamped_rounds"] <= x["spec_rounds"]
            assert x["expand_us"] > 0 and x["claim_us"] > 0 and x["exchange_us"] >= 0 and x["status_us"] >= 0
            # microseconds per round, not garbage from a stale ring slot
            assert (x["expand_us"] + x["claim_us"]) / x["stamped_rounds"] < 50000


def test_capped_hbm_graph_only_partitioned_and_verified_without_copy():
    """A graph that does not fit one rank's (artificially capped) HBM: the
    one-rank build is refused, the 4-rank build holds it (the shards together
    exceed the cap), and its answers are verified with no full copy of the
    graph on the device: paths edge by edge by the owners (validate_path) and
    hop counts by a unidirectional partitioned BFS -- both also held to the
    host oracle here.  The build's peak is measured per allocation."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import dist_local_generate_run, make_tuning

    spec = "rmat:65536:16777216:3"  # 33.5M directed entries: ~134 MB of columns
    cap = 80 << 20
    qs = _pairs(65536, 6, 53)[2:] + [(0, 65535)]
    with pytest.raises(RuntimeError, match="HBM cap"):
        dist_local_generate_run(1, spec, qs[:1], tuning=make_tuning(hbm_cap_bytes=cap))
    rs, t = dist_local_generate_run(4, spec, qs, tuning=make_tuning(hbm_cap_bytes=cap), verify=4)
    assert sum(t["shard_bytes"]) > cap, t["shard_bytes"]
    assert max(t["resident_bytes"]) <= cap
    for sb, pk, rb in zip(t["shard_bytes"], t["gen_peak_bytes"], t["resident_bytes"]):
        # measured, not a formula: the build held at least the shard plus the
        # scatter cursor at once; afterwards the shard plus search state
        assert sb + 65536 // 4 * 8 <= pk <= cap and sb < rb <= cap, (sb, pk, rb)
    g = bb.from_spec(spec)
    for i, ((s, d), r) in enumerate(zip(qs, rs)):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
        assert t["path_valid"][i] == (1 if r.found else -1)
        if i < 4:
            assert t["uni_hops"][i] == r.hops


def test_eight_rank_rehearsal_of_the_bench_path():
    """The bench's multi-GPU partitioned path rehearsed with 8 ranks on one GPU:
    device-generated shards, small and multi-workgroup rounds, stamps, and the
    distributed checks (path per owner, unidirectional BFS) -- every answer
    against the host oracle."""
    import torch  # noqa: F401
    from bidirectional_bfs_amd.parallel import dist_local_generate_run, make_tuning

    for spec in ("gnp:60000::7", "kron:15:16:4"):
        g = bb.from_spec(spec)
        qs = _pairs(g.n, 8, 61)[2:]
        rs, t = dist_local_generate_run(8, spec, qs, tuning=make_tuning(stamps=True), verify=3)
        assert len(t["local_nnz"]) == 8 and sum(t["local_nnz"]) == g.csr.nnz
        for i, ((s, d), r) in enumerate(zip(qs, rs)):
            h = native.bfs_oracle(g.csr, s, d).hops
            check_result(g.csr, s, d, r.hops, r.path, h)
            assert t["path_valid"][i] == (1 if r.found else -1)
            if i < 3:
                assert t["uni_hops"][i] == h
        assert any(st["stamped_rounds"] > 0 for st in t["stats"])
