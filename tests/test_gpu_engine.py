"""Single-GPU HIP engine (v3 capability) on a real MI355X, against the CPU oracle."""
import ctypes
import random

import numpy as np
import pytest

import bidirectional_bfs_amd as bb
from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.models import Graph, gnp, kronecker, rmat
from bidirectional_bfs_amd.ops import make_options
from bidirectional_bfs_amd.utils.oracle import check_result

pytestmark = pytest.mark.gpu


def pairs_for(n, k, seed):
    rnd = random.Random(seed)
    return [(0, n - 1)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(k)]


def assert_engine(eng, g, pairs, **opt):
    o = make_options(**opt)
    for s, d in pairs:
        r = eng.search(s, d, o)
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)


@pytest.mark.parametrize("spec", ["gnp:1000::1", "gnp:100000::6", "gnp:1000000::2", "rmat:65536:1048576:3",
                                  "kron:16:16:2"])
def test_lds_and_grid_vs_oracle(gpu_engine, spec):
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 25, 7)
    assert_engine(gpu_engine, g, pairs)
    assert_engine(gpu_engine, g, pairs[:8], force_grid=True)
    assert_engine(gpu_engine, g, pairs[:5], force_grid=True, direction="topdown")
    assert_engine(gpu_engine, g, pairs[:5], force_grid=True, direction="bottomup")
    assert_engine(gpu_engine, g, pairs[:5], side="frontier")
    assert_engine(gpu_engine, g, pairs[:5], side="alternate")
    assert_engine(gpu_engine, g, pairs[:8], lockstep=False)


def test_device_csr_equals_host(gpu_engine):
    g = gnp(50000, seed=3)
    gpu_engine.load(g)
    d = gpu_engine.download_csr()
    h = g.csr
    assert np.array_equal(d.row_off, h.row_off)
    for v in range(0, g.n, 97):
        a, b = slice(h.row_off[v], h.row_off[v + 1]), slice(d.row_off[v], d.row_off[v + 1])
        assert sorted(h.col[a]) == sorted(d.col[b])


def test_device_generators_match_host(gpu_engine):
    gpu_engine.generate_gnp(30000, 3.0 / 30000, 9)
    assert np.array_equal(gpu_engine.download_edges().edges(), native.gen_gnp(30000, 3.0 / 30000, 9).edges())
    gpu_engine.generate_rmat(20000, 150000, 5)
    assert np.array_equal(gpu_engine.download_edges().edges(), native.gen_rmat(20000, 150000, 5).edges())


def test_handoff_to_grid_on_10m(gpu_engine):
    gpu_engine.generate_gnp(10_000_000, 2.2000000001 / 10_000_000, 1)
    r = gpu_engine.search(0, 9_999_999)
    assert r.found and r.hops == 19 and len(r.path) == 20
    el = gpu_engine.download_edges()
    g = Graph(el)
    check_result(g.csr, 0, 9_999_999, r.hops, r.path, 19)


def test_edge_cases(gpu_engine):
    g = Graph.from_edges(8, [[0, 1], [1, 2], [3, 4], [4, 5]])
    gpu_engine.load(g)
    assert gpu_engine.search(1, 1).hops == 0
    assert not gpu_engine.search(0, 5).found
    assert not gpu_engine.search(7, 0).found  # isolated source
    assert gpu_engine.search(0, 2).hops == 2
    # hub source (degree > LDS capacity => immediate hand-off)
    star = Graph.from_edges(20001, [[0, i] for i in range(1, 20001)] + [[5, 20000 - 1]])
    gpu_engine.load(star)
    r = gpu_engine.search(0, 7)
    check_result(star.csr, 0, 7, r.hops, r.path, 1)
    r = gpu_engine.search(3, 7)
    check_result(star.csr, 3, 7, r.hops, r.path, 2)


def test_long_path_goes_to_device_buffer(gpu_engine):
    n = (1 << 20) + 500  # hops + 1 > pinned path capacity (2^20)
    g = Graph.from_edges(n, np.stack([np.arange(n - 1), np.arange(1, n)], 1).astype(np.uint32))
    gpu_engine.load(g)
    r = gpu_engine.search(0, n - 1)
    assert r.hops == n - 1 and r.path[0] == 0 and r.path[-1] == n - 1
    assert np.array_equal(np.asarray(r.path), np.arange(n))


def test_stepwise_api(gpu_engine):
    g = gnp(100000, seed=6)
    gpu_engine.load(g)
    gpu_engine.begin(0, 99999)
    met, side, levels = False, 0, 0
    while not met and levels < 100:
        claimed, met = gpu_engine.expand(side)
        levels += 1
        if claimed == 0 and not met:
            break
        side ^= 1
    assert met and gpu_engine.check_meet()
    r = gpu_engine.finish()
    check_result(g.csr, 0, 99999, r.hops, r.path, 17)
    assert gpu_engine.search(0, 99999).hops == 17  # state fully reset


def test_c_api(repo_root):
    lib = ctypes.CDLL(f"{repo_root}/build/lib/libbibfs.so")

    class Res(ctypes.Structure):
        _fields_ = [("found", ctypes.c_int32), ("hops", ctypes.c_int64), ("meet", ctypes.c_uint32),
                    ("levels", ctypes.c_int32), ("edges_inspected", ctypes.c_uint64), ("search_ms", ctypes.c_double),
                    ("total_ms", ctypes.c_double), ("path_len", ctypes.c_size_t)]

    lib.bibfs_create.restype = ctypes.c_void_p
    lib.bibfs_last_error.restype = ctypes.c_char_p
    ctx = ctypes.c_void_p(lib.bibfs_create(0))
    assert ctx.value, lib.bibfs_last_error()
    el = native.gen_gnp(10000, native.reference_p(10000), 1)
    uv = np.ascontiguousarray(el.edges().ravel())
    assert lib.bibfs_init_graph_edges(ctx, ctypes.c_uint32(10000), ctypes.c_uint64(el.m),
                                      uv.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))) == 0
    res = Res()
    path = (ctypes.c_uint32 * 64)()
    assert lib.bibfs_search(ctx, ctypes.c_uint32(0), ctypes.c_uint32(9999), ctypes.byref(res), path, 64) == 0
    assert res.found == 1 and res.hops == 12 and res.path_len == 13 and path[0] == 0 and path[12] == 9999
    # step-wise entry points
    assert lib.bibfs_init_frontiers(ctx, ctypes.c_uint32(0), ctypes.c_uint32(9999)) == 0
    met, claimed, side = ctypes.c_int(0), ctypes.c_uint64(0), 0
    for _ in range(64):
        assert lib.bibfs_expand_frontier(ctx, side, ctypes.byref(claimed), ctypes.byref(met)) == 0
        if met.value:
            break
        side ^= 1
    found = ctypes.c_int(0)
    assert lib.bibfs_check_intersect(ctx, ctypes.byref(found)) == 0 and found.value == 1
    assert lib.bibfs_finish(ctx, ctypes.byref(res), path, 64) == 0 and res.hops == 12
    lib.bibfs_destroy(ctx)


def test_trace_and_stats(gpu_engine):
    g = gnp(100000, seed=6)
    gpu_engine.load(g)
    r = gpu_engine.search(0, 99999, make_options(trace=True))
    tr = r.stats["trace"]
    assert len(tr) == r.stats["levels"] == 17
    assert all(t["mode"] in (1, 2, 3) for t in tr)
    assert sum(t["edges"] for t in tr) == r.stats["edges_inspected"]


@pytest.mark.parametrize("spec", ["gnp:100000::6", "gnp:1000000::2", "rmat:65536:1048576:3"])
def test_resident_server_vs_oracle(gpu_engine, spec):
    """Resident query server (pinned mailbox, no launch per query), interleaved
    with one-shot grid / trace queries that must not disturb it."""
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 30, 21)
    gpu_engine.set_resident(True)
    try:
        assert gpu_engine.resident
        assert_engine(gpu_engine, g, pairs)
        assert_engine(gpu_engine, g, pairs[:4], force_grid=True)
        assert_engine(gpu_engine, g, pairs[:4], trace=True)
        assert_engine(gpu_engine, g, pairs[:10], lockstep=False, side="alternate")
        assert_engine(gpu_engine, g, pairs)
    finally:
        gpu_engine.set_resident(False)


def test_resident_idle_exit_and_relaunch(gpu_engine):
    import time

    g = gnp(100000, seed=6)
    gpu_engine.load(g)
    gpu_engine.set_resident(True, idle_ms=5.0)
    try:
        for k in range(3):
            r = gpu_engine.search(0, 99999)
            assert r.found and r.hops == 17
            time.sleep(0.05)  # the server idles out; the next query relaunches it
    finally:
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("resident", [False, True])
def test_path_longer_than_lds_staging(gpu_engine, resident):
    n = 50_000  # 50k-vertex path: longer than the LDS staging buffer, shorter than the pinned buffer
    g = Graph.from_edges(n, np.stack([np.arange(n - 1), np.arange(1, n)], 1).astype(np.uint32))
    gpu_engine.load(g)
    gpu_engine.set_resident(resident)
    try:
        r = gpu_engine.search(0, n - 1)
        assert r.hops == n - 1
        assert np.array_equal(np.asarray(r.path), np.arange(n))
    finally:
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("spec", ["gnp:100000::6", "gnp:1000000::2", "rmat:65536:1048576:3"])
def test_search_batch_vs_oracle(gpu_engine, spec):
    """Batched serving (one workgroup per query) gives the single-query answers;
    queries that outgrow LDS are re-run through the single-query engines."""
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 300, 31)
    rs = gpu_engine.search_batch(pairs)
    assert len(rs) == len(pairs)
    for (s, d), r in zip(pairs, rs):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
    hops, off, flat = gpu_engine.search_batch_arrays([s for s, _ in pairs[:64]], [d for _, d in pairs[:64]])
    for i, (s, d) in enumerate(pairs[:64]):
        path = list(flat[off[i]:off[i + 1]])
        check_result(g.csr, s, d, int(hops[i]), path, native.bfs_oracle(g.csr, s, d).hops)


@pytest.mark.parametrize("spec", ["gnp:1000000::2", "gnp:3000000::5", "rmat:262144:4194304:4"])
def test_search_batch_global_pass(gpu_engine, spec):
    """Queries that outgrow LDS take the batched HBM-bitmap pass (batch_global.hip):
    exact hops + valid paths, bitmaps left clean for the next batch (three
    back-to-back batches agree), and the edge-cap fallback gives the same answers."""
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 200, 57) + [(5, 5), (g.n - 1, g.n - 1)]
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    cap0 = gpu_engine.batch_edge_cap
    try:
        runs = []
        for _ in range(3):
            rs = gpu_engine.search_batch(pairs)
            for (s, d), r, h in zip(pairs, rs, truth):
                check_result(g.csr, s, d, r.hops, r.path, h)
            runs.append([r.hops for r in rs])
        assert runs[0] == runs[1] == runs[2]
        if g.n > 131072:
            assert any(r.handoff for r in rs), "expected queries to take the HBM-bitmap pass"
        for lds_first, threads in ((0, 1024), (0, 256), (1, 1024)):
            gpu_engine.set_batch_tuning(lds_first, threads)
            rs = gpu_engine.search_batch(pairs)
            for (s, d), r, h in zip(pairs, rs, truth):
                check_result(g.csr, s, d, r.hops, r.path, h)
        gpu_engine.set_batch_tuning(-1, 0)
        gpu_engine.batch_edge_cap = 16  # almost every query falls back to search()
        rs = gpu_engine.search_batch(pairs[:40])
        for (s, d), r, h in zip(pairs[:40], rs, truth[:40]):
            check_result(g.csr, s, d, r.hops, r.path, h)
        assert gpu_engine.last_batch_fallbacks > 0
    finally:
        gpu_engine.batch_edge_cap = cap0
        gpu_engine.set_batch_tuning(-1, 0)


def _lollipop(n_path, n_blob, p_blob, seed):
    """A long path glued to a dense G(n, p) blob: a query from the path's far
    end into the blob has one tiny frontier and one that grows fast -- the
    unbalanced shape the all-wave rounds serve one side at a time."""
    blob = native.gen_gnp(n_blob, p_blob, seed).edges().astype(np.int64) + n_path
    path = [[i, i + 1] for i in range(n_path - 1)] + [[n_path - 1, n_path]]
    return Graph.from_edges(n_path + n_blob, np.concatenate([np.asarray(path, dtype=np.int64), blob]))


@pytest.mark.parametrize("resident", [False, True])
def test_unbalanced_frontiers_in_lds(gpu_engine, resident):
    """Bitmap-mode graphs (n <= 131072) whose two frontiers outgrow the
    lockstep round unevenly: single-side all-wave rounds, meets right after a
    switch, empty frontiers (no path), all against the oracle."""
    rnd = random.Random(11)
    graphs = [gnp(100000, 3.2 / 100000, 9),          # fast-growing frontiers
              gnp(120000, 1.6 / 120000, 4),          # many small components: no-path pairs
              rmat(65536, 400000, 7),                # hubs next to leaves
              _lollipop(40, 60000, 6.0 / 60000, 3)]  # tiny side vs big side
    for g in graphs:
        gpu_engine.load(g)
        gpu_engine.set_resident(resident)
        n = g.n
        pairs = [(0, n - 1), (n - 1, 0)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(40)]
        if g.n == 60040:
            pairs += [(rnd.randrange(40), 40 + rnd.randrange(60000)) for _ in range(20)]
        assert_engine(gpu_engine, g, pairs)
        gpu_engine.set_resident(False)


def test_resident_back_to_back_handoffs(gpu_engine):
    """Back-to-back resident queries that all leave LDS: the server (own
    stream) must not start the next search while the previous one's cleanup
    (engine stream) still reads and clears the global visited words."""
    g = kronecker(22, 16, 5)
    gpu_engine.load(g)
    probe0 = gpu_engine.lds_probe_edges
    gpu_engine.lds_probe_edges = 0  # every search leaves LDS (no meet probe)
    rnd = random.Random(3)
    pairs = []
    while len(pairs) < 8:
        s, d = rnd.randrange(g.n), rnd.randrange(g.n)
        h = native.bfs_oracle(g.csr, s, d).hops
        if h > 0:
            pairs.append((s, d, h))
    gpu_engine.set_resident(True)
    try:
        for i in range(600):
            s, d, h = pairs[i % len(pairs)]
            r = gpu_engine.search(s, d)
            assert r.hops == h, (i, s, d, r.hops, h)
            if i % 100 == 0:
                check_result(g.csr, s, d, r.hops, r.path, h)
    finally:
        gpu_engine.lds_probe_edges = probe0
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("spec", ["kron:20:16:2", "gnp:3000000::4"])
def test_resident_auto_handoff_vs_oracle(gpu_engine, spec):
    """Device hand-off (grid_auto): resident searches that leave LDS continue in
    a grid level enqueued before they started, gated on the device.  Back to
    back on both state sets with the knob on, off and on again (the auto
    chain's no-op launches and cleanups must not disturb the host loop), plus
    first levels the Beamer rule sends bottom-up (the auto level declines and
    the host loop takes them); every answer against the oracle."""
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 40, 5)
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    gpu_engine.set_resident(True)
    probe0 = gpu_engine.lds_probe_edges
    gpu_engine.lds_probe_edges = 0  # hub graphs: searches must leave LDS
    try:
        for on in (True, False, True):
            gpu_engine.auto_handoff = on
            assert gpu_engine.auto_handoff == on
            handed = 0
            for (s, d), h in zip(pairs, truth):
                r = gpu_engine.search(s, d)
                check_result(g.csr, s, d, r.hops, r.path, h)
                handed += bool(r.handoff)
            assert handed > 0, "expected searches that leave LDS"
        for (s, d), h in zip(pairs[:10], truth[:10]):
            r = gpu_engine.search(s, d, make_options(alpha=1e-9))
            check_result(g.csr, s, d, r.hops, r.path, h)
        for (s, d), h in zip(pairs[:10], truth[:10]):  # query() serving path
            hops, path = gpu_engine.query(s, d)
            check_result(g.csr, s, d, hops, path, h)
    finally:
        gpu_engine.auto_handoff = True
        gpu_engine.lds_probe_edges = probe0
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("spec", ["gnp:3000000::4", "kron:20:16:2"])
def test_resident_auto_levels_chain_vs_oracle(gpu_engine, spec):
    """Chained device-planned grid levels (auto_levels): the finisher of each
    auto level plans the next one into aux, and the host only hears from the
    chain's end (result, or the mirror when the search goes on or a level is
    declined).  Chains of 1, 2, 3 and 8 levels, back to back, hub graphs
    included (auto_max_degree lifted: the hub pass runs behind auto levels);
    every answer against the oracle, and grid levels are counted from the
    result's level count."""
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 32, 9)
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    gpu_engine.set_resident(True)
    md0, lv0, probe0 = gpu_engine.auto_max_degree, gpu_engine.auto_levels, gpu_engine.lds_probe_edges
    gpu_engine.lds_probe_edges = 0  # hub graphs: searches must reach the grid levels
    try:
        gpu_engine.auto_max_degree = 1 << 40
        for lv in (1, 2, 3, 8, 2):
            gpu_engine.auto_levels = lv
            assert gpu_engine.auto_levels == lv
            grid = 0
            for (s, d), h in zip(pairs, truth):
                r = gpu_engine.search(s, d)
                check_result(g.csr, s, d, r.hops, r.path, h)
                grid += r.stats["grid_levels"]
            assert grid > 0, "expected searches with grid levels"
        with pytest.raises(Exception):
            gpu_engine.auto_levels = 0
    finally:
        gpu_engine.auto_max_degree = md0
        gpu_engine.auto_levels = lv0
        gpu_engine.lds_probe_edges = probe0
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("spec", ["kron:20:16:2", "rmat:262144:4194304:4", "rmat:65536:1048576:3"])
def test_lds_meet_probe_vs_oracle(gpu_engine, spec):
    """LDS meet probe (hub graphs): before a level that does not fit LDS goes
    to the grid engine, up to lds_probe_edges of its frontier edges are tested
    against the other side's visited set, and a hit ends the search.  Default
    budget, one pass (4096 edges) and off; resident and one-shot searches
    (hash-set and bitmap LDS modes); every answer against the oracle with its
    path validated; hits and hand-offs both seen, the budget never exceeded."""
    g = bb.from_spec(spec)
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 40, 21)
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    b0 = gpu_engine.lds_probe_edges
    assert b0 > 0
    hits = handed = handed0 = 0
    try:
        for budget in (b0, 4096, 0):
            gpu_engine.lds_probe_edges = budget
            assert gpu_engine.lds_probe_edges == budget
            for resident in (True, False):
                gpu_engine.set_resident(resident)
                for (s, d), h in zip(pairs, truth):
                    r = gpu_engine.search(s, d)
                    check_result(g.csr, s, d, r.hops, r.path, h)
                    st = r.stats
                    assert st["probe_edges"] <= budget, (s, d, st["probe_edges"], budget)
                    if st["probe_hit"]:
                        assert not r.handoff
                        hits += 1
                    handed += bool(r.handoff)
                    if budget == 0:
                        assert not st["probe_hit"]
                        handed0 += bool(r.handoff)
                gpu_engine.set_resident(False)
        if spec.startswith("kron"):  # Kronecker searches leave LDS, and the probe ends many of them
            assert handed0 > 0 and hits > 0, (handed0, hits, handed)
    finally:
        gpu_engine.lds_probe_edges = b0
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("spec", ["kron:18:16:2", "gnp:1000000::2"])
def test_wide_offsets_resident_server_vs_oracle(gpu_engine, spec, monkeypatch):
    """64-bit row offsets (what a graph with nnz >= 2^32 gets, forced here on a
    small one): the resident LDS server, its hand-offs and the meet probe run
    the OffT = uint64 kernels; one-shot and resident answers against the
    oracle."""
    g = bb.from_spec(spec)
    pairs = pairs_for(g.n, 40, 33)
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    gpu_engine.set_build_flags(wide_offsets=True)
    gpu_engine.load(g)
    try:
        handed = 0
        for resident in (True, False):
            gpu_engine.set_resident(resident)
            for (s, d), h in zip(pairs, truth):
                r = gpu_engine.search(s, d)
                check_result(g.csr, s, d, r.hops, r.path, h)
                handed += bool(r.handoff)
            for (s, d), h in zip(pairs[:8], truth[:8]):
                hops, path = gpu_engine.query(s, d)
                check_result(g.csr, s, d, hops, path, h)
        assert handed > 0 or spec.startswith("kron"), "expected hand-offs on the G(n, p) graph"
    finally:
        gpu_engine.set_resident(False)
        gpu_engine.set_build_flags()
        gpu_engine.load(g)  # 32-bit offsets again for the tests after this one


def test_row_bases_above_2_31_vs_grid_engine(gpu_engine):
    """A graph whose CSR row bases pass 2^31 (Kronecker 26, edge factor 20:
    2.7B directed edges, generated on the device): resident LDS searches --
    meet probe, cooperative hub appends, lost-record rebuild, hand-offs --
    against the grid-only engine on 300 random pairs.  (A 64-bit row base
    sign-extended through a 32-bit lane read once sent a whole hub's records
    to one edge and returned too-long paths on Kronecker 27.)"""
    gpu_engine.generate_rmat(1 << 26, 20 << 26, 1)
    assert gpu_engine.nnz > (1 << 31)
    n = 1 << 26
    rnd = random.Random(27)
    pairs = [(rnd.randrange(n), rnd.randrange(n)) for _ in range(300)]
    gpu_engine.set_resident(True)
    try:
        got = []
        for s, d in pairs:
            r = gpu_engine.search(s, d)
            assert r.hops < 0 or (len(r.path) == r.hops + 1 and r.path[0] == s and r.path[-1] == d)
            got.append(r.hops)
    finally:
        gpu_engine.set_resident(False)
    grid = make_options(force_grid=True)
    wrong = [(s, d, h, gpu_engine.search(s, d, grid).hops) for (s, d), h in zip(pairs, got)
             if gpu_engine.search(s, d, grid).hops != h]
    assert not wrong, wrong[:5]


def test_auto_handoff_gate_timeout_falls_back_to_host(gpu_engine):
    """The gated first grid level gives up when its search has not left LDS in
    time (forced here: a zero wait).  Such a search still hands off later; the
    host must then see the auto chain drain unpublished and continue like a
    non-auto hand-off (scatter + host levels from the mirror) -- every answer
    against the oracle, and the fallback counted."""
    g = bb.from_spec("gnp:3000000::4")
    gpu_engine.load(g)
    pairs = pairs_for(g.n, 24, 9)
    truth = [native.bfs_oracle(g.csr, s, d).hops for s, d in pairs]
    gpu_engine.set_resident(True)
    m0 = gpu_engine.auto_gate_misses
    try:
        gpu_engine.auto_gate_timeout_us = 0.0
        handed = 0
        for (s, d), h in zip(pairs, truth):
            r = gpu_engine.search(s, d)
            check_result(g.csr, s, d, r.hops, r.path, h)
            handed += bool(r.handoff)
        assert handed > 0, "expected searches that leave LDS"
        assert gpu_engine.auto_gate_misses > m0, "the host fallback never ran"
        gpu_engine.auto_gate_timeout_us = 6e6  # back to the default: the next searches are fine too
        for (s, d), h in zip(pairs[:8], truth[:8]):
            hops, path = gpu_engine.query(s, d)
            check_result(g.csr, s, d, hops, path, h)
    finally:
        gpu_engine.auto_gate_timeout_us = 6e6
        gpu_engine.set_resident(False)


# ---------------------------------------------------------------- tiny server
def test_tiny_server_query_vs_oracle(gpu_engine):
    """Resident small-graph server (tiny_engine.hip): hops + path of query()
    and search() against the oracle, connected and disconnected pairs, src ==
    dst, interleaved with one-shot queries of non-default options."""
    g = gnp(100000, seed=6)
    gpu_engine.load(g)
    assert gpu_engine.tiny_engine
    pairs = pairs_for(g.n, 300, 41) + [(7, 7)]
    gpu_engine.set_resident(True)
    ovf0 = gpu_engine.tiny_overflows
    try:
        for i, (s, d) in enumerate(pairs):
            h, path = gpu_engine.query(s, d)
            truth = native.bfs_oracle(g.csr, s, d).hops
            check_result(g.csr, s, d, h, path, truth)
            if h > 0:
                assert gpu_engine.last_search_ms > 0
            if i % 50 == 0:  # the general engine beside the resident server
                r = gpu_engine.search(s, d, make_options(force_grid=True))
                check_result(g.csr, s, d, r.hops, r.path, truth)
                r = gpu_engine.search(s, d, make_options(trace=True))
                check_result(g.csr, s, d, r.hops, r.path, truth)
        assert_engine(gpu_engine, g, pairs[:40])
        assert gpu_engine.query(0, 99999)[0] == 17
        # reference-shape queries fit the tiny server: few may fall back (a
        # fallback still answers correctly, so only this count catches a
        # server that hands everything back)
        ovf = gpu_engine.tiny_overflows - ovf0
        assert ovf <= len(pairs) // 20, ovf
    finally:
        gpu_engine.set_resident(False)


def test_tiny_server_overflow_falls_back(gpu_engine):
    """Frontiers beyond the tiny server's LDS capacity (a round above 2048
    edges, a queue above 4096 vertices): the query is re-run on the general
    engine with the same answer."""
    g = gnp(120000, 12.0 / 120000, 3)
    gpu_engine.load(g)
    assert gpu_engine.tiny_engine
    gpu_engine.set_resident(True)
    ovf0 = gpu_engine.tiny_overflows
    try:
        for s, d in pairs_for(g.n, 40, 5):
            h, path = gpu_engine.query(s, d)
            check_result(g.csr, s, d, h, path, native.bfs_oracle(g.csr, s, d).hops)
        assert gpu_engine.tiny_overflows > ovf0  # this graph's frontiers do outgrow the tiny server
    finally:
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("deg", [3.2, 5.0])
def test_tiny_server_spilled_records_vs_oracle(gpu_engine, deg):
    """Frontiers whose next-round records pass the LDS buffers: the records
    spill to global memory and big single-side rounds run in two passes, so
    long-path queries stay on the tiny server -- every answer against the
    oracle, paths validated, and fewer fallbacks than queries."""
    n = 110000
    g = gnp(n, deg / n, 17)
    gpu_engine.load(g)
    assert gpu_engine.tiny_engine
    gpu_engine.set_resident(True)
    ovf0 = gpu_engine.tiny_overflows
    rnd = random.Random(int(deg * 10))
    pairs = [(0, n - 1)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(120)]
    try:
        for s, d in pairs:
            h, path = gpu_engine.query(s, d)
            check_result(g.csr, s, d, h, path, native.bfs_oracle(g.csr, s, d).hops)
        assert gpu_engine.tiny_overflows - ovf0 < len(pairs) // 4
    finally:
        gpu_engine.set_resident(False)


def test_tiny_server_not_used_for_hubs(gpu_engine):
    """A degree above the packed-word limit keeps the graph on the general server."""
    star = Graph.from_edges(5001, [[0, i] for i in range(1, 5001)])
    gpu_engine.load(star)
    assert not gpu_engine.tiny_engine
    gpu_engine.set_resident(True)
    try:
        h, path = gpu_engine.query(1, 4000)
        assert h == 2 and path == [1, 0, 4000]
    finally:
        gpu_engine.set_resident(False)


def test_tiny_server_relaunch_and_kind_switch(gpu_engine):
    """Idle exit + relaunch of the tiny server, and a switch to a big graph
    (general server) and back."""
    import time

    small = gnp(100000, seed=6)
    gpu_engine.load(small)
    gpu_engine.set_resident(True, idle_ms=5.0)
    try:
        for _ in range(3):
            assert gpu_engine.query(0, 99999)[0] == 17
            time.sleep(0.05)
        gpu_engine.generate_gnp(1_000_000, 2.2000000001 / 1_000_000, 2)
        assert not gpu_engine.tiny_engine
        r = gpu_engine.search(0, 999_999)
        assert r.found
        gpu_engine.load(small)
        assert gpu_engine.query(0, 99999)[0] == 17
    finally:
        gpu_engine.set_resident(False)


@pytest.mark.parametrize("spec", ["gnp:30000:0.0002:9", "rmat:20000:150000:5"])
def test_streamed_generation_equals_edge_list_csr(gpu_engine, spec, monkeypatch):
    """Graphs generated straight into the CSR (two passes over the
    counter-based generator, no edge list -- the large-graph path) have exactly
    the rows of the CSR built from the materialised edge list."""
    kind, n, arg, seed = spec.split(":")[0], int(spec.split(":")[1]), float(spec.split(":")[2]), int(spec.split(":")[3])
    el = native.gen_gnp(n, arg, seed) if kind == "gnp" else native.gen_rmat(n, int(arg), seed)
    h = native.build_csr(el)
    gpu_engine.set_build_flags(stream_gen=True)
    try:
        if kind == "gnp":
            gpu_engine.generate_gnp(n, arg, seed)
        else:
            gpu_engine.generate_rmat(n, int(arg), seed)
    finally:
        gpu_engine.set_build_flags()
    d = gpu_engine.download_csr()
    assert gpu_engine.m == el.m
    assert np.array_equal(d.row_off, h.row_off)
    for v in range(0, n, 37):
        a, b = slice(h.row_off[v], h.row_off[v + 1]), slice(d.row_off[v], d.row_off[v + 1])
        assert sorted(h.col[a]) == sorted(d.col[b])
    r = gpu_engine.search(0, n - 1)
    check_result(h, 0, n - 1, r.hops, r.path, native.bfs_oracle(h, 0, n - 1).hops)
