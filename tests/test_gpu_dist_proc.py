"""The partitioned engine (csrc/dist/dist_engine.hip) as P SEPARATE PROCESSES on
one GPU, exchanging over the HIP-IPC transport (csrc/dist/ipc_comm.hip): separate
HIP contexts and address spaces, cross-process collective order, and failure
propagation between processes.  This is the reference's own v4 launch shape --
`mpirun -n 4` with every rank on the machine's one GPU
(single_machine_bench.sh:9,52; v4/mpi_bas.cpp:79-132) -- and the same transport
reads peer HBM over xGMI when the ranks sit on different GPUs.

Mirrors tests/test_gpu_dist_local.py (P threads over an in-process group):
oracle, protocol spec, continuation rounds, capped HBM, and a failing / hanging
/ killed rank that must make every other rank exit non-zero within the timeout.
"""
import os
import random
import time

import numpy as np
import pytest

import bidirectional_bfs_amd as bb
from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.models import Graph
from bidirectional_bfs_amd.parallel import (MPIEXEC, ProcRunError, dist_proc_launch, dist_proc_matrix,
                                            dist_proc_run, run_mpi)
from bidirectional_bfs_amd.utils.oracle import check_result

pytestmark = pytest.mark.gpu


def _pairs(n, k, seed):
    rnd = random.Random(seed)
    return [(0, n - 1), (5, 5)] + [(rnd.randrange(n), rnd.randrange(n)) for _ in range(k)]


def _check(g, qs, rs):
    for (s, d), r in zip(qs, rs):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)


@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("spec", ["gnp:20000::6", "rmat:16384:262144:3"])
def test_processes_match_oracle_every_branch(ranks, spec):
    """Every option set and exchange branch over one group of processes that
    read their shards from one .bin: default, single-side, forced directions,
    alternate sides, host-planned rounds, tiny blocks (count syncs, overflow
    to bottom-up), 2-pair owner blocks (continuation rounds) and exact plans
    (pipeline off)."""
    g = bb.from_spec(spec)
    qs = _pairs(g.n, 10, ranks)
    runs = [({}, {}), ({"lockstep": False}, None), ({"direction": "topdown"}, None),
            ({"direction": "bottomup"}, None), ({"side": "alternate"}, None),
            ({"side": "frontier", "lockstep": False}, None),
            ({}, {"spec_rounds": 0}),
            ({}, {"cap": 4, "nosync_bytes": 0, "spec_cap_max": 1024, "spec_stall_edges": 1024}),
            ({}, {"owner_cap": 2}), ({"lockstep": False}, {"owner_cap": 2}),
            ({}, {"pipeline": False}), ({"direction": "bottomup"}, {"pipeline": False})]
    got, outs = dist_proc_matrix(ranks, g, qs, runs)
    assert all(o["backend"] == "ipc" for o in outs)
    assert len({o["pid"] for o in outs}) == ranks  # really separate processes
    assert sum(o["local_nnz"] for o in outs) == g.csr.nnz  # the shards partition the edges
    for rs, _, _ in got:
        _check(g, qs, rs)
    cont = sum(x.get("cont_rounds", 0) for rs, st, _ in got[8:10] for x in st)
    host = sum(x.get("host_rounds", 0) for x in got[6][1])
    assert cont > 0 and host > 0, (cont, host)


@pytest.mark.parametrize("ranks", [2, 3])
def test_processes_device_ordered_exchange(ranks):
    """The processes order their small rounds' exchange on the device (epoch
    flags in the exported windows, DevSync) by default; the same queries with
    DistTuning.dev_sync off take the host rendezvous.  Both answer like the
    oracle, and the counters show which path ran."""
    g = bb.from_spec("gnp:20000::6")
    qs = _pairs(g.n, 12, 40 + ranks)
    runs = [({}, {}), ({}, {"dev_sync": False}), ({}, {"pipeline": False}),
            ({}, {"pipeline": False, "dev_sync": False})]
    got, _ = dist_proc_matrix(ranks, g, qs, runs)
    for rs, _, _ in got:
        _check(g, qs, rs)
    dev = [sum(x.get("dev_sync_rounds", 0) for x in st) for _, st, _ in got]
    assert dev[0] > 0 and dev[2] > 0, dev
    assert dev[1] == 0 and dev[3] == 0, dev
    for rs_on, rs_off in ((got[0][0], got[1][0]), (got[2][0], got[3][0])):
        assert [r.hops for r in rs_on] == [r.hops for r in rs_off]


def test_processes_follow_protocol_spec():
    """Round by round, the processes expand the sides the protocol spec says
    and discover what the BFS levels say (tests/dist_round_spec.py)."""
    from dist_round_spec import round_trace

    g = bb.from_spec("gnp:20000::6")
    qs = _pairs(g.n, 6, 13)
    kws = [{}, {"lockstep": False}, {"side": "alternate"}, {"direction": "bottomup"}]
    tunes = [{}, {"owner_cap": 2}, {"pipeline": False, "owner_cap": 64}]
    runs = [(dict(kw, trace=True), t) for kw in kws for t in tunes]
    got, _ = dist_proc_matrix(3, g, qs, runs)
    for (opts, tune), (rs, lst, _) in zip(runs, got):
        for (s, d), r, x in zip(qs, rs, lst):
            # pipelined rounds (the default with 3 ranks): the spec's lagged side
            # choice, unless the search drained to exact plans (hops checked)
            piped = bool(x["pipelined"])
            if s != d:  # (src == dst is answered without a round)
                assert piped == tune.get("pipeline", True), (s, d, opts, tune)
            want, hops = round_trace(g.csr, s, d, side=opts.get("side", "edges"), lockstep=opts.get("lockstep", True),
                                     pipelined=piped)
            if piped and (x["pipe_drains"] or x["host_rounds"]):
                assert r.hops == hops, (s, d, opts, tune)
                continue
            tr = r.stats.get("trace", [])
            gotr = [(t["side"], t["depth"], t["frontier"], t["edges"], t["discovered"]) for t in tr]
            exp = [w[:5] for w in want]
            if gotr and exp and len(gotr) == len(exp) and gotr[-1][4] < exp[-1][4]:
                assert gotr[-1][:4] == exp[-1][:4] and 0 < gotr[-1][4]
                gotr, exp = gotr[:-1], exp[:-1]
            assert gotr == exp, (s, d, opts)
            assert r.hops == hops


def test_processes_disconnected_tiny_and_bad_queries():
    """Unreachable pairs, a 200-vertex graph over 4 processes (some own almost
    nothing), a long path, and out-of-range queries that fail on every rank
    before any collective while the group keeps serving."""
    g = Graph.from_edges(200, [[0, 1], [1, 2], [2, 3], [150, 151], [151, 199]])
    qs = [(0, 3), (3, 0), (0, 199), (150, 199), (7, 8), (199, 150), (500, 3), (0, 3)]
    rs = dist_proc_run(4, g, qs)
    assert rs[6].hops == -2
    for i in (0, 1, 2, 3, 4, 5, 7):
        s, d = qs[i]
        check_result(g.csr, s, d, rs[i].hops, rs[i].path, native.bfs_oracle(g.csr, s, d).hops)
    n = 3000
    line = Graph.from_edges(n, np.stack([np.arange(n - 1), np.arange(1, n)], 1).astype(np.uint32))
    rs = dist_proc_run(3, line, [(0, n - 1), (17, 2900)])
    assert rs[0].hops == n - 1 and rs[0].path == list(range(n)) and rs[1].hops == 2900 - 17


def test_processes_capped_hbm_device_generated_and_verified():
    """A graph that does not fit one rank's (capped) HBM, generated on the GPU
    shard by shard in 4 processes, verified collectively (paths edge by edge
    by their owners, hops by a unidirectional partitioned BFS) and against
    the host oracle."""
    spec = "rmat:65536:16777216:3"
    cap = 80 << 20
    qs = _pairs(65536, 6, 53)[2:] + [(0, 65535)]
    with pytest.raises(ProcRunError) as ei:
        dist_proc_run(1, spec, qs[:1], tuning={"hbm_cap_bytes": cap})
    assert "HBM cap" in str(ei.value)
    got, outs = dist_proc_matrix(4, spec, qs, [({}, {"hbm_cap_bytes": cap})], verify=4)
    assert sum(o["shard_bytes"] for o in outs) > cap
    assert max(o["resident_bytes"] for o in outs) <= cap
    rs, _, run = got[0]
    g = bb.from_spec(spec)
    for i, ((s, d), r) in enumerate(zip(qs, rs)):
        check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
        assert run["path_valid"][i] == (1 if r.found else -1)
        if i < 4:
            assert run["uni_hops"][i] == r.hops


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_failing_hanging_or_killed_rank_fails_every_process(mode):
    """Rank 1 throws (1), hangs past the watchdog (2) or its process is killed
    (3) mid-search: every process exits non-zero, well within the launcher's
    timeout, and no rank hangs."""
    g = bb.from_spec("gnp:20000::6")
    qs = _pairs(g.n, 4, 2)
    timeout_s = 3.0
    rcs, outs, elapsed = dist_proc_launch(3, g, qs, [({}, {"timeout_s": timeout_s})], fault=(1, 2, mode),
                                          timeout=240)
    assert all(rc != 0 for rc in rcs), (rcs, outs)
    assert elapsed < 120, elapsed
    errs = [o.get("error", "") for o in outs]
    if mode == 3:
        assert rcs[1] < 0 or rcs[1] == 137, rcs  # SIGKILL
        assert all("aborted" in e or "died" in e for i, e in enumerate(errs) if i != 1), errs
    else:
        assert "injected fault" in errs[1], errs
        assert all(e for e in errs), errs


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH not installed")
@pytest.mark.parametrize("np_", [2, 4])
def test_mpi_bibfs_ranks_share_one_gpu(np_):
    """The v4 CLI with more ranks than GPUs (the reference's `mpirun -n 4` on one
    machine): --comm auto picks the IPC transport; hops and path verified."""
    r = run_mpi("mpi_bibfs", ["gnp:1000000::2", 0, 999999, "--verify", "--repeat", "3"], np=np_, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Verify: OK" in r.stdout, r.stdout
    assert f"Ranks: {np_} over ipc" in r.stdout, r.stdout


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH not installed")
def test_mpi_bibfs_killed_rank_fails_the_job():
    t0 = time.monotonic()
    r = run_mpi("mpi_bibfs", ["gnp:200000::2", 0, 199999, "--comm", "ipc", "--timeout", "5", "--fault", "1:2:3",
                              "--repeat", "3"], np=3, timeout=200)
    assert r.returncode != 0, r.stdout + r.stderr
    assert time.monotonic() - t0 < 150


def test_torchrun_ranks_share_one_gpu_over_ipc(repo_root):
    """torch.distributed bootstrap (gloo process group) of 3 ranks on one GPU,
    engine collectives over IPC: G(1M) and Kronecker-16 against the oracle."""
    import json
    import socket
    import subprocess
    import sys

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BIBFS_TEST_BACKEND="ipc")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3",
           "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.join(repo_root, "tests", "helpers", "dist_torchrun_worker.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=repo_root)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    d = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["world"] == 3 and d["backend"] == "ipc" and d["checked"] > 0 and d["bad_total"] == 0, d


def test_spill_overflow_fails_every_rank_and_group_keeps_serving():
    """A candidate spill list shrunk below what a round offers: the
    search raises on EVERY rank at the same point (no rank left in a
    collective, the communicator is not aborted), and the same processes then
    answer the queries exactly with the default sizing."""
    g = bb.from_spec("rmat:16384:262144:3")  # dense: many candidates per owner and round
    qs = _pairs(g.n, 6, 71)
    # (top-down: a bottom-up level exchanges bitmaps, not candidates)
    got, outs = dist_proc_matrix(3, g, qs, [({"_catch": True, "direction": "topdown"},
                                             {"owner_cap": 2, "spill_cap": 1}),
                                            ({}, {"owner_cap": 0, "spill_cap": 0})])
    failed = [r for r in outs[0]["runs"][0]["results"] if r["hops"] == -3]
    assert failed and all("spill list overflowed" in r["error"] for r in failed), outs[0]["runs"][0]["results"]
    for o in outs[1:]:  # every rank failed the same queries
        assert [r["hops"] for r in o["runs"][0]["results"]] == [r["hops"] for r in outs[0]["runs"][0]["results"]]
    _check(g, qs, got[1][0])
