"""Multi-GPU engine (world size 1 on the single-GPU box: the in-process group
of one rank, and an RCCL communicator of one rank), the GPU CLI tools and the
bench.py contract."""
import json
import os
import random
import subprocess
import sys

import pytest

import bidirectional_bfs_amd as bb
from bidirectional_bfs_amd import native
from bidirectional_bfs_amd._lib import tool_path
from bidirectional_bfs_amd.parallel import MPIEXEC, run_mpi
from bidirectional_bfs_amd.utils.oracle import check_result

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world1_comm", ["", "rccl"])
def test_dist_engine_world1(world1_comm, monkeypatch):
    """World size 1: by default the engine's collectives go to an in-process
    group of one (no RCCL bootstrap); BIBFS_WORLD1_COMM=rccl keeps a one-rank
    RCCL communicator, so the RCCL backend stays exercised on one GPU."""
    import torch  # noqa: F401

    from bidirectional_bfs_amd.parallel import DistEngine

    if world1_comm:
        monkeypatch.setenv("BIBFS_WORLD1_COMM", world1_comm)
    eng = DistEngine(0, 1, 0, DistEngine.unique_id())
    assert eng.backend == (world1_comm or "local")
    for spec in ["gnp:100000::6", "rmat:65536:1048576:3"]:
        g = bb.from_spec(spec)
        eng.load(g)
        rnd = random.Random(3)
        for single in (True, False):  # the single-GPU engine on the rank's CSR, then the partitioned rounds
            eng.set_tuning(world1_single=single)
            for s, d in [(0, g.n - 1)] + [(rnd.randrange(g.n), rnd.randrange(g.n)) for _ in range(10)]:
                for direction in ("auto", "topdown", "bottomup"):
                    r = eng.search(s, d, direction=direction)
                    check_result(g.csr, s, d, r.hops, r.path, native.bfs_oracle(g.csr, s, d).hops)
                    assert eng.last_stats["single_engine"] == (1 if single and s != d else 0)
    eng.set_tuning()
    eng.generate_gnp(1_000_000, None, 2)
    r = eng.search(0, 999_999)
    assert r.hops == 19 and len(r.path) == 20


def test_dist_engine_distributed_checks_world1():
    """validate_path accepts the engine's own paths and rejects a broken edge,
    a wrong length or wrong endpoints; search_unidirectional (a plain
    partitioned BFS) agrees with the bidirectional hop counts and the oracle,
    including an unreachable pair."""
    import torch  # noqa: F401

    from bidirectional_bfs_amd.parallel import DistEngine

    eng = DistEngine(0, 1, 0, DistEngine.unique_id())
    g = bb.from_spec("rmat:65536:1048576:3")
    eng.load(g)
    rnd = random.Random(8)
    for s, d in [(rnd.randrange(g.n), rnd.randrange(g.n)) for _ in range(8)]:
        r = eng.search(s, d)
        oh = native.bfs_oracle(g.csr, s, d).hops
        assert eng.search_unidirectional(s, d).hops == r.hops == oh
        if not r.found or r.hops < 2:
            continue
        p = list(r.path)
        assert eng.validate_path(s, d, r.hops, p)
        bad = p[:]
        bad[1] = (bad[1] + 1) % g.n
        while native.bfs_oracle(g.csr, bad[0], bad[1]).hops == 1 and native.bfs_oracle(g.csr, bad[1], bad[2]).hops == 1:
            bad[1] = (bad[1] + 1) % g.n
        assert not eng.validate_path(s, d, r.hops, bad)
        assert not eng.validate_path(s, d, r.hops + 1, p)
        assert not eng.validate_path(d, s, r.hops, p) or s == d
    g2 = bb.Graph.from_edges(100, [[0, 1], [1, 2], [50, 51]])
    eng.load(g2)
    assert eng.search_unidirectional(0, 2).hops == 2
    assert eng.search_unidirectional(0, 51).hops == -1


def test_bibfs_hip_cli():
    out = subprocess.run([tool_path("bibfs_hip"), "gnp:100000::6", "0", "99999", "--verify", "--repeat", "3"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    assert lines[0] == "Shortest path length = 17"
    assert lines[2].startswith("[Time] HIP bi-BFS query = ") and lines[2].endswith(" s")
    assert "GPU BFS: PATH FOUND" in out.stdout and "Verify: OK" in out.stdout
    js = subprocess.run([tool_path("bibfs_cuda_only"), "gnp:100000::6", "0", "99999", "--json"],
                        capture_output=True, text=True, timeout=120)
    d = json.loads(js.stdout)
    assert d["hops"] == 17 and d["gteps"] > 0.952  # beats the best published 100k number


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH not installed")
def test_mpi_bibfs_one_rank():
    r = run_mpi("mpi_bibfs", ["gnp:100000::6", 0, 99999, "--verify"], np=1, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Shortest path length = 17" in r.stdout and "Verify: OK" in r.stdout


def test_bibfs_bench_tool():
    out = subprocess.run([tool_path("bibfs_bench"), "gnp:100000::6", "--queries", "30", "--warmup", "5"],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout)
    assert d["queries"] == 30 and d["median_query_ms"] > 0


def test_bench_py_contract(repo_root):
    out = subprocess.run([sys.executable, os.path.join(repo_root, "bench.py"), "--steps", "20", "--warmup", "5",
                          "--extra-graph", ""], capture_output=True, text=True, timeout=300, cwd=repo_root)
    assert out.returncode == 0, out.stderr
    d = json.loads(out.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["value"] > 0
    assert d["detail"]["secondary_errors"] == [], d["detail"]["secondary_errors"]  # partitioned configs verified
