"""MPI engines (v2 capability: C3 bitmap, C4 frontier list) under mpiexec on
the CPU, 1-4 ranks, against the oracle."""
import json
import os
import random

import pytest

from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.models import gnp, rmat
from bidirectional_bfs_amd.parallel import MPIEXEC, run_mpi

pytestmark = pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH not installed")


def run_json(tool, graph, s, d, np_):
    r = run_mpi(tool, [graph, s, d, "--json", "--repeat", "2"], np=np_, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("tool", ["second_try", "mpi_queue_bibfs"])
@pytest.mark.parametrize("np_", [1, 2, 3, 4])
def test_mpi_engines_vs_oracle(tool, np_, tmp_path):
    g = gnp(100000, seed=6)
    p = str(tmp_path / "g.bin")
    g.save_bin(p)
    rnd = random.Random(np_)
    pairs = [(0, 99999)] + [(rnd.randrange(100000), rnd.randrange(100000)) for _ in range(3)]
    for s, d in pairs:
        out = run_json(tool, p, s, d, np_)
        assert out["hops"] == native.bfs_oracle(g.csr, s, d).hops


@pytest.mark.parametrize("tool", ["second_try", "mpi_queue_bibfs"])
def test_mpi_verify_path_and_stdout_contract(tool):
    r = run_mpi(tool, ["gnp:10000::1", 0, 9999, "--verify"], np=2)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.splitlines()
    assert lines[0] == "Shortest path length = 12"  # v2 printed ceil(h/2)
    assert lines[1].startswith("[Time] ") and lines[1].endswith(" seconds")
    assert lines[2].startswith("Path: 0 ") and lines[2].endswith(" 9999")
    assert "Verify: OK" in r.stdout


def test_mpi_src_eq_dst_and_unreachable(tmp_path):
    out = run_json("second_try", "gnp:10000::1", 5, 5, 2)
    assert out["hops"] == 0
    out = run_json("mpi_queue_bibfs", "gnp:100000::1", 0, 99999, 3)  # 0 and N-1 disconnected (seed 1)
    assert out["hops"] == -1 and out["found"] is False


def test_mpi_rmat():
    g = rmat(4096, 30000, 2)
    for s, d in [(1, 2), (7, 4000), (100, 3000)]:
        out = run_json("second_try", "rmat:4096:30000:2", s, d, 3)
        assert out["hops"] == native.bfs_oracle(g.csr, s, d).hops


def test_mpi_bibfs_more_ranks_than_gpus_fails_clearly():
    """--comm rccl is one rank per GPU: a launch with more ranks on the node than
    visible GPUs (every rank here: no GPU at all, or np 3 on a 1-GPU box) ends
    with one clear message on the over-subscribed ranks and rc 1 -- no raw HIP
    error, no rank left waiting in RCCL bootstrap.  (--comm auto / ipc run such
    a launch over the IPC transport: tests/test_gpu_dist_proc.py.)"""
    from bidirectional_bfs_amd.parallel import gpu_count

    np_ = gpu_count() + 2
    r = run_mpi("mpi_bibfs", ["gnp:1000::1", 0, 999, "--comm", "rccl"], np=np_, timeout=60)
    assert r.returncode != 0
    assert "one rank per GPU" in r.stderr and "ranks on this node > GPUs" in r.stderr


def test_mpi_bibfs_without_gpu_fails_clearly():
    from bidirectional_bfs_amd.parallel import gpu_count

    if gpu_count():
        pytest.skip("a GPU is visible")
    r = run_mpi("mpi_bibfs", ["gnp:1000::1", 0, 999], np=2, timeout=60)
    assert r.returncode != 0 and "no usable GPU" in r.stderr, r.stderr
