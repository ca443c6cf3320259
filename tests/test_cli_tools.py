"""CLI contract: reference argv, stdout lines, the harness awk
regex (benchmark_test.sh:61-69) matching a SECONDS value, generator outputs."""
import json
import re
import subprocess
import sys

import pytest

from bidirectional_bfs_amd._lib import tool_path

HARNESS = re.compile(r"search time|^\[time\]|took[ \t]+[0-9]|gpu bfs time", re.IGNORECASE)


def harness_time(stdout: str) -> float:
    for line in stdout.splitlines():
        if HARNESS.search(line):
            return float(re.findall(r"[0-9]+\.?[0-9]*(?:[eE][-+]?[0-9]+)?", line)[0])
    raise AssertionError("no harness-parsable timing line")


def test_serial_cli_contract(tmp_path):
    out = subprocess.run([tool_path("bibfs_serial"), "gnp:10000::1", "0", "9999"], capture_output=True, text=True)
    assert out.returncode == 0
    lines = out.stdout.splitlines()
    assert lines[0] == "Shortest path length = 12"
    assert lines[1].startswith("Path: 0 ") and lines[1].endswith(" 9999")
    assert re.match(r"Serial bidirectional BFS took [0-9.e-]+ seconds", lines[2])
    assert 0 < harness_time(out.stdout) < 1.0


def test_serial_cli_usage_and_errors():
    out = subprocess.run([tool_path("bibfs_serial")], capture_output=True, text=True)
    assert out.returncode == 1 and "Usage" in out.stderr
    out = subprocess.run([tool_path("bibfs_serial"), "/nonexistent.bin", "0", "1"], capture_output=True, text=True)
    assert out.returncode == 1 and "Cannot open" in out.stderr
    out = subprocess.run([tool_path("bibfs_serial"), "gnp:100::1", "0", "100"], capture_output=True, text=True)
    assert out.returncode == 1


def test_gen_tool_and_python_generator(tmp_path):
    b = tmp_path / "10k.bin"
    out = subprocess.run([tool_path("bibfs_gen"), "--type", "gnp", "--n", "10000", "--seed", "1", "--out", str(b)],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    d = json.loads((tmp_path / "10k.json").read_text())
    assert d["hop_count"] == 12
    # C16-compatible python CLI (networkx backend, like the reference)
    out = subprocess.run([sys.executable, "-m", "bidirectional_bfs_amd.models.generate_graph", "--n", "1000",
                          "--p", str(2.2 / 1000), "--seed", "3", "--out", str(tmp_path / "1k.bin")],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    d = json.loads((tmp_path / "1k.json").read_text())
    from bidirectional_bfs_amd import native
    from bidirectional_bfs_amd.models import Graph

    g = Graph.from_bin(str(tmp_path / "1k.bin"))
    r = native.bfs_oracle(g.csr, 0, 999)
    assert (d["hop_count"] if d["hop_count"] is not None else -1) == r.hops
    if r.found:
        ok, why = native.validate_path(g.csr, 0, 999, r.hops, d["nodes"])
        assert ok, why


def test_show_matrix(tmp_path):
    import numpy as np

    from bidirectional_bfs_amd import native

    a = np.eye(3, dtype=np.uint8)
    native.write_dense(str(tmp_path / "graph.bin"), a)
    out = subprocess.run([tool_path("show_matrix")], cwd=tmp_path, capture_output=True, text=True)
    assert out.stdout == "1 0 0\n0 1 0\n0 0 1\n"


def test_python_cli_serial():
    out = subprocess.run([sys.executable, "-m", "bidirectional_bfs_amd", "gnp:10000::1", "0", "9999",
                          "--engine", "serial"], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert "Shortest path length = 12" in out.stdout


def test_read_graph_tool(tmp_path):
    from bidirectional_bfs_amd import native

    native.write_bin(str(tmp_path / "g.bin"), native.gen_gnp(100, 0.05, 1))
    out = subprocess.run([sys.executable, "-m", "bidirectional_bfs_amd.utils.read_graph", str(tmp_path / "g.bin"),
                          "--limit", "3"], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("Loaded CSR with shape (100, 100)")
    assert len(out.stdout.splitlines()) == 4


def test_visual(tmp_path):
    pytest.importorskip("matplotlib")
    out = subprocess.run([tool_path("bibfs_gen"), "--type", "gnp", "--n", "60", "--p", "0.08", "--seed", "2",
                          "--out", str(tmp_path / "v.bin")], capture_output=True, text=True)
    assert out.returncode == 0
    from bidirectional_bfs_amd.utils.visual import draw

    png = draw(str(tmp_path / "v.bin"), str(tmp_path / "v.json"), str(tmp_path / "v.png"), layout="spring")
    assert (tmp_path / "v.png").stat().st_size > 1000 and png.endswith(".png")


def test_ipc_group_control_plane_with_processes():
    """The IPC transport's control plane (csrc/dist/ipc_group.cpp), host only,
    with real processes: 4 ranks rendezvous 2000 times exchanging ping-pong
    values, and a rank that is SIGKILLed, hangs past the timeout or aborts
    makes every other rank fail (not hang)."""
    import json
    import subprocess

    from bidirectional_bfs_amd._lib import tool_path

    for mode, n in (("ok", 2000), ("kill", 50), ("hang", 50), ("abort", 50)):
        r = subprocess.run([tool_path("ipc_group_check"), mode, "4", str(n)], capture_output=True, text=True,
                           timeout=60)
        d = json.loads(r.stdout.strip().splitlines()[-1])
        assert r.returncode == 0 and d["ok"], (mode, r.stdout, r.stderr)
        if mode == "kill":
            assert d["status"][1] == -9 and all(x == 10 for i, x in enumerate(d["status"]) if i != 1), d
