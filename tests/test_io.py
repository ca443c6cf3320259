"""Formats: .bin edge list, .json sidecar, legacy dense matrix, .csr cache."""
import json
import os
import struct

import numpy as np
import pytest

from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.utils.io import (
    PathJson,
    read_bin_numpy,
    read_graph_csr,
    read_path_json,
    write_bin_numpy,
    write_path_json,
)


def test_bin_roundtrip(tmp_path):
    el = native.gen_gnp(500, 0.01, 3)
    p = str(tmp_path / "g.bin")
    native.write_bin(p, el)
    el2 = native.read_bin(p)
    assert el2.n == el.n and el2.m == el.m
    assert np.array_equal(el2.edges(), el.edges())
    n, e = read_bin_numpy(p)
    assert n == 500 and np.array_equal(e, el.edges())
    # byte layout: u32 N, u32 M, pairs (graphs/generate_graph.py:35-39)
    raw = open(p, "rb").read()
    assert struct.unpack("<II", raw[:8]) == (500, el.m)
    assert len(raw) == 8 + 8 * el.m


def test_bin_truncated_and_bad_ids(tmp_path):
    p = str(tmp_path / "t.bin")
    with open(p, "wb") as f:
        f.write(struct.pack("<II", 10, 5))
        f.write(struct.pack("<II", 1, 2))
    with pytest.raises(RuntimeError, match="Unexpected EOF"):
        native.read_bin(p)
    with open(p, "wb") as f:
        f.write(struct.pack("<IIII", 3, 1, 0, 7))
    with pytest.raises(RuntimeError, match=">= N"):
        native.read_bin(p)
    with pytest.raises(RuntimeError, match="Cannot open"):
        native.read_bin(str(tmp_path / "missing.bin"))


def test_json_sidecar_matches_python_json_dump(tmp_path):
    pj = PathJson(0, 999, 3, [0, 5, 7, 999])
    p1 = str(tmp_path / "a.json")
    write_path_json(p1, pj)
    assert read_path_json(p1) == pj
    # native writer produces json.dump(indent=2) byte-for-byte
    native_out = tmp_path / "b.bin"
    el = native.gen_gnp(1000, native.reference_p(1000), 1)
    native.write_bin(str(native_out), el)
    from bidirectional_bfs_amd._lib import tool_path
    import subprocess

    subprocess.run([tool_path("bibfs_gen"), "--type", "gnp", "--n", "1000", "--seed", "1",
                    "--out", str(native_out)], check=True, capture_output=True)
    txt = open(tmp_path / "b.json").read()
    d = json.loads(txt)
    assert txt == json.dumps(d, indent=2)
    assert d["source"] == 0 and d["target"] == 999 and d["hop_count"] == 9 and len(d["nodes"]) == 10
    # unreachable -> null + []
    subprocess.run([tool_path("bibfs_gen"), "--type", "gnp", "--n", "100000", "--seed", "1",
                    "--out", str(tmp_path / "c.bin")], check=True, capture_output=True)
    d = json.loads(open(tmp_path / "c.json").read())
    assert d["hop_count"] is None and d["nodes"] == []


def test_sidecar_path():
    assert native.sidecar_path("graphs/1k.bin") == "graphs/1k.json"
    assert native.sidecar_path("../graphs/1k.bin") == "../graphs/1k.json"
    assert native.sidecar_path("noext") == "noext.json"


def test_dense_legacy(tmp_path):
    a = (np.random.default_rng(0).random((6, 6)) > 0.5).astype(np.uint8)
    p = str(tmp_path / "graph.bin")
    native.write_dense(p, a)
    assert np.array_equal(native.read_dense(p), a)
    with open(p, "ab") as f:
        f.write(b"\0")
    with pytest.raises(RuntimeError, match="Size mismatch"):
        native.read_dense(p)


def test_csr_cache_roundtrip(tmp_path):
    g = native.build_csr(native.gen_gnp(2000, 0.002, 5))
    p = str(tmp_path / "g.csr")
    native.write_csr_cache(p, g)
    h = native.read_csr_cache(p)
    assert h.n == g.n and h.m_input == g.m_input
    assert np.array_equal(h.row_off, g.row_off) and np.array_equal(h.col, g.col)


def test_read_graph_csr_scipy(tmp_path):
    n, e = 7, np.array([[0, 1], [1, 2], [5, 6]], dtype=np.uint32)
    p = str(tmp_path / "s.bin")
    write_bin_numpy(p, n, e)
    A = read_graph_csr(p)
    assert A.shape == (7, 7) and A.nnz == 6
    assert A[1, 0] == 1 and A[6, 5] == 1
