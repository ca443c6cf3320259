"""Graph file formats (reference SURVEY.md §2.6).

* ``.bin``: little-endian ``u32 N, u32 M`` then ``M`` pairs ``(u32 u, u32 v)``
  (writer ``graphs/generate_graph.py:35-39``).
* ``.json`` sidecar: ``{"source", "target", "hop_count" (int|null), "nodes"}``
  with ``indent=2`` (``graphs/generate_graph.py:53-62``).

The heavy lifting (mmap read, validation) is native; the numpy helpers here
are for tests and scripts.  ``read_graph_csr`` is the C18 capability
(``graphs/read_graph.py:4-22``): a symmetric scipy CSR of the edge list.
"""
from __future__ import annotations

import json
import os
import struct
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from .._lib import native

read_bin = native.read_bin
write_bin = native.write_bin
sidecar_path = native.sidecar_path


def read_bin_numpy(path: str):
    """Return ``(n, edges[M, 2] uint32)`` with size validation."""
    with open(path, "rb") as f:
        hdr = f.read(8)
        if len(hdr) < 8:
            raise ValueError(f"Unexpected EOF reading header of {path}")
        n, m = struct.unpack("<II", hdr)
        e = np.fromfile(f, dtype="<u4", count=2 * m)
    if e.size != 2 * m:
        raise ValueError(f"Unexpected EOF reading edges of {path}")
    return int(n), e.reshape(-1, 2)


def write_bin_numpy(path: str, n: int, edges) -> None:
    edges = np.ascontiguousarray(np.asarray(edges, dtype="<u4").reshape(-1, 2))
    with open(path, "wb") as f:
        f.write(struct.pack("<II", int(n), int(edges.shape[0])))
        edges.tofile(f)


def edges_numpy(el) -> np.ndarray:
    return el.edges()


def read_graph_csr(path: str):
    """C18: symmetric scipy CSR (0/1 uint8) of a ``.bin`` edge list."""
    from scipy.sparse import csr_matrix

    n, e = read_bin_numpy(path)
    allv = np.vstack([e, e[:, ::-1]]) if e.size else np.zeros((0, 2), np.uint32)
    data = np.ones(allv.shape[0], dtype=np.uint8)
    return csr_matrix((data, (allv[:, 0], allv[:, 1])), shape=(n, n))


@dataclass
class PathJson:
    source: int
    target: int
    hop_count: Optional[int]
    nodes: List[int] = field(default_factory=list)


def write_path_json(path: str, pj: PathJson) -> None:
    with open(path, "w") as f:
        json.dump(
            {"source": pj.source, "target": pj.target, "hop_count": pj.hop_count, "nodes": list(pj.nodes)},
            f,
            indent=2,
        )


def read_path_json(path: str) -> PathJson:
    with open(path) as f:
        d = json.load(f)
    return PathJson(int(d["source"]), int(d["target"]), d.get("hop_count"), [int(x) for x in d.get("nodes", [])])


def default_sidecar(bin_path: str) -> str:
    root, _ = os.path.splitext(bin_path)
    return root + ".json"
