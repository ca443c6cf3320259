"""Graph models: the reference's G(n, p) suite plus R-MAT / Kronecker.

``Graph`` bundles an edge list (the ``.bin`` payload) and its symmetric CSR.
Generators are native, seeded and multi-threaded; the device generators in
``ops`` produce bit-identical edges on the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from .._lib import native

REFERENCE_SIZES = {"1k": 1000, "10k": 10000, "50k": 50000, "100k": 100000}  # graphs/make_graphs:13
REFERENCE_AVG_DEG = 2.2000000001  # graphs/make_graphs:8


def reference_p(n: int) -> float:
    return native.reference_p(int(n))


@dataclass
class Graph:
    """An undirected graph: edge list + symmetric CSR (built lazily)."""

    edges: "native.EdgeList"
    name: str = "graph"
    _csr: Optional["native.Csr"] = None

    @property
    def n(self) -> int:
        return int(self.edges.n)

    @property
    def m(self) -> int:
        return int(self.edges.m)

    @property
    def csr(self):
        if self._csr is None:
            self._csr = native.build_csr(self.edges)
        return self._csr

    def edge_array(self) -> np.ndarray:
        return self.edges.edges()

    def save_bin(self, path: str) -> None:
        native.write_bin(path, self.edges)

    @staticmethod
    def from_bin(path: str) -> "Graph":
        return Graph(native.read_bin(path), name=path)

    @staticmethod
    def from_edges(n: int, edges) -> "Graph":
        arr = np.ascontiguousarray(np.asarray(edges, dtype=np.uint32).reshape(-1, 2))
        return Graph(native.EdgeList.from_numpy(int(n), arr), name="edges")


def gnp(n: int, p: Optional[float] = None, seed: int = 1) -> Graph:
    """G(n, p) by geometric skipping; default p = 2.2/n (graphs/make_graphs:8)."""
    p = reference_p(n) if p is None else float(p)
    return Graph(native.gen_gnp(int(n), p, int(seed)), name=f"gnp:{n}:{p}:{seed}")


def rmat(n: int, m: int, seed: int = 1, a: float = 0.57, b: float = 0.19, c: float = 0.19) -> Graph:
    return Graph(native.gen_rmat(int(n), int(m), int(seed), a, b, c), name=f"rmat:{n}:{m}:{seed}")


def kronecker(scale: int, edgefactor: int = 16, seed: int = 1) -> Graph:
    return Graph(native.gen_kronecker(int(scale), int(edgefactor), int(seed)), name=f"kron:{scale}:{edgefactor}:{seed}")


def parse_spec(spec: str):
    """Generator spec -> ``(kind, n, arg, seed)``: kind ``"gnp"`` (arg = p) or
    ``"rmat"`` (arg = undirected edge count; ``kron:S:EF`` is R-MAT with
    n = 2^S, m = EF * 2^S).  For engines that generate on the device."""
    f = spec.split(":")
    if f[0] == "gnp":
        n = int(f[1])
        p = float(f[2]) if len(f) > 2 and f[2] else reference_p(n)
        return "gnp", n, p, int(f[3]) if len(f) > 3 else 1
    if f[0] == "rmat":
        return "rmat", int(f[1]), int(f[2]), int(f[3]) if len(f) > 3 else 1
    if f[0] == "kron":
        scale, ef = int(f[1]), int(f[2]) if len(f) > 2 else 16
        return "rmat", 1 << scale, ef << scale, int(f[3]) if len(f) > 3 else 1
    raise ValueError(f"generator spec must be gnp:/rmat:/kron:, got {spec!r}")


def from_spec(spec: str) -> Graph:
    """``gnp:N[:p[:seed]]``, ``rmat:N:M[:seed]``, ``kron:S[:EF[:seed]]`` or a ``.bin`` path."""
    f = spec.split(":")
    if f[0] == "gnp":
        n = int(f[1])
        p = float(f[2]) if len(f) > 2 and f[2] else None
        return gnp(n, p, int(f[3]) if len(f) > 3 else 1)
    if f[0] == "rmat":
        return rmat(int(f[1]), int(f[2]), int(f[3]) if len(f) > 3 else 1)
    if f[0] == "kron":
        return kronecker(int(f[1]), int(f[2]) if len(f) > 2 else 16, int(f[3]) if len(f) > 3 else 1)
    return Graph.from_bin(spec)


__all__ = ["Graph", "gnp", "rmat", "kronecker", "from_spec", "parse_spec", "reference_p", "REFERENCE_SIZES", "REFERENCE_AVG_DEG"]
