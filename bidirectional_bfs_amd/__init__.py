"""bidirectional_bfs_amd -- an MI355X-native bidirectional BFS framework.

Capabilities of Tomaszbrauntsch/Bidirectional-BFS (four engine tiers, the
``<graph.bin> <src> <dst>`` CLI, the ``.bin`` + ``.json`` formats, the
benchmark harness) re-designed for AMD Instinct MI355X (gfx950):

=================  =====================================  ==========================
reference          here                                   where
=================  =====================================  ==========================
v1 serial          ``SerialEngine`` / ``bibfs_serial``    csrc/cpu/serial_bibfs.cpp
v2 MPI bitmap      ``run_mpi('second_try')``              csrc/cpu/mpi_bitmap_bibfs.cpp
v2 MPI list proto  ``run_mpi('mpi_queue_bibfs')``         csrc/cpu/mpi_queue_bibfs.cpp
v3 CUDA            ``ops.HipEngine`` / ``bibfs_hip``      csrc/hip/engine_kernels.hip
v4 MPI+CUDA        ``parallel.DistEngine`` / mpi_bibfs    csrc/dist/dist_engine.hip
v4 comp.h C API    ``bibfs_hip.h``                        csrc/hip/capi.hip
generate_graph.py  ``models.generate_graph``              + native ``bibfs_gen``
read_graph.py      ``utils.read_graph``                   scipy CSR
visual/m3.py       ``utils.visual``                       matplotlib (headless)
benchmark_test.sh  ``scripts/benchmark_test.sh``          + bench.py, bibfs_bench
=================  =====================================  ==========================
"""
from __future__ import annotations

from ._lib import BibfsError, native
from .models import Graph, from_spec, gnp, kronecker, reference_p, rmat

__version__ = "0.1.0"


class SerialEngine:
    """v1 capability: serial bidirectional BFS on the CPU."""

    def __init__(self, graph: "Graph"):
        self.graph = graph
        self._e = native.SerialBiBfs(graph.csr)

    def search(self, src: int, dst: int, options=None, **kw):
        from .ops import make_options

        return self._e.search(int(src), int(dst), options if options is not None else make_options(**kw))


def shortest_path(graph: "Graph", src: int, dst: int, engine: str = "auto", device: int = 0):
    """One-call convenience: returns a SearchResult (hops, path, timings)."""
    if engine == "serial":
        return SerialEngine(graph).search(src, dst)
    from .ops import HipEngine

    return HipEngine(device).load(graph).search(src, dst)


__all__ = [
    "BibfsError",
    "Graph",
    "SerialEngine",
    "from_spec",
    "gnp",
    "kronecker",
    "native",
    "reference_p",
    "rmat",
    "shortest_path",
]
