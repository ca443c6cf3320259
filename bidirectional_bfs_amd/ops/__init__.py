"""MI355X compute path: the hand-written HIP/CDNA4 kernels behind a Python API.

``HipEngine`` owns one GPU's copy of a graph (CSR in HBM, built on the device)
and answers shortest-path queries with the single-workgroup LDS engine,
handing large frontiers to the grid engine (top-down / bottom-up with a
Beamer switch).  No CPU fallback: constructing it without a GPU raises.
"""
from __future__ import annotations

from typing import Optional

from .._lib import native
from ..models import Graph

SearchOptions = native.SearchOptions
SidePolicy = native.SidePolicy
Direction = native.Direction


def make_options(
    side: str = "edges",
    direction: str = "auto",
    alpha: float = 14.0,
    beta: float = 24.0,
    want_path: bool = True,
    force_grid: bool = False,
    trace: bool = False,
    lockstep: bool = True,
) -> "native.SearchOptions":
    o = native.SearchOptions()
    o.side = {"edges": SidePolicy.SMALLER_EDGES, "frontier": SidePolicy.SMALLER_FRONTIER,
              "alternate": SidePolicy.ALTERNATE}[side]
    o.direction = {"auto": Direction.AUTO, "topdown": Direction.TOPDOWN, "bottomup": Direction.BOTTOMUP}[direction]
    o.alpha, o.beta = float(alpha), float(beta)
    o.want_path, o.force_grid, o.trace = bool(want_path), bool(force_grid), bool(trace)
    o.lockstep = bool(lockstep)
    return o


_DEFAULT_OPTIONS = make_options()


class HipEngine:
    """Single-GPU bidirectional BFS (v3 capability)."""

    def __init__(self, device: int = 0):
        self._e = native.HipBiBfs(int(device))
        # the serving call goes straight to the native method (no Python frame
        # per query); `query` below documents it
        self.query = self._e.query

    # ---- ingest
    def load(self, graph: Graph, build_on_device: bool = True) -> "HipEngine":
        if build_on_device:
            self._e.load_edges(graph.edges)
        else:
            self._e.load_csr(graph.csr)
        return self

    def load_csr(self, csr) -> "HipEngine":
        self._e.load_csr(csr)
        return self

    def generate_gnp(self, n: int, p: Optional[float] = None, seed: int = 1) -> "HipEngine":
        self._e.generate_gnp(int(n), native.reference_p(int(n)) if p is None else float(p), int(seed))
        return self

    def generate_rmat(self, n: int, m: int, seed: int = 1, a=0.57, b=0.19, c=0.19) -> "HipEngine":
        self._e.generate_rmat(int(n), int(m), int(seed), a, b, c)
        return self

    # ---- queries
    def search(self, src: int, dst: int, options: Optional["native.SearchOptions"] = None, **kw):
        if options is None:
            options = make_options(**kw) if kw else _DEFAULT_OPTIONS
        return self._e.search(int(src), int(dst), options)

    def query(self, src: int, dst: int):
        """Serving entry point: ``(hops, path)`` with hops = -1 when there is no
        path.  With ``set_resident(True)`` a small graph (n <= 2^17) is answered
        by the resident tiny server (csrc/hip/tiny_engine.hip: one launch for
        the engine's lifetime, one mailbox round trip per query); everything
        else goes through ``search``."""
        return self._e.query(src, dst)

    @property
    def last_search_ms(self) -> float:
        """Device time of the last ``query`` (request seen -> answer written)."""
        return self._e.last_search_ms

    @property
    def last_edges_inspected(self) -> int:
        return self._e.last_edges_inspected

    @property
    def tiny_overflows(self) -> int:
        """Queries the tiny server could not hold (re-run on the general engine), cumulative."""
        return self._e.tiny_overflows

    @property
    def tiny_engine(self) -> bool:
        """The loaded graph carries the tiny server's packed adjacency."""
        return self._e.tiny_engine

    def search_batch(self, pairs, options: Optional["native.SearchOptions"] = None, **kw):
        """Answer many queries with one launch, one CU per query (throughput serving)."""
        if options is None:
            options = make_options(**kw) if kw else _DEFAULT_OPTIONS
        src = [int(s) for s, _ in pairs]
        dst = [int(d) for _, d in pairs]
        return self._e.search_batch(src, dst, options)

    def search_batch_arrays(self, src, dst, options: Optional["native.SearchOptions"] = None, **kw):
        """Batched queries with a compact result: (hops[K] (-1 = no path), path offsets[K+1], flat paths)."""
        import numpy as np

        if options is None:
            options = make_options(**kw) if kw else _DEFAULT_OPTIONS
        return self._e.search_batch_arrays(np.asarray(src, dtype=np.uint32), np.asarray(dst, dtype=np.uint32),
                                           options)

    def release(self) -> None:
        """Free the graph and search state on the device."""
        self._e.release()

    # resident query server (no kernel launch per query; see docs/DESIGN.md)
    def set_resident(self, on: bool = True, idle_ms: float = 200.0) -> "HipEngine":
        """Serve queries from a resident workgroup (no kernel launch per query).

        The server kernel stays on the GPU until ``idle_ms`` pass without a
        query, so a device-wide synchronize (``torch.cuda.synchronize()``)
        waits for it: call ``set_resident(False)`` before one (the next query
        with ``set_resident(True)`` relaunches it).
        """
        self._e.set_resident(bool(on), float(idle_ms))
        return self

    @property
    def batch_edge_cap(self) -> int:
        """Largest level (frontier edges) the batched HBM-bitmap pass expands
        before handing the query to the single-query engine."""
        return self._e.batch_edge_cap

    @batch_edge_cap.setter
    def batch_edge_cap(self, edges: int) -> None:
        self._e.batch_edge_cap = int(edges)

    @property
    def last_batch_fallbacks(self) -> int:
        """Queries of the last batched call that were re-run one by one through
        ``search`` (a level above ``batch_edge_cap``, a path longer than the
        batch path slot)."""
        return self._e.last_batch_fallbacks

    def set_batch_tuning(self, lds_first: int = -1, threads: int = 0) -> "HipEngine":
        """Batched serving knobs: LDS pass first (1), HBM-bitmap pass only (0) or
        auto by graph size (-1); HBM-pass workgroup size 256/1024 (0 = auto)."""
        self._e.set_batch_tuning(int(lds_first), int(threads))
        return self

    @property
    def resident(self) -> bool:
        return self._e.resident

    @property
    def auto_handoff(self) -> bool:
        """Resident searches enqueue their first grid level before they start,
        gated on the device (no host round trip when a search leaves LDS)."""
        return self._e.auto_handoff

    @auto_handoff.setter
    def auto_handoff(self, on: bool) -> None:
        self._e.auto_handoff = bool(on)

    @property
    def auto_gate_timeout_us(self) -> float:
        """How long the gated first grid level waits on the device for its
        search to leave LDS (default 6 s, above the host's 5 s server wait)."""
        return self._e.auto_gate_timeout_us

    @auto_gate_timeout_us.setter
    def auto_gate_timeout_us(self, us: float) -> None:
        self._e.auto_gate_timeout_us = float(us)

    @property
    def auto_gate_misses(self) -> int:
        """Hand-offs the gated level missed (gave up first); each continued
        on the host from the LDS engine's mirror."""
        return self._e.auto_gate_misses

    @property
    def auto_levels(self) -> int:
        """Device-planned grid levels chained behind the hand-off (1-8): each
        level's finisher plans the next, so no host round trip between them."""
        return self._e.auto_levels

    @auto_levels.setter
    def auto_levels(self, levels: int) -> None:
        self._e.auto_levels = int(levels)

    @property
    def auto_max_degree(self) -> int:
        """The device hand-off runs on graphs whose largest degree is at most
        this (default 64)."""
        return self._e.auto_max_degree

    @auto_max_degree.setter
    def auto_max_degree(self, deg: int) -> None:
        self._e.auto_max_degree = int(deg)

    @property
    def lds_probe_edges(self) -> int:
        """Meet probe of the LDS engine on hub graphs: frontier edges of a level
        that does not fit LDS tested against the other side's visited set
        before the level is handed to the grid engine (default 16384; 0 = off).  ``stats["probe_edges"]`` /
        ``stats["probe_hit"]`` report it per search."""
        return self._e.lds_probe_edges

    @lds_probe_edges.setter
    def lds_probe_edges(self, edges: int) -> None:
        self._e.lds_probe_edges = int(edges)

    def set_build_flags(self, wide_offsets: bool = False, stream_gen: bool = False,
                        tiny: bool = True) -> "HipEngine":
        """Applied by the next load / generate: ``wide_offsets`` keeps no 32-bit
        row-offset copy (a small graph then runs the kernels of an nnz >= 2^32
        graph), ``stream_gen`` generates even small graphs straight into the
        CSR (the large-graph path), ``tiny=False`` keeps the tiny server off
        (the general resident server answers every graph)."""
        self._e.set_build_flags(bool(wide_offsets), bool(stream_gen), bool(tiny))
        return self

    # step-wise API (reference v4/comp.h parity)
    def begin(self, src: int, dst: int) -> None:
        self._e.begin(int(src), int(dst))

    def expand(self, side: int, direction: str = "topdown"):
        d = Direction.BOTTOMUP if direction == "bottomup" else Direction.TOPDOWN
        return self._e.expand(int(side), d)

    def check_meet(self) -> bool:
        return self._e.check_meet()

    def finish(self):
        return self._e.finish()

    # ---- introspection
    @property
    def n(self) -> int:
        return self._e.n

    @property
    def m(self) -> int:
        return self._e.m_input

    @property
    def nnz(self) -> int:
        return self._e.nnz

    @property
    def build_ms(self) -> float:
        return self._e.last_build_ms

    @property
    def device_bytes(self) -> int:
        return self._e.device_bytes

    def info(self):
        return self._e.info()

    def download_csr(self):
        return self._e.download_csr()

    def download_edges(self):
        return self._e.download_edges()

    def neighbors(self, u: int):
        """Row ``u`` of the device CSR (one row copied to the host)."""
        return self._e.neighbors(int(u))

    def check_path(self, src: int, dst: int, hops: int, path) -> bool:
        """``path`` is a src -> dst walk of ``hops`` edges of the loaded graph
        (each edge checked against its row on the device)."""
        p = [int(x) for x in path]
        if len(p) != hops + 1 or p[0] != src or p[-1] != dst:
            return False
        return all(b in set(self._e.neighbors(a)) for a, b in zip(p, p[1:]))

    def synchronize(self) -> None:
        self._e.synchronize()

    @property
    def native(self):
        return self._e


__all__ = ["HipEngine", "make_options", "SearchOptions", "SidePolicy", "Direction"]
