"""Utilities: graph file I/O, oracles, timing (no GPU needed)."""
from .io import (  # noqa: F401
    PathJson,
    edges_numpy,
    read_bin,
    read_bin_numpy,
    read_graph_csr,
    read_path_json,
    sidecar_path,
    write_bin,
    write_bin_numpy,
    write_path_json,
)
from .oracle import bfs_hops, check_result, scipy_hops  # noqa: F401
