"""Independent oracles for correctness checks.

``bfs_hops`` uses the native single-source BFS; ``scipy_hops`` uses
``scipy.sparse.csgraph`` (entirely independent code) and ``networkx`` is used
by the C16-compatible generator.  ``check_result`` validates the contract of
SURVEY.md §2.2: exact hop count, a real src->dst walk of that length.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np

from .._lib import native


def bfs_hops(csr, src: int, dst: int) -> int:
    r = native.bfs_oracle(csr, int(src), int(dst))
    return int(r.hops)


def scipy_hops(n: int, edges: np.ndarray, src: int, dst: int) -> int:
    from scipy.sparse import csr_matrix
    from scipy.sparse.csgraph import shortest_path

    e = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    if e.size == 0:
        return 0 if src == dst else -1
    allv = np.vstack([e, e[:, ::-1]])
    a = csr_matrix((np.ones(allv.shape[0]), (allv[:, 0], allv[:, 1])), shape=(n, n))
    d = shortest_path(a, directed=False, unweighted=True, indices=int(src))
    x = d[int(dst)]
    return -1 if not np.isfinite(x) else int(x)


def check_result(csr, src: int, dst: int, hops: int, path: Optional[Sequence[int]], expect: int) -> None:
    if hops != expect:
        raise AssertionError(f"{src}->{dst}: hops {hops} != expected {expect}")
    if expect < 0:
        return
    ok, why = native.validate_path(csr, int(src), int(dst), int(hops), list(path or []))
    if not ok:
        raise AssertionError(f"{src}->{dst}: invalid path ({why})")
