"""C18 capability (reference ``graphs/read_graph.py``): load a ``.bin`` as a
symmetric scipy CSR and print every directed edge.

    python -m bidirectional_bfs_amd.utils.read_graph graphs/1k.bin [--limit K]
"""
from __future__ import annotations

import argparse
import sys

from .io import read_graph_csr


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("bin")
    ap.add_argument("--limit", type=int, default=None, help="print at most this many edges")
    a = ap.parse_args(argv)
    A = read_graph_csr(a.bin)
    print("Loaded CSR with shape", A.shape, "and", A.nnz, "nonzeros")
    rows, cols = A.nonzero()
    for i, (u, v) in enumerate(zip(rows, cols)):
        if a.limit is not None and i >= a.limit:
            break
        print(f"{u} -> {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
