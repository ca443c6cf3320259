#!/usr/bin/env python3
"""C16-compatible graph generator (reference ``graphs/generate_graph.py``).

Same flags (``--n --p --src --dst --out``), same outputs: ``<out>`` as a
``.bin`` edge list and ``<stem>.json`` with the shortest path.  Additions:
``--seed`` (the reference is unseeded), ``--backend`` (``networkx`` =
``fast_gnp_random_graph`` exactly like the reference; ``native`` = the seeded
C++ generator, needed beyond ~1M nodes) and no O(N^2) dense matrix
(the reference builds one it never uses, generate_graph.py:32).
"""
from __future__ import annotations

import argparse
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Generate a random G(n,p) graph (.bin) and its shortest path (.json)")
    ap.add_argument("--n", type=int, default=50000, help="number of nodes")
    ap.add_argument("--p", type=float, default=3 / 129000, help="edge probability")
    ap.add_argument("--src", type=int, default=0, help="source node")
    ap.add_argument("--dst", type=int, default=None, help="destination node (default n-1)")
    ap.add_argument("--out", type=str, default="50k.bin", help="file to write as")
    ap.add_argument("--seed", type=int, default=None, help="RNG seed (reference: unseeded)")
    ap.add_argument("--backend", choices=["auto", "networkx", "native"], default="auto")
    a = ap.parse_args(argv)
    n, p = a.n, a.p
    src = a.src
    dst = a.dst if a.dst is not None else n - 1
    backend = a.backend
    if backend == "auto":
        backend = "networkx" if n <= 200000 else "native"
    print(f"Generating G({n}, p={p})…")
    if backend == "networkx":
        import networkx as nx
        import numpy as np

        from ..utils.io import write_bin_numpy

        G = nx.fast_gnp_random_graph(n, p, seed=a.seed, directed=False)
        edges = np.array(list(G.edges()), dtype=np.uint32).reshape(-1, 2)
        write_bin_numpy(a.out, n, edges)
        print(f"Computing shortest path from {src} to {dst}…")
        try:
            nodes = nx.shortest_path(G, source=src, target=dst)
            hop = len(nodes) - 1
            print(f"  → hop count = {hop}")
        except nx.NetworkXNoPath:
            nodes, hop = [], None
            print("  → no path found")
    else:
        from .._lib import native

        el = native.gen_gnp(n, p, 1 if a.seed is None else a.seed)
        native.write_bin(a.out, el)
        print(f"Computing shortest path from {src} to {dst}…")
        r = native.bfs_oracle(native.build_csr(el), src, dst)
        nodes, hop = (list(r.path), int(r.hops)) if r.found else ([], None)
        print(f"  → hop count = {hop}" if r.found else "  → no path found")
    from ..utils.io import PathJson, default_sidecar, write_path_json

    out_json = default_sidecar(a.out)
    write_path_json(out_json, PathJson(src, dst, hop, [int(x) for x in nodes]))
    print("Wrote path info to", out_json)
    return 0


if __name__ == "__main__":
    sys.exit(main())
