"""C19 capability (reference ``visual/m3.py``): draw a graph with the shortest
path from its ``.json`` sidecar highlighted (Kamada-Kawai layout, path edges
red).  Writes a PNG instead of opening a window so it works headless.

    python -m bidirectional_bfs_amd.utils.visual graphs/1k.bin [--json graphs/1k.json] [--out path.png]
"""
from __future__ import annotations

import argparse
import sys


def draw(bin_path: str, json_path: str, out: str, font_size: int = 10, layout: str = "kamada_kawai") -> str:
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    import networkx as nx

    from .io import read_bin_numpy, read_path_json

    n, e = read_bin_numpy(bin_path)
    G = nx.Graph()
    G.add_nodes_from(range(n))
    G.add_edges_from(map(tuple, e.tolist()))
    nodes = read_path_json(json_path).nodes
    marked = list(zip(nodes, nodes[1:]))
    ms = set(marked) | {(v, u) for u, v in marked}
    other = [x for x in G.edges() if x not in ms]
    plt.figure(figsize=(8, 8))
    pos = nx.kamada_kawai_layout(G) if layout == "kamada_kawai" else nx.spring_layout(G, seed=0)
    nx.draw_networkx_nodes(G, pos, node_size=50)
    nx.draw_networkx_edges(G, pos, alpha=0.0, edgelist=other)
    nx.draw_networkx_edges(G, pos, alpha=0.4, edgelist=marked, edge_color="red", width=5.0)
    nx.draw_networkx_labels(G, pos, font_size=font_size)
    plt.title(f"Graph with {G.number_of_nodes()} nodes and {G.number_of_edges()} edges")
    plt.axis("off")
    plt.tight_layout()
    plt.savefig(out)
    plt.close()
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("bin")
    ap.add_argument("--json", default=None)
    ap.add_argument("--out", default="path.png")
    ap.add_argument("--layout", default="kamada_kawai", choices=["kamada_kawai", "spring"])
    a = ap.parse_args(argv)
    from .io import default_sidecar

    print(draw(a.bin, a.json or default_sidecar(a.bin), a.out, layout=a.layout))
    return 0


if __name__ == "__main__":
    sys.exit(main())
