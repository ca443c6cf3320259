#!/usr/bin/env python3
"""Host-oracle hop counts (plain BFS on the host CSR) for a few pairs of a
generated graph, beside the GPU engine's resident / grid-only answers.

    python benchmarks/oracle_pairs.py kron:27:16:1 S:D [S:D ...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    spec = sys.argv[1]
    pairs = [tuple(int(x) for x in p.split(":")) for p in sys.argv[2:]]
    import torch  # noqa: F401
    import bench
    import bidirectional_bfs_amd as bb
    from bidirectional_bfs_amd import native
    from bidirectional_bfs_amd.ops import HipEngine, make_options

    g = bb.from_spec(spec)
    print(json.dumps({"host_graph": spec, "n": g.n}), flush=True)
    eng = HipEngine(0).load(g)
    for s, d in pairs:
        o = native.bfs_oracle(g.csr, s, d).hops
        r = eng.search(s, d)
        f = eng.search(s, d, make_options(force_grid=True))
        print(json.dumps({"pair": [s, d], "oracle": o, "engine": r.hops, "grid": f.hops, "engine_path": list(r.path),
                          "grid_path": list(f.path), "handoff": r.handoff}), flush=True)


if __name__ == "__main__":
    main()
