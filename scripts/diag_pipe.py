"""One partitioned query batch per mode (exact / pipelined) with a short engine
timeout: a protocol hang surfaces as the engine's own error, not a test timeout.

  python scripts/diag_pipe.py [graph] [ranks]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time

import torch  # noqa: F401  (binds the HIP runtime first)

import bidirectional_bfs_amd as bb
from bidirectional_bfs_amd import native
from bidirectional_bfs_amd.parallel import dist_local_run, make_tuning

spec = sys.argv[1] if len(sys.argv) > 1 else "gnp:20000::6"
ranks = int(sys.argv[2]) if len(sys.argv) > 2 else 2
g = bb.from_spec(spec)
qs = [(0, g.n - 1), (5, 5), (1, g.n // 2), (5, 7)]
expect = [native.bfs_oracle(g.csr, s, d).hops for s, d in qs]
print("oracle:", expect, flush=True)
for kw in ({}, {"lockstep": False}, {"direction": "topdown"}):
    for pipe in (True, False):
        t0 = time.time()
        try:
            rs, st = dist_local_run(ranks, g, qs, tuning=make_tuning(timeout_s=8.0, pipeline=pipe),
                                    return_stats=True, **kw)
            print(f"{kw} pipeline={pipe} ok {time.time() - t0:.2f}s hops={[r.hops for r in rs]}", flush=True)
            print("  stats:", st if not isinstance(st, list) else st[0], flush=True)
        except Exception as e:  # the engine's own diagnosis
            print(f"{kw} pipeline={pipe} FAILED after {time.time() - t0:.2f}s: {e}", flush=True)
