"""Diagnostic: do owner-addressed rounds spill, and does a shrunk spill list
(DistTuning.spill_cap) fail the search?  Prints per-query round statistics."""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bidirectional_bfs_amd as bb  # noqa: E402
from bidirectional_bfs_amd.parallel import dist_proc_matrix  # noqa: E402

for spec in ("gnp:20000::6", "rmat:16384:262144:3"):
    g = bb.from_spec(spec)
    rnd = random.Random(71)
    qs = [(0, g.n - 1)] + [(rnd.randrange(g.n), rnd.randrange(g.n)) for _ in range(6)]
    runs = [({"_catch": True, "direction": "topdown"}, {"owner_cap": 2, "spill_cap": 1}),
            ({"_catch": True, "direction": "topdown"}, {"owner_cap": 2, "spill_cap": 0}),
            ({"_catch": True}, {"owner_cap": 2, "spill_cap": 1})]
    got, outs = dist_proc_matrix(3, g, qs, runs)
    for i, (rs, st, run) in enumerate(got):
        print(json.dumps({"spec": spec, "run": i, "hops": [r.hops for r in rs],
                          "errors": [r.get("error", "")[:60] for r in run["results"]],
                          "cont": [x.get("cont_rounds") for x in st], "spec_rounds": [x.get("spec_rounds") for x in st],
                          "host_rounds": [x.get("host_rounds") for x in st],
                          "small": [x.get("small_expand_rounds") for x in st]}), flush=True)
