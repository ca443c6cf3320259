import sys, os, json
sys.path.insert(0, os.getcwd())
import torch  # noqa
import bench
from bidirectional_bfs_amd.ops import HipEngine, make_options
spec = sys.argv[1] if len(sys.argv) > 1 else "kron:27:16:1"
pairs = [tuple(int(x) for x in a.split(":")) for a in sys.argv[2:]] or [(26740478, 130093872)]
eng = bench.generate(HipEngine(0), spec)
for s, d in pairs:
    for resident in (False, True):
        for probe in (16384, 0):
            eng.lds_probe_edges = probe
            eng.set_resident(resident)
            r = eng.search(s, d)
            st = r.stats
            print(json.dumps({"resident": resident, "probe": probe, "hops": r.hops, "handoff": r.handoff,
                              "probe_hit": st["probe_hit"], "probe_edges": st["probe_edges"], "lds_levels": st["lds_levels"],
                              "grid_levels": st["grid_levels"], "path": list(r.path)}), flush=True)
        eng.set_resident(False)
    r = eng.search(s, d, make_options(force_grid=True))
    print(json.dumps({"force_grid": True, "hops": r.hops, "path": list(r.path)}), flush=True)
    for fg in (False, True):
        r = eng.search(s, d, make_options(trace=True, force_grid=fg))
        print(json.dumps({"trace": True, "force_grid": fg, "hops": r.hops, "levels": [(t["side"], t["depth"], t["frontier"], t["edges"], t["discovered"], t["mode"]) for t in r.stats["trace"]]}), flush=True)
