#!/usr/bin/env python3
"""Print the bibfs_hip --json lines of gpurun_out/lat.txt as a table."""
import json
import sys

for line in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lat.txt"):
    if line.startswith("{"):
        d = json.loads(line)
        print(f"{d['graph']:>18} hops {d['hops']:>3} query_ms {d['query_ms']:.4f} search_ms {d['search_ms']:.4f} "
              f"handoff {d['handoff']}")
