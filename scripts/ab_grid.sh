#!/bin/bash
# A/B of the grid-level variants in build/var (scripts/build_variants.sh) on
# the bench's secondary configs: 10M G(n,p) and Kronecker 22, resident server,
# interleaved, 2 reps.  Writes gpurun_out/ab_grid.txt.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_grid.txt
: > $out
for rep in 1 2; do
  for g in ${GRAPHS:-gnp:10000000::1 kron:22:16:1}; do
    for d in build/var/*/; do
      v=$(basename $d)
      r=$(LD_LIBRARY_PATH=$d timeout -k 5 120 python3 bench.py --graph $g --steps 200 --warmup 20 --extra-graph "" \
          --dist-graphs "" --batch 0 --no-cpu-ref 2>/dev/null | tail -1) || exit 1
      echo "$v $g $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("query_ms %.4f device_ms %.4f" % (d["ms_per_step"], d["detail"]["device_ms_per_query"]))')" >> $out
    done
  done
done
