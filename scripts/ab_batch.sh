#!/bin/bash
# A/B of batched serving (bench.py's batched block: 256 queries per launch) on
# the secondary configs, per library variant in build/var, interleaved.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_batch.txt
: > $out
for rep in 1 2; do
  for g in ${GRAPHS:-gnp:10000000::1 kron:22:16:1}; do
    for d in build/var/*/; do
      v=$(basename $d)
      r=$(LD_LIBRARY_PATH=$d timeout -k 5 120 python3 bench.py --graph $g --steps 80 --warmup 10 --extra-graph "" \
          --dist-graphs "" --batch 256 --no-cpu-ref 2>/dev/null | tail -1) || exit 1
      echo "$v $g $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read())["detail"]["batched_serving"]; print("us_per_query %.3f fallbacks %.2f" % (d["us_per_query"], d["fallback_queries_per_batch"]))')" >> $out
    done
  done
done
