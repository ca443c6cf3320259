#!/bin/bash
# A/B latency of the variants in build/var (see scripts/build_variants.sh):
# bibfs_hip resident on (0, N-1) of 100k / 1M, and the bench's own 100k query
# loop (64 connected pairs rotated, resident server) per variant.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab.txt
: > $out
for g in "gnp:100000::6 0 99999" "gnp:1000000::2 0 999999" "gnp:10000000::1 0 9999999"; do
  for rep in 1 2; do
    for d in build/var/*/; do
      v=$(basename $d)
      r=$(LD_LIBRARY_PATH=$d timeout -k 5 60 ./build/bin/bibfs_hip $g --json --repeat 300 --resident) || exit 1
      echo "$v $g $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("hops", d["hops"], "query_ms %.4f search_ms %.4f" % (d["query_ms"], d["search_ms"]))')" >> $out
    done
  done
done
for rep in 1 2; do
  for d in build/var/*/; do
    v=$(basename $d)
    r=$(LD_LIBRARY_PATH=$d timeout -k 5 120 python3 bench.py --steps 800 --warmup 50 --extra-graph "" --dist-graphs "" \
        --batch 0 --no-cpu-ref 2>/dev/null | tail -1) || exit 1
    echo "$v bench100k $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("query_ms %.4f device_ms %.4f" % (d["ms_per_step"], d["detail"]["device_ms_per_query"]))')" >> $out
  done
done
