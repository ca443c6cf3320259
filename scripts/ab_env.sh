#!/bin/bash
# A/B latency across environment settings: scripts/ab_env.sh "NAME=ENV..." ...
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab_env.txt
: > $out
GRAPHS=${GRAPHS:-"gnp:100000::6,0,99999 gnp:1000000::2,0,999999 gnp:10000000::1,0,9999999"}
for g in $GRAPHS; do
  IFS=, read spec s d <<< "$g"
  for rep in 1 2; do
    for cfg in "$@"; do
      name=${cfg%%=*}; envs=${cfg#*=}
      r=$(env $envs timeout -k 5 90 ./build/bin/bibfs_hip $spec $s $d --json --repeat 200) || exit 1
      echo "$name $spec $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("hops", d["hops"], "query_ms %.4f search_ms %.4f handoff %s" % (d["query_ms"], d["search_ms"], d["handoff"]))')" >> $out
    done
  done
done
