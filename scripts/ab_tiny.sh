#!/bin/bash
# A/B of the small-graph server variants in build/var (scripts/build_tiny_variants.sh):
# benchmarks/tiny_latency.py per variant, twice, interleaved.
set -o pipefail
out=gpurun_out/ab_tiny.jsonl
: > $out
for rep in 1 2; do
  for d in build/var/*/; do
    v=$(basename $d)
    LD_LIBRARY_PATH=$d timeout -k 5 120 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/ab_tiny_one.jsonl 2>gpurun_out/ab_tiny_one.err || { cat gpurun_out/ab_tiny_one.err | tail -5; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_tiny_one.jsonl').readline()); d['variant']='$v'; print(json.dumps(d))" >> $out
  done
done
cat $out
