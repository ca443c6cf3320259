#!/bin/bash
# Round 3z: tiny-server A/B -- 16-byte first-edge loads (x4) vs one 8-byte
# load per edge word (base), build/var from scripts/build_tiny_variants.sh;
# then the tiny GPU tests on the in-tree build and a bench line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
out=gpurun_out/r3z_tiny_ab.jsonl
: > $out
for rep in 1 2; do
  for v in base x4; do
    LD_LIBRARY_PATH=build/var/$v $T 120 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/r3z_one.jsonl 2> gpurun_out/r3z_one_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/r3z_one.jsonl').readline()); d['variant']='$v'; print(json.dumps(d))" >> $out
  done
done
echo done
