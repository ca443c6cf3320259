#!/bin/bash
# Round 3n: partitioned bench entries alone vs dist_ab on the same box.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --extra-graph "" --batch 0 --dist-graphs gnp:1000000::2,kron:22:16:1 \
  > gpurun_out/r3n_bench.json 2> gpurun_out/r3n_bench.err || exit $?
timeout -k 10 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2 --modes 1 --queries 24 --reps 2 \
  > gpurun_out/r3n_ab.jsonl 2> gpurun_out/r3n_ab.err || exit $?
echo done
