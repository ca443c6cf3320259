#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/dist_ab.py --specs kron:22,kron:27 --modes 1 --queries 24 --reps 2 --slow-ms 0.3 \
  > gpurun_out/r3p_slow.jsonl 2> gpurun_out/r3p_slow.err || exit $?
echo done
