#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist_local.py \
  > gpurun_out/r3q_dist_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22,kron:27 --modes 1 --queries 24 --reps 2 --slow-ms 0.3 \
  > gpurun_out/r3q_ab.jsonl 2> gpurun_out/r3q_ab.err || exit $?
echo done
