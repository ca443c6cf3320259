#!/bin/bash
# Round 3k: dist tests (local groups P=1..4) + world-1 A/B after the gathered reduction.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist_local.py \
  > gpurun_out/r3k_dist_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 benchmarks/dist_shard.py --specs gnp:1000000::2,kron:22 --ranks 1,2,4 --queries 16 > gpurun_out/r3k_dist_shard.jsonl 2> gpurun_out/r3k_dist_shard.err || exit $?
echo done
