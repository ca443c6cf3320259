#!/bin/bash
# Round 3i: solo-kernel stamps + solo edge-cap A/B at world 1 + dist tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist_local.py \
  > gpurun_out/r3i_dist_tests.log 2>&1 || exit $?
BIBFS_DIST_STAMP=1 timeout -k 10 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1:2048 --queries 8 --reps 1 \
  > gpurun_out/r3i_stamp.jsonl 2> gpurun_out/r3i_stamp.err || exit $?
timeout -k 10 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1:2048,1:4096,2:2048 --queries 24 --reps 2 \
  > gpurun_out/r3i_ab.jsonl 2> gpurun_out/r3i_ab.err || exit $?
echo done
