#!/bin/bash
# Round 3g: partitioned engine after the terminal-Ctl / local-walk / deferred-cleanup change.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dist_local.py \
  > gpurun_out/r3g_dist_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1,2,4 --queries 24 --reps 2 \
  > gpurun_out/r3g_dist_ab.jsonl 2> gpurun_out/r3g_dist_ab.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_prof_dist -o run -- \
  python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 2 --queries 16 --reps 1 \
  > gpurun_out/r3g_dist_prof.jsonl 2> gpurun_out/r3g_dist_prof.err || exit $?
echo done
