#!/bin/bash
# Round-4 session e: phase stamps of the small P > 1 rounds on the local group.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 300 $PT -m gpu tests/test_gpu_dist_local.py -k "stamps or capped or local_group_matches or owner" > gpurun_out/r4e_pytest.log 2>&1 && \
$T 600 python3 benchmarks/dist_rounds.py --specs gnp:1000000::2 --ranks 2,4 --overlap 0 --queries 16 > gpurun_out/r4e_dist_rounds.jsonl 2> gpurun_out/r4e_dist_rounds.err
