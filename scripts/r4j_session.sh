#!/bin/bash
# Round-4 session j: partitioned-engine GPU tests incl. the 8-rank rehearsal.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 180 --timeout-method thread"
$T 900 $PT -m gpu tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/r4j_pytest.log 2>&1
