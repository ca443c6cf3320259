#!/bin/bash
# Partitioned-engine GPU check: local-group tests (P = 1..4 ranks on one GPU),
# the world-1 RCCL tests, then a short bench with the partitioned configs.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 600 $PT -m gpu tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/pytest_dist.log 2>&1 && \
$T 400 python bench.py --steps 100 --warmup 10 --extra-graph "" > gpurun_out/bench_dist.json 2> gpurun_out/bench_dist.err
