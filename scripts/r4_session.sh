#!/bin/bash
# Round-4 working session on the GPU box (scratch; the durable entry point is
# scripts/gpu_tasks.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 600 $PT -m gpu tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/r4c_pytest.log 2>&1 && \
$T 600 python3 benchmarks/dist_rounds.py --specs gnp:1000000::2,kron:22 --ranks 2,4 --overlap 0 --queries 16 > gpurun_out/r4c_dist_rounds.jsonl 2> gpurun_out/r4c_dist_rounds.err
[ $? -eq 0 ] && bash scripts/ab_tiny.sh > gpurun_out/r4c_ab_tiny.log 2>&1
[ $? -eq 0 ] && timeout -k 10 300 python3 benchmarks/host_path.py > gpurun_out/r4c_host_path.jsonl 2> gpurun_out/r4c_host_path.err
