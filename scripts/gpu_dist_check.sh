#!/bin/bash
# GPU check of the partitioned engine (local group, P = 2..4 ranks on one GPU),
# then the whole GPU suite and the headline bench.  Each GPU step has its own
# limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 400 $PT tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/pytest_dist.log 2>&1 && \
$T 900 $PT -m gpu tests > gpurun_out/pytest_gpu.log 2>&1 && \
$T 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
