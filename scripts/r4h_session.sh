#!/bin/bash
# Round-4 session h: tiny server all-wave split A/B + tiny stamps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 300 $PT -m gpu tests/test_gpu_engine.py -k "tiny or resident" > gpurun_out/r4h_pytest.log 2>&1 && \
bash scripts/ab_tiny.sh > gpurun_out/r4h_ab_tiny.log 2>&1 && cp gpurun_out/ab_tiny.jsonl gpurun_out/r4h_ab_tiny.jsonl && \
TAG=r4h bash scripts/gpu_tasks.sh stamp
