#!/bin/bash
# Round-4 session g: tiny server single-wave split A/B + stamps + tiny GPU tests.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 300 $PT -m gpu tests/test_gpu_engine.py -k "tiny" > gpurun_out/r4g_pytest.log 2>&1 && \
bash scripts/ab_tiny.sh > gpurun_out/r4g_ab_tiny.log 2>&1 && cp gpurun_out/ab_tiny.jsonl gpurun_out/r4g_ab_tiny.jsonl && \
BIBFS_STAMP=1 BIBFS_STAMP_SERVER=1 $T 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --verify --trace --resident --repeat 5 > gpurun_out/r4g_stamp_100k.txt 2>&1
