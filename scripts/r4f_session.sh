#!/bin/bash
# Round-4 session f: whole GPU suite, smoke, bench (world-1 single-engine path + rounds engine side by side).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 900 $PT -m gpu tests > gpurun_out/r4f_pytest.log 2>&1 && \
$T 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 && \
$T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err
