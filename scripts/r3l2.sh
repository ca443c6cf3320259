#!/bin/bash
# Round 3l2: device-gated first level only on hub-free graphs (max degree <= 64):
# single-GPU engine GPU tests, then the driver-style bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/rl_pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -eq 0 ] || exit $rc
$T 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rl_smoke.log 2>&1 || exit $?
$T 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rl_bench.json 2> gpurun_out/rl_bench.err || exit $?
echo done
