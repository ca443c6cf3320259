#!/bin/bash
# Round 3m: full GPU test suite + driver-style bench + kernel stats of the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r3m_gpu_tests.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3m_bench.json 2> gpurun_out/r3m_bench.err || exit $?
echo done
