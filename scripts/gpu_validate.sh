#!/bin/bash
# Full validation of the tree on one GPU box: the GPU suite, the driver-style
# 1-GPU bench, and the bench's N > 1 contract rehearsed with 2 ranks sharing
# the GPU (gloo + the IPC transport).  Stops at the first failing step.
#   gpurun --timeout 1200 -- 'TAG=r5v bash scripts/gpu_validate.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG="${TAG:-r5v}"
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/${TAG}_pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || exit 1
timeout -k 10 600 python3 bench.py --gpus 2 --steps 10 --warmup 3 > $O/${TAG}_bench_2rank.json 2> $O/${TAG}_bench_2rank.err || exit 1
