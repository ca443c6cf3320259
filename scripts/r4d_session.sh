#!/bin/bash
# Round-4 session d: world-1 solo phase stamps and timings, round stamps at P = 2 / 4, bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 600 $PT -m gpu tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/r4d_pytest.log 2>&1 && \
BIBFS_DIST_STAMP=1 $T 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2 --modes 1 --queries 16 --reps 1 > gpurun_out/r4d_solo_stamps.jsonl 2> gpurun_out/r4d_solo_stamps.err && \
$T 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1 --queries 24 --reps 3 > gpurun_out/r4d_world1.jsonl 2> gpurun_out/r4d_world1.err && \
$T 600 python3 benchmarks/dist_rounds.py --specs gnp:1000000::2,kron:22 --ranks 2,4 --overlap 0 --queries 16 > gpurun_out/r4d_dist_rounds.jsonl 2> gpurun_out/r4d_dist_rounds.err && \
$T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err
