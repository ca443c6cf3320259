#!/bin/bash
# Round 3o: the driver's default bench, twice (variance of the partitioned entries).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3o_bench1.json 2> gpurun_out/r3o_bench1.err || exit $?
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --batch 0 > gpurun_out/r3o_bench2.json 2> gpurun_out/r3o_bench2.err || exit $?
echo done
