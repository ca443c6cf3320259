#!/bin/bash
# Round 3m2: per-kernel stats of a bench run on the final HEAD.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rm_prof -o rm -- python3 bench.py --steps 20 --warmup 5 --extra-steps 50 --batch 0 --no-cpu-ref > gpurun_out/rm_prof_bench.json 2> gpurun_out/rm_prof_bench.err || exit $?
echo done
