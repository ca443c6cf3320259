#!/bin/bash
# Round-end style GPU check: the whole GPU suite, smoke(), the headline bench
# (with the partitioned block at N = 1), the partitioned-engine A/B and a
# kernel-trace profile of a short bench.  Every GPU step has its own limit;
# the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 900 $PT -m gpu tests > gpurun_out/pytest_gpu.log 2>&1 && \
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && \
$T 500 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
$T 400 python benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22,kron:27 --modes 0,1,2,4 --queries 16 --reps 2 \
    > gpurun_out/dist_ab.jsonl 2> gpurun_out/dist_ab.err && \
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -- \
    python3 bench.py --steps 200 --warmup 20 --batch 64 --dist-graphs "" > gpurun_out/prof_bench.log 2>&1
