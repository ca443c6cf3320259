#!/bin/bash
# Round-end style GPU check: the whole GPU suite, smoke(), the headline bench,
# a 2-rank replicated rehearsal on one GPU (gloo barriers) with a short
# secondary-config watchdog, and a kernel-trace profile of a short bench.
# Every GPU step has its own limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 900 $PT -m gpu tests > gpurun_out/pytest_gpu.log 2>&1 && \
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && \
$T 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
$T 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 200 --warmup 20 --dist-backend gloo --secondary-timeout 8 \
    > gpurun_out/bench_2rank.json 2> gpurun_out/bench_2rank.err && \
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -- \
    python3 bench.py --steps 200 --warmup 20 --batch 64 > gpurun_out/prof_bench.log 2>&1
