#!/bin/bash
# Round 3y: re-verify HEAD after the container was re-created: whole GPU
# suite, smoke, driver-style bench, kernel stats of the bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 900 $PT -m gpu tests > gpurun_out/r3y_pytest.log 2>&1 || exit $?
$T 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3y_smoke.log 2>&1 || exit $?
$T 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3y_bench.json 2> gpurun_out/r3y_bench.err || exit $?
$T 60 ./build/bin/mailbox_rtt > gpurun_out/r3y_mailbox_rtt.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in 0 1; do
    BIBFS_VRAM_MAILBOX=$v BIBFS_DEBUG= $T 120 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/r3y_tiny_vram${v}_$rep.jsonl 2> gpurun_out/r3y_tiny_vram${v}_$rep.err || exit $?
  done
done
echo done
