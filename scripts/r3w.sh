#!/bin/bash
# Round 3w: hand-off v3 (hash tables dumped raw, scattered grid-wide by
# k_handoff; one-store-per-lane hand-off/result records) -- engine GPU tests,
# interleaved A/B of the extras with the auto level on / off, publish stamps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 600 $PT -m gpu tests/test_gpu_engine.py > gpurun_out/r3w_pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for a in 1 0; do
    BIBFS_AUTO_HANDOFF=$a $T 300 python3 bench.py --steps 20 --warmup 5 --extra-steps 200 --dist-graphs "" --batch 0 \
      --no-cpu-ref > gpurun_out/r3w_ab_auto${a}_$rep.json 2> gpurun_out/r3w_ab_auto${a}_$rep.err || exit $?
  done
done
BIBFS_STAMP=1 $T 120 ./build/bin/bibfs_hip gnp:10000000::1 0 9999999 --verify --trace --repeat 3 > gpurun_out/r3w_stamp10m.log 2>&1 || exit $?
echo done
