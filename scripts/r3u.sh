#!/bin/bash
# Round 3u: device hand-off (grid_auto) -- resident/hand-off GPU tests, then an
# interleaved A/B of the extras (10M G(n,p), Kronecker 22) with the auto level
# on / off, then a kernel trace of resident 10M queries with it on.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 600 $PT -m gpu tests/test_gpu_engine.py -k "resident or handoff or tiny" > gpurun_out/r3u_pytest.log 2>&1 || exit $?
B="python3 bench.py --steps 20 --warmup 5 --extra-steps 200 --dist-graphs '' --batch 0 --no-cpu-ref"
for rep in 1 2; do
  for a in 1 0; do
    BIBFS_AUTO_HANDOFF=$a $T 300 python3 bench.py --steps 20 --warmup 5 --extra-steps 200 --dist-graphs "" --batch 0 \
      --no-cpu-ref > gpurun_out/r3u_ab_auto${a}_$rep.json 2> gpurun_out/r3u_ab_auto${a}_$rep.err || exit $?
  done
done
$T 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3u_tr_10m -- python3 bench.py --graph gnp:10000000::1 \
  --steps 40 --warmup 10 --extra-graph "" --dist-graphs "" --batch 0 --no-cpu-ref > gpurun_out/r3u_tr_10m.log 2>&1 || exit $?
echo done
