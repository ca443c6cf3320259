#!/bin/bash
# Round 3x: single-GPU hand-off v3 (raw hash dump + grid-wide scatter, per-lane
# records, auto level) and the one-rank packed adjacency of the partitioned
# engine: GPU tests, extras A/B (auto on/off), partitioned A/B (packed
# adjacency on / off), publish stamps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 600 $PT -m gpu tests/test_gpu_engine.py tests/test_gpu_dist_local.py > gpurun_out/r3x_pytest.log 2>&1 || exit $?
for rep in 1 2; do
  for a in 1 0; do
    BIBFS_AUTO_HANDOFF=$a $T 300 python3 bench.py --steps 20 --warmup 5 --extra-steps 200 --dist-graphs "" --batch 0 \
      --no-cpu-ref > gpurun_out/r3x_ab_auto${a}_$rep.json 2> gpurun_out/r3x_ab_auto${a}_$rep.err || exit $?
  done
done
for rep in 1 2; do
  for mb in 4096 0; do
    BIBFS_PADJ_MAX_MB=$mb $T 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1 --queries 48 \
      --reps 1 > gpurun_out/r3x_dist_padj${mb}_$rep.jsonl 2> gpurun_out/r3x_dist_padj${mb}_$rep.err || exit $?
  done
done
BIBFS_STAMP=1 $T 120 ./build/bin/bibfs_hip gnp:10000000::1 0 9999999 --verify --trace --repeat 3 > gpurun_out/r3x_stamp10m.log 2>&1 || exit $?
echo done
