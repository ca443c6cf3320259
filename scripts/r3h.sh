#!/bin/bash
# Round 3h: the solo workgroup's degree scan as conflict-free 64-entry DPP
# steps (was 32 fixed lane-blocked steps) -- world-1 / local-group tests, the
# solo phase stamps on G(1M), and the world-1 A/B against the last bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
$T 500 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dist_local.py tests/test_gpu_dist_and_tools.py > gpurun_out/rh_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
BIBFS_DIST_STAMP=1 $T 120 python3 benchmarks/dist_ab.py --specs gnp:1000000::2 --modes 1 --queries 24 --reps 1 > gpurun_out/rh_stamps.jsonl 2> gpurun_out/rh_stamps.err || exit $?
for rep in 1 2; do
  $T 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1 --queries 48 --reps 1 > gpurun_out/rh_dist_$rep.jsonl 2> gpurun_out/rh_dist_$rep.err || exit $?
done
echo done
