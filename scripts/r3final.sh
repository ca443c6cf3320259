#!/bin/bash
# Round 3 (re-entry): HEAD with the solo self-cleanup barrier and the x4
# tiny-server default -- the world-1 tests that failed (twice), the whole GPU
# suite, smoke, the driver-style bench, and a rocprofv3 kernel-stats run of it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
K="tiny_capacities_force_count_sync_and_overflow or native_rounds_follow_protocol_spec or world1"
for rep in 1 2; do
  $T 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dist_local.py -k "$K" > gpurun_out/rf_diag_$rep.log 2>&1
  rc=$?; echo "diag $rep rc=$rc"; [ $rc -le 1 ] || exit $rc
done
$T 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/rf_pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -le 1 ] || exit $rc
$T 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rf_smoke.log 2>&1 || exit $?
$T 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rf_bench.json 2> gpurun_out/rf_bench.err || exit $?
$T 300 rocprofv3 --kernel-trace --stats -d gpurun_out/rf_prof -o rf -- python3 bench.py --steps 20 --warmup 5 --extra-steps 50 --batch 0 --no-cpu-ref > gpurun_out/rf_prof_bench.json 2> gpurun_out/rf_prof_bench.err || exit $?
echo done
