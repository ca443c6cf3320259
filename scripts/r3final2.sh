#!/bin/bash
# Round 3, last HEAD check: whole GPU suite, smoke, driver-style bench, and
# the bench's per-kernel stats as CSV.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/rz_pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -le 1 ] || exit $rc
$T 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rz_smoke.log 2>&1 || exit $?
$T 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rz_bench.json 2> gpurun_out/rz_bench.err || exit $?
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rz_prof -o rz -- python3 bench.py --steps 20 --warmup 5 --extra-steps 50 --batch 0 --no-cpu-ref > gpurun_out/rz_prof_bench.json 2> gpurun_out/rz_prof_bench.err || exit $?
echo done
