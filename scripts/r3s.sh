#!/bin/bash
# Round 3s: HEAD check after the container re-creation -- GPU suite, smoke, driver-style bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
$T 900 $PT -m gpu tests > gpurun_out/r3s_pytest_gpu.log 2>&1 || exit $?
$T 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3s_smoke.log 2>&1 || exit $?
$T 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err || exit $?
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P -d gpurun_out/r3s_tr_kron22 -- python3 bench.py --graph kron:22:16:1 --steps 40 --warmup 10 --extra-graph "" \
   --dist-graphs "" --batch 0 --no-cpu-ref --no-resident > gpurun_out/r3s_tr_kron22.log 2>&1 || exit $?
$P -d gpurun_out/r3s_tr_10m -- python3 bench.py --graph gnp:10000000::1 --steps 40 --warmup 10 --extra-graph "" \
   --dist-graphs "" --batch 0 --no-cpu-ref --no-resident > gpurun_out/r3s_tr_10m.log 2>&1 || exit $?
echo done
