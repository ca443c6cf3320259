#!/bin/bash
# GPU round check: selftest (engine vs oracle), latency table, pytest -m gpu,
# bench.py.  Every GPU step has its own time limit; the chain stops at the
# first failure.
set -o pipefail
mkdir -p gpurun_out
B=./build/bin
T="timeout -k 10"
$T 300 $B/bibfs_selftest gnp:1000::1 gnp:100000::6 gnp:1000000::2 rmat:65536:1048576:3 kron:16:16:2 \
    > gpurun_out/selftest.log 2>&1 && \
: > gpurun_out/lat.txt && \
for g in "gnp:100000::6 0 99999" "gnp:1000000::2 0 999999" "gnp:10000000::1 0 9999999"; do
  $T 120 $B/bibfs_hip $g --json --repeat 200 >> gpurun_out/lat.txt 2>&1 && \
  $T 120 $B/bibfs_hip $g --json --repeat 200 --resident >> gpurun_out/lat.txt 2>&1 || exit 1
done && \
$T 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
$T 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
