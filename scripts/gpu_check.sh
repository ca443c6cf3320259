#!/bin/bash
# GPU round check: selftest (engine vs oracle), stamped per-level latency,
# pytest -m gpu, bench.py.  Every GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
B=./build/bin
T="timeout -k 10"
$T 240 $B/bibfs_selftest gnp:1000::1 gnp:100000::6 gnp:1000000::2 rmat:65536:1048576:3 kron:16:16:2 \
    > gpurun_out/selftest.log 2>&1 && \
BIBFS_STAMP=1 $T 120 $B/bibfs_hip gnp:100000::6 0 99999 --verify --trace --repeat 20 > gpurun_out/stamp.log 2>&1 && \
$T 120 $B/bibfs_hip gnp:100000::6 0 99999 --json --repeat 200 > gpurun_out/lat.txt 2>&1 && \
$T 120 $B/bibfs_hip gnp:100000::6 0 99999 --json --repeat 200 --no-lockstep >> gpurun_out/lat.txt 2>&1 && \
$T 120 $B/bibfs_hip gnp:1000000::2 0 999999 --json --repeat 100 >> gpurun_out/lat.txt 2>&1 && \
$T 120 $B/bibfs_hip gnp:10000000::1 0 9999999 --json --repeat 50 >> gpurun_out/lat.txt 2>&1 && \
$T 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && \
$T 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
