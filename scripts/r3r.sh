#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BIBFS_TINY_STAMP=1 timeout -k 10 120 ./build/bin/bibfs_hip gnp:100000::6 0 99999 --resident --repeat 4 > gpurun_out/r3r_stamp.txt 2>&1 || exit $?
timeout -k 10 300 python3 benchmarks/tiny_latency.py --pairs 64 --reps 30 > gpurun_out/r3r_lat.jsonl 2> gpurun_out/r3r_lat.err || exit $?
timeout -k 10 300 python3 benchmarks/tiny_latency.py --pairs 64 --reps 30 >> gpurun_out/r3r_lat.jsonl 2>> gpurun_out/r3r_lat.err || exit $?
echo done
