#!/bin/bash
# Cycle-level phase split of the single-workgroup search (BIBFS_STAMP builds
# the instrumented kernel variant): per round rec+col / claim / append cycles
# and election / init / loop / walk / publish totals.  Run on the GPU box:
#   scripts/gpu.sh 300 'bash scripts/stamp.sh'
set -o pipefail
mkdir -p gpurun_out
B=./build/bin/bibfs_hip
BIBFS_STAMP=1 timeout -k 10 60 $B gnp:100000::6 0 99999 --verify --trace --repeat 5 > gpurun_out/stamp.log 2>&1 && \
BIBFS_STAMP=1 timeout -k 10 60 $B gnp:1000000::2 0 999999 --verify --trace --repeat 5 > gpurun_out/stamp1m.log 2>&1
