#!/bin/bash
# Cycle-level phase split of the single-workgroup search (BIBFS_STAMP builds
# the instrumented kernel variant): per round cycles by phase and election /
# init / loop / walk / publish totals.  The last run uses the resident
# server's profiling build (BIBFS_STAMP_SERVER): the same query with the graph
# warm in L2, as in the bench.  Run on the GPU box:
#   gpurun -- 'bash scripts/stamp.sh'
set -o pipefail
mkdir -p gpurun_out
B=./build/bin/bibfs_hip
BIBFS_STAMP=1 timeout -k 10 60 $B gnp:100000::6 0 99999 --verify --trace --repeat 5 > gpurun_out/stamp.log 2>&1 && \
BIBFS_STAMP=1 timeout -k 10 60 $B gnp:1000000::2 0 999999 --verify --trace --repeat 5 > gpurun_out/stamp1m.log 2>&1 && \
BIBFS_STAMP=1 BIBFS_STAMP_SERVER=1 timeout -k 10 60 $B gnp:100000::6 0 99999 --verify --trace --resident \
  --repeat 5 > gpurun_out/stamp_res.log 2>&1
