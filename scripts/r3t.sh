#!/bin/bash
# Round 3t: in-kernel phase stamps of the LDS engine on the 10M G(n,p) and
# Kronecker-22 extras (the graphs whose queries hand off to the grid).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B=./build/bin/bibfs_hip
BIBFS_STAMP=1 timeout -k 10 120 $B gnp:10000000::1 0 9999999 --verify --trace --repeat 3 > gpurun_out/r3t_stamp10m.log 2>&1 || exit $?
BIBFS_STAMP=1 timeout -k 10 120 $B gnp:10000000::1 12345 7654321 --verify --trace --repeat 3 > gpurun_out/r3t_stamp10m_b.log 2>&1 || exit $?
BIBFS_STAMP=1 timeout -k 10 120 $B kron:22:16:1 1 4000000 --verify --trace --repeat 3 > gpurun_out/r3t_stampk22.log 2>&1 || exit $?
echo done
