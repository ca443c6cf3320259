#!/bin/bash
# First GPU bring-up: correctness + latency of the single-GPU engine.
set -o pipefail
B=./build/bin/bibfs_hip
T="timeout -k 10 120"
$T $B gnp:1000::1 0 999 --verify --trace && \
$T $B gnp:100000::6 0 99999 --verify --repeat 20 && \
$T $B gnp:100000::6 0 99999 --json --repeat 50 && \
$T $B gnp:1000000::2 0 999999 --verify --json --repeat 50 && \
$T $B gnp:10000000::1 0 9999999 --verify --repeat 20 --trace && \
$T $B gnp:10000000::1 0 9999999 --json --repeat 50 && \
$T $B gnp:10000000::1 0 9999999 --json --repeat 20 --force-grid && \
$T $B gnp:100000::1 0 99999 --verify && \
$T $B rmat:1048576:16777216:1 0 1048575 --verify --trace --repeat 5 && \
$T $B rmat:1048576:16777216:1 0 1048575 --json --repeat 10 && \
$T $B kron:22:16:1 5 77777 --verify --trace --repeat 5 && \
$T $B kron:22:16:1 5 77777 --json --repeat 10
