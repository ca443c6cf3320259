#!/bin/bash
# Latency table (one-shot and resident) for the 100k / 1M / 10M G(n,p) queries.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/lat.txt
for g in "gnp:100000::6 0 99999" "gnp:1000000::2 0 999999" "gnp:10000000::1 0 9999999"; do
  timeout -k 10 120 ./build/bin/bibfs_hip $g --json --repeat 200 >> gpurun_out/lat.txt 2>&1 && \
  timeout -k 10 120 ./build/bin/bibfs_hip $g --json --repeat 200 --resident >> gpurun_out/lat.txt 2>&1 || exit 1
done
