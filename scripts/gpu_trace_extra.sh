#!/bin/bash
# Kernel timelines of single queries on the secondary configs (one-shot
# kernels, so every query's LDS phase is its own dispatch), plus a roctx
# marker trace of a partitioned-engine query.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
P="timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv"
$P -d gpurun_out/tr_kron22 -- python3 bench.py --graph kron:22:16:1 --steps 40 --warmup 10 --extra-graph "" \
   --dist-graphs "" --batch 0 --no-cpu-ref --no-resident > gpurun_out/tr_kron22.log 2>&1 && \
$P -d gpurun_out/tr_10m -- python3 bench.py --graph gnp:10000000::1 --steps 40 --warmup 10 --extra-graph "" \
   --dist-graphs "" --batch 0 --no-cpu-ref --no-resident > gpurun_out/tr_10m.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d gpurun_out/tr_marker -- \
   python3 benchmarks/dist_ab.py --specs gnp:1000000::2 --modes 4 --queries 8 --reps 1 > gpurun_out/tr_marker.log 2>&1
