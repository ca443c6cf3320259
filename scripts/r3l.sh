#!/bin/bash
# Round 3l: kernel timelines of the single-GPU engine's grid hand-off (10M G(n,p), Kronecker 22).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3l_prof_10m -o run -- \
  python3 benchmarks/pair_latency.py --graph gnp:10000000::1 --pairs 16 --reps 5 \
  > gpurun_out/r3l_10m.jsonl 2> gpurun_out/r3l_10m.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3l_prof_k22 -o run -- \
  python3 benchmarks/pair_latency.py --graph kron:22:16:1 --pairs 16 --reps 5 \
  > gpurun_out/r3l_k22.jsonl 2> gpurun_out/r3l_k22.err || exit $?
echo done
