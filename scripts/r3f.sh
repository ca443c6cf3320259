#!/bin/bash
# Round 3f: mailbox placement micro + kernel trace of the partitioned engine at world 1.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 ./build/bin/mailbox_rtt > gpurun_out/r3f_mailbox.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f_prof_dist -o run -- \
  python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 4 --queries 16 --reps 1 \
  > gpurun_out/r3f_dist.jsonl 2> gpurun_out/r3f_dist.err || exit $?
echo done
