#!/bin/bash
# Round 3j: dist tests + solo stamps/A-B (r3i) + the kron:29 one-GPU rehearsal.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
./scripts/r3i.sh || exit $?
timeout -k 10 600 python3 -u benchmarks/big_rehearsal.py --spec kron:29:16:1 --pairs 8 \
  > gpurun_out/r3j_kron29.jsonl 2> gpurun_out/r3j_kron29.err || exit $?
echo done
