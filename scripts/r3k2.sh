#!/bin/bash
# Round 3k2: device-gated first grid level on / off, bench extras (10M G(n,p),
# Kronecker 22), 200 queries each, interleaved, twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
for rep in 1 2; do
  for a in 1 0; do
    BIBFS_AUTO_HANDOFF=$a $T 150 python3 bench.py --steps 20 --warmup 5 --extra-steps 200 --dist-graphs "" --batch 0 \
      --no-cpu-ref > gpurun_out/rk_auto${a}_$rep.json 2> gpurun_out/rk_auto${a}_$rep.err || exit $?
  done
done
echo done
