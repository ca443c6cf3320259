#!/bin/bash
# Round 3g: world-1 packed adjacency of the partitioned engine (16 B per edge:
# the neighbour's row comes with its id) on / off, now that the world-1
# failure is traced to the solo self-cleanup race: correctness on the world-1
# tests with it on, then an interleaved A/B on G(1M) and Kronecker 22.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
K="tiny_capacities_force_count_sync_and_overflow or native_rounds_follow_protocol_spec or world1 or local_group"
BIBFS_PADJ_MAX_MB=4096 $T 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dist_local.py -k "$K" > gpurun_out/rg_padj_tests.log 2>&1
rc=$?; echo "padj tests rc=$rc"; [ $rc -le 1 ] || exit $rc
for rep in 1 2; do
  for mb in 4096 0; do
    BIBFS_PADJ_MAX_MB=$mb $T 300 python3 benchmarks/dist_ab.py --specs gnp:1000000::2,kron:22 --modes 1 --queries 48 \
      --reps 1 > gpurun_out/rg_dist_padj${mb}_$rep.jsonl 2> gpurun_out/rg_dist_padj${mb}_$rep.err || exit $?
  done
done
echo done
