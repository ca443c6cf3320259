#!/bin/bash
# Round 3 (re-entry): everything one GPU call should bring back, most
# important first -- GPU suite, smoke, driver-style bench, then the A/Bs:
# device hand-off auto level on/off (extras), tiny-server 16-byte first-edge
# loads (build/var base vs x4), mailbox probe, VRAM request slot on/off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T="timeout -k 10"
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
# world-1 partitioned diagnosis: the two tests that failed (wrong parent chain at
# world 1), with the solo workgroup's self-cleanup on (default) / off, solo off
K="tiny_capacities_force_count_sync_and_overflow or native_rounds_follow_protocol_spec or world1"
for cfg in default selfclean0 solo0; do
  case $cfg in selfclean0) E="BIBFS_SOLO_SELFCLEAN=0";; solo0) E="BIBFS_DIST_SOLO=0";; *) E="BIBFS_NONE=1";; esac
  env $E $T 400 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dist_local.py -k "$K" > gpurun_out/ra_diag_$cfg.log 2>&1
  rc=$?; echo "diag $cfg rc=$rc"; [ $rc -le 1 ] || exit $rc
done
$T 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/ra_pytest.log 2>&1
rc=$?; echo "suite rc=$rc"; [ $rc -le 1 ] || exit $rc
$T 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ra_smoke.log 2>&1 || exit $?
$T 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ra_bench.json 2> gpurun_out/ra_bench.err || exit $?
for a in 1 0; do
  BIBFS_AUTO_HANDOFF=$a $T 120 python3 bench.py --steps 20 --warmup 5 --extra-steps 200 --dist-graphs "" --batch 0 \
    --no-cpu-ref > gpurun_out/ra_ab_auto${a}.json 2> gpurun_out/ra_ab_auto${a}.err || exit $?
done
out=gpurun_out/ra_tiny_x4_ab.jsonl
: > $out
for rep in 1 2; do
  for v in base x4; do
    LD_LIBRARY_PATH=build/var/$v $T 90 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/ra_one.jsonl 2> gpurun_out/ra_one_$v.err || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/ra_one.jsonl').readline()); d['variant']='$v'; print(json.dumps(d))" >> $out
  done
done
$T 60 ./build/bin/mailbox_rtt > gpurun_out/ra_mailbox_rtt.txt 2>&1 || exit $?
for v in 0 1; do
  BIBFS_VRAM_MAILBOX=$v $T 90 python3 benchmarks/tiny_latency.py --reps 30 > gpurun_out/ra_tiny_vram${v}.jsonl 2> gpurun_out/ra_tiny_vram${v}.err || exit $?
done
# the world-1 packed adjacency (off by default since the suite failure): does it reproduce?
BIBFS_PADJ_MAX_MB=4096 $T 300 $PT -m gpu tests/test_gpu_dist_local.py -k "tiny_capacities or speculative or local_group_matches" > gpurun_out/ra_padj_on.log 2>&1
echo "padj-on pytest status $?"
echo done
